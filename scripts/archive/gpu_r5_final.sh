#!/bin/bash
# Round-5 closing validation of the tree, one box. Part a: GPU tier, smoke, the driver's bench
# line x2 (headline + one PUT + CRC'd relay + torrent A/B), headline vs reference mode,
# configs 1/3/4/5 tuned (3/4 x3 reps), config 6 as the whole magnet job. Part b: configs
# 1/3/4/5 in reference mode and the chaos soak (worker SIGKILLs, AMQP drops, S3 503s).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_final}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
PART=${PART:-ab}
if [[ $PART == *a* ]]; then
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || { tail -20 $F/smoke.txt; exit 1; }
for i in 1 2; do
  step bench$i; timeout -k 10 400 python bench.py > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python -c "import json;j=json.load(open('$F/bench_$i.json'));print('bench', j['value'], j['p50_job_latency_s'], j['integrity'], 'one PUT', j['single_put_MBps'], 'crc', j['crc_relay_MBps'], j['sink_mismatches'], 'torrent', j.get('torrent_gpu_MBps'), j.get('torrent_host_MBps'), j.get('torrent_error'))"
done
step ref; timeout -k 10 600 python bench.py --compare-reference --no-compare-single-put --no-compare-crc --torrent-gb 0 > $F/bench_vs_reference.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
python -c "import json;j=json.load(open('$F/bench_vs_reference.json'));print('vs reference', j['value'], j['reference_mode_MBps'], j['vs_reference_mode'])"
step configs; timeout -k 10 600 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 --reps 3 > $F/configs_tuned.jsonl 2> $F/configs.err || { tail -20 $F/configs.err; exit 1; }
step swarmjob; timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --swarm-job --reps 3 > $F/swarm_job.json 2>> $F/configs.err || { tail -20 $F/configs.err; exit 1; }
fi
if [[ $PART == *b* ]]; then
step configs_ref; timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 --mode reference > $F/configs_ref.jsonl 2>> $F/configs.err || { tail -20 $F/configs.err; exit 1; }
step chaos; timeout -k 10 600 python -m downloader_amd.bench.configs --config 7 --scale 2 --workers 4 --concurrency 4 --qps 40 --chaos-interval 1.0 --s3-fail-rate 0.03 --chaos-timeout 400 --chaos-multipart-mb 16 > $F/chaos.jsonl 2> $F/chaos.err || { tail -20 $F/chaos.err; exit 1; }
tail -1 $F/chaos.jsonl | cut -c1-600
fi
python3 - <<PY
import json
import os
for f in ("configs_tuned", "configs_ref"):
    if not os.path.exists("$F/" + f + ".jsonl"):
        continue
    for l in open("$F/" + f + ".jsonl"):
        j = json.loads(l)
        print(f, {k: j.get(k) for k in ("config", "mode", "MBps", "MBps_reps", "p50_latency_s", "p50_s", "worker_rss_peak_MB", "part_pool_peak_MiB")})
if os.path.exists("$F/swarm_job.json"):
    j = json.loads(open("$F/swarm_job.json").read().strip().splitlines()[-1])
    print("swarm job", j["MBps_reps"], j["worker_cpu_s_per_GB_reps"], j["s3_bytes_received"])
PY
