#!/bin/bash
# Round-4 closing validation of the tree, one box: GPU tier, smoke, the driver's bench line x3
# (headline + one PUT + CRC'd relay), headline vs reference mode, configs 1/3/4/5 tuned (3/4
# x3 reps) and in reference mode, config 4 with two jobs under a 2 GiB budget, TLS config 2,
# gfx950 kernel, and the chaos soak (worker SIGKILLs, AMQP drops, S3 503s).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_final}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
PART=${PART:-abc}
if [[ $PART == *a* ]]; then
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || { tail -20 $F/smoke.txt; exit 1; }
for i in 1 2 3; do
  step bench$i; timeout -k 10 300 python bench.py > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python -c "import json;j=json.load(open('$F/bench_$i.json'));print('bench', j['value'], j['p50_job_latency_s'], j['integrity'], 'one PUT', j['single_put_MBps'], 'crc', j['crc_relay_MBps'], j['sink_mismatches'])"
done
step ref; timeout -k 10 600 python bench.py --compare-reference --no-compare-single-put --no-compare-crc > $F/bench_vs_reference.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
python -c "import json;j=json.load(open('$F/bench_vs_reference.json'));print('vs reference', j['value'], j['reference_mode_MBps'], j['vs_reference_mode'])"
step configs; timeout -k 10 600 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 --reps 3 > $F/configs_tuned.jsonl 2> $F/configs.err || { tail -20 $F/configs.err; exit 1; }
fi
if [[ $PART == *b* ]]; then
step configs_ref; timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 --mode reference > $F/configs_ref.jsonl 2>> $F/configs.err || { tail -20 $F/configs.err; exit 1; }
fi
if [[ $PART == *a* ]]; then
step c4j2; timeout -k 10 400 python -m downloader_amd.bench.configs --config 4 --reps 3 --torrent-jobs 2 --relay-memory-mb 2048 > $F/c4_j2_2g.json 2>> $F/configs.err || { tail -20 $F/configs.err; exit 1; }
step tls; timeout -k 10 300 python bench.py --tls native --no-compare-single-put --no-compare-crc > $F/bench_tls_native.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
step kernel; timeout -k 10 300 python -u -m downloader_amd.bench.verify_bench --kernel-only > $F/kernel.jsonl 2> $F/kernel.err || { tail -20 $F/kernel.err; exit 1; }
fi
if [[ $PART == *b* ]]; then
step chaos; timeout -k 10 600 python -m downloader_amd.bench.configs --config 7 --scale 2 --workers 4 --concurrency 4 --qps 40 --chaos-interval 1.0 --s3-fail-rate 0.03 --chaos-timeout 400 --chaos-multipart-mb 16 > $F/chaos.jsonl 2> $F/chaos.err || { tail -20 $F/chaos.err; exit 1; }
tail -1 $F/chaos.jsonl
fi
if [[ $PART == *c* ]]; then
# PMC pass (its own run, counters only): the PartHasher's sha1_lanes in the relay context -
# config 4, one job, GPU hashing, 2 GiB budget; 5 SQ + 1 GRBM counters fit one pass
R=$PWD
step pmc; ( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$F/pmc -o pmc -- python3 -m downloader_amd.bench.configs --config 4 --reps 1 --stream-verify gpu --relay-memory-mb 2048 > $R/$F/pmc_c4.json 2> $R/$F/pmc.err ) || { tail -20 $F/pmc.err; exit 1; }
P=$(find $F/pmc -name '*counter_collection.csv' | head -1)
[ -n "$P" ] && python -m downloader_amd.bench.pmc_summary "$P" 4194304 > $F/pmc_summary.json && cat $F/pmc_summary.json
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
if os.path.exists("$F/c4_j2_2g.json"):
    j = json.loads(open("$F/c4_j2_2g.json").read().strip().splitlines()[-1])
    print("c4 two jobs 2 GiB", j["MBps_reps"], j["part_pool_peak_MiB"], j["worker_rss_peak_MB"], j["torrent"].get("gpu_parts"))
    print("tls", json.load(open("$F/bench_tls_native.json"))["value"])
PY
