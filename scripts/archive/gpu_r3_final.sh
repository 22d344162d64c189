#!/bin/bash
# Round-3 closing validation of the tree: GPU tier, smoke, the driver's default bench twice,
# config 4 (one and two 20 GB jobs, GPU relay hashing in auto) and config 3, then the config 7
# chaos soak (worker SIGKILLs, AMQP drops, S3 503s; torrents staged as multipart so kills
# leave uploads open for the sweep) - the paths that cancel transfers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_final}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || exit 1
tail -1 $F/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || exit 1
tail -1 $F/smoke.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py > $F/bench_$i.json 2>> $F/bench.err || exit 1
  python -c "import json;j=json.load(open('$F/bench_$i.json'));print('bench', j['value'], j['single_put_MBps'], j['crc_relay_MBps'], j['sink_mismatches'])"
done
run() {   # name, config, jobs, extra args
  timeout -k 10 400 python -m downloader_amd.bench.configs --config $2 --reps 3 --torrent-jobs $3 ${@:4} > $F/$1.json 2>> $F/err.txt || exit 1
  python -c "
import json; j=json.loads(open('$F/$1.json').read().strip().splitlines()[-1])
print('$1', j['MBps_reps'], 'worker', [r['worker_cpu_s'] for r in j['reps_detail']], 'gpu_parts', j['torrent'].get('gpu_parts'), j['torrent'].get('verify'))"
}
run c4 4 1
run c4_j2 4 2
run c3 3 1
timeout -k 10 600 python -m downloader_amd.bench.configs --config 7 --scale 2 --workers 4 --concurrency 4 --qps 40 --chaos-interval 1.0 --s3-fail-rate 0.03 --chaos-timeout 400 --chaos-multipart-mb 16 > $F/chaos.jsonl 2> $F/chaos.err || exit 1
tail -1 $F/chaos.jsonl
