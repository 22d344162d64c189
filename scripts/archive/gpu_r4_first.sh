#!/bin/bash
# Round-4 first call: GPU tier (incl. the eventfd completion path and the part budget on the
# device), smoke, the driver's bench line, then config 4 (one 20 GB job) at the default and a
# 2 GiB part budget, GPU relay hashing (auto) vs host.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_first}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
cat /sys/fs/cgroup/memory.max > $F/memory_max.txt 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || { tail -20 $F/smoke.txt; exit 1; }
tail -1 $F/smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench.json 2> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
cat $F/bench.json
run() {   # name, args
  timeout -k 10 400 python -m downloader_amd.bench.configs --config 4 --reps 3 ${@:2} > $F/$1.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
  python -c "
import json; j=json.loads(open('$F/$1.json').read().strip().splitlines()[-1])
print('$1', j['MBps_reps'], 'worker', [r['worker_cpu_s'] for r in j['reps_detail']], 'rss_peak', j['worker_rss_peak_MB'], 'budget', j['part_budget_MiB'], 'pool_peak', j['part_pool_peak_MiB'], 'gpu_parts', j['torrent'].get('gpu_parts'))"
}
run c4_auto --stream-verify auto
run c4_cpu --stream-verify cpu
run c4_auto_2g --stream-verify auto --relay-memory-mb 2048
run c4_cpu_2g --stream-verify cpu --relay-memory-mb 2048
