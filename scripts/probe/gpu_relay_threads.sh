#!/bin/bash
# Probe: where the worker's CPU goes in config 4 with piece SHA-1 on the host vs on the GPU
# (per-thread CPU deltas over the reps, buffer / registration counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/probe_relay_threads}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD} STAGER_THREAD_CPU=1
for v in cpu gpu; do
  timeout -k 10 300 python -m downloader_amd.bench.configs --config 4 --reps 3 --stream-verify $v --stream-gpu-pending 160 > $F/c4_$v.json 2>> $F/err.txt || exit 1
  python -c "
import json; j=json.loads(open('$F/c4_$v.json').read().strip().splitlines()[-1])
print('$v', j['MBps_reps'], 'worker', j['worker_cpu_s'], 'pool', j['relay_pool_after'])
print('  gpu', {k: v for k, v in (j.get('gpu_relay') or {}).items()})
for r in j['thread_cpu'][:10]: print('  ', r)"
done
