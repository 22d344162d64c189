#!/bin/bash
# Round-3: stream_verify_backend auto (the new default) on the box: GPU tier, smoke, and
# config 4 with one and two jobs at once in auto mode next to forced host hashing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_auto}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || exit 1
tail -1 $F/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || exit 1
tail -1 $F/smoke.txt
for jobs in 2 1; do
  for v in auto cpu; do
    timeout -k 10 400 python -m downloader_amd.bench.configs --config 4 --reps 4 --torrent-jobs $jobs --stream-verify $v > $F/c4_j${jobs}_$v.json 2>> $F/err.txt || exit 1
    python -c "
import json; j=json.loads(open('$F/c4_j${jobs}_$v.json').read().strip().splitlines()[-1])
print('jobs $jobs $v', j['MBps_reps'], 'worker', [r['worker_cpu_s'] for r in j['reps_detail']], 'gpu_parts', j['torrent'].get('gpu_parts'), j['torrent'].get('verify'))"
  done
done
