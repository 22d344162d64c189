#!/bin/bash
# Round-3: GPU relay hashing tail sweep, second pass: config 4 one job at tail 96 / 128 / 160
# and two jobs at tail 96, config 3 at tail 96, each next to host hashing in the same call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_tail2}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
run() {   # name, config, jobs, verify args
  timeout -k 10 400 python -m downloader_amd.bench.configs --config $2 --reps 4 --torrent-jobs $3 ${@:4} > $F/$1.json 2>> $F/err.txt || exit 1
  python -c "
import json; j=json.loads(open('$F/$1.json').read().strip().splitlines()[-1])
print('$1', j['MBps_reps'], 'worker', [r['worker_cpu_s'] for r in j['reps_detail']], 'gpu_parts', j['torrent'].get('gpu_parts'))"
}
run c4_j1_cpu 4 1 --stream-verify cpu
run c4_j1_t96 4 1 --stream-verify gpu --stream-gpu-tail 96
run c4_j1_t128 4 1 --stream-verify gpu --stream-gpu-tail 128
run c4_j1_t160 4 1 --stream-verify gpu --stream-gpu-tail 160
run c4_j2_cpu 4 2 --stream-verify cpu
run c4_j2_t96 4 2 --stream-verify gpu --stream-gpu-tail 96
run c3_j1_cpu 3 1 --stream-verify cpu
run c3_j1_t96 3 1 --stream-verify gpu --stream-gpu-tail 96
