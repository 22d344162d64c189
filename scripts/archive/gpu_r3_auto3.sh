#!/bin/bash
# Round-3: the final stream-verification default (auto, tail 96) on the box: GPU tier, smoke,
# then configs 4 and 3 in default settings next to forced host hashing, and config 4 with two
# jobs at once.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_auto3}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || exit 1
tail -1 $F/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || exit 1
tail -1 $F/smoke.txt
run() {   # name, config, jobs, extra args
  timeout -k 10 400 python -m downloader_amd.bench.configs --config $2 --reps 4 --torrent-jobs $3 ${@:4} > $F/$1.json 2>> $F/err.txt || exit 1
  python -c "
import json; j=json.loads(open('$F/$1.json').read().strip().splitlines()[-1])
print('$1', j['MBps_reps'], 'worker', [r['worker_cpu_s'] for r in j['reps_detail']], 'gpu_parts', j['torrent'].get('gpu_parts'), j['torrent'].get('verify'))"
}
run c4_default 4 1
run c4_cpu 4 1 --stream-verify cpu
run c3_default 3 1
run c3_cpu 3 1 --stream-verify cpu
run c4_j2_default 4 2
run c4_j2_cpu 4 2 --stream-verify cpu
