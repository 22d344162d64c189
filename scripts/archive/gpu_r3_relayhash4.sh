#!/bin/bash
# Round-3: GPU relay hashing with one process-wide budget of parts awaiting digests (160,
# shared by every stream job) vs host hashing; config 4 with 1 and 2 jobs at once, 4 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_relayhash4}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD} STAGER_THREAD_CPU=1
for jobs in 1 2; do
  for v in cpu gpu; do
    timeout -k 10 400 python -m downloader_amd.bench.configs --config 4 --reps 4 --torrent-jobs $jobs --stream-verify $v > $F/c4_j${jobs}_$v.json 2>> $F/err.txt || exit 1
    python -c "
import json; j=json.loads(open('$F/c4_j${jobs}_$v.json').read().strip().splitlines()[-1])
print('jobs $jobs $v', j['MBps_reps'], 'worker', [r['worker_cpu_s'] for r in j['reps_detail']], 'created', j['relay_pool_after'].get('created'))"
  done
done
