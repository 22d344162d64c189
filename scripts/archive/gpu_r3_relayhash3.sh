#!/bin/bash
# Round-3: GPU relay hashing with fewer parts awaiting digests (stream_gpu_pending 32 / 64)
# now that the part-buffer pool keeps what the jobs have out; config 4, 1 and 2 jobs at once.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_relayhash3}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD} STAGER_THREAD_CPU=1
for PEND in 32 64; do
for jobs in 1 2; do
  for v in gpu; do
    timeout -k 10 400 python -m downloader_amd.bench.configs --config 4 --reps 4 --torrent-jobs $jobs --stream-verify $v --stream-gpu-pending $PEND > $F/c4_j${jobs}_${v}_p$PEND.json 2>> $F/err.txt || exit 1
    python -c "
import json; j=json.loads(open('$F/c4_j${jobs}_${v}_p$PEND.json').read().strip().splitlines()[-1])
print('pend $PEND jobs $jobs $v', j['MBps_reps'], 'worker', [r['worker_cpu_s'] for r in j['reps_detail']], 'created', j['relay_pool_after'].get('created'))"
  done
done
done
