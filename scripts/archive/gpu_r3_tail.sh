#!/bin/bash
# Round-3: one config-4 job with GPU relay hashing at stream_gpu_tail 16 / 48 / 96 (the job's
# last N queued parts hash on the host) vs host hashing, same call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_tail}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
for t in 16 48 96 cpu; do
  if [ $t = cpu ]; then a="--stream-verify cpu"; else a="--stream-verify gpu --stream-gpu-tail $t"; fi
  timeout -k 10 400 python -m downloader_amd.bench.configs --config 4 --reps 4 $a > $F/c4_$t.json 2>> $F/err.txt || exit 1
  python -c "
import json; j=json.loads(open('$F/c4_$t.json').read().strip().splitlines()[-1])
print('$t', j['MBps_reps'], 'worker', [r['worker_cpu_s'] for r in j['reps_detail']], 'gpu_parts', j['torrent'].get('gpu_parts'))"
done
