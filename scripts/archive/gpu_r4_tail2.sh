#!/bin/bash
# Round 4: the tail sweep went 0 / 48 / 96 and still rose at 96 - past it, config 4 (312 parts
# of 64 MiB) alternating tails 96 / 144 / 192, 3 rounds of 3 reps, to find where host hashing
# of the last parts stops paying.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_tail2}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
for r in 1 2 3; do
  for t in 96 144 192; do
    n=c4_t${t}_$r
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 4 --reps 3 --stream-verify auto --stream-gpu-tail $t > $F/$n.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
    python -c "
import json; j=json.loads(open('$F/$n.json').read().strip().splitlines()[-1])
print('$n', j['MBps_reps'], [r['worker_cpu_s'] for r in j['reps_detail']], j['part_pool_peak_MiB'], j['torrent'].get('gpu_parts'))"
  done
done
