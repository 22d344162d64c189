#!/bin/bash
# Round 4: with copies on their own hardware queues (2 copy + 2 compute streams), re-decide
# how many of a job's last parts hash on the host (download.stream_gpu_tail, 96 since round
# 3) - config 4, alternating tails 0 / 48 / 96, 3 rounds of 3 reps - and whether config 3
# (4 GB, 64 parts: all inside the 96-part tail today) gains from the device.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_tail}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
show() { python -c "
import json; j=json.loads(open('$F/$1.json').read().strip().splitlines()[-1])
print('$1', j['MBps_reps'], [r['worker_cpu_s'] for r in j['reps_detail']], j['part_pool_peak_MiB'], j['torrent'].get('gpu_parts'))"; }
for r in 1 2 3; do
  for t in 0 48 96; do
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 4 --reps 3 --stream-verify auto --stream-gpu-tail $t > $F/c4_t${t}_$r.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
    show c4_t${t}_$r
  done
done
for r in 1 2 3; do
  for m in "cpu --stream-verify cpu" "gpu0 --stream-verify gpu --stream-gpu-tail 0" "gpu16 --stream-verify gpu --stream-gpu-tail 16"; do
    set -- $m; n=$1; shift
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 3 --reps 3 "$@" > $F/c3_${n}_$r.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
    show c3_${n}_$r
  done
done
