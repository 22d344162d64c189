#!/bin/bash
# Round 5, fourth swarm call: config 6 at 2, 4 and 8 GB with pieces SHA-1'd on the host
# (--swarm-verify cpu) vs on the gfx950 PartHasher (--swarm-verify gpu; the download.swarm_gpu_inflight / swarm_pool_mb defaults)
# to place download.swarm_gpu_min_gb
# (where `auto` switches to the device). 2 alternating rounds, 3 downloads per process.
# SCALES="4 8": other sizes (x GB of 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_swarm14}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
df -h /tmp | tail -1
for sc in ${SCALES:-1 2 4}; do
  for i in 1 2; do
    for v in cpu gpu; do
      step "$v x$sc $i"
      timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --reps 3 --scale $sc --swarm-verify $v > $F/swarm_${v}_x${sc}_$i.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
      python -c "import json;j=json.loads(open('$F/swarm_${v}_x${sc}_$i.json').read().strip().splitlines()[-1]);w=j.get('wire_stats',{});print('$v x$sc', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB', [(t['name'], round(t['user_s']+t['sys_s'],2)) for t in j['leech_thread_cpu'][:6]], 'gpu', w.get('gpu_pieces'), 'overflow', w.get('gpu_overflow'), 'allocs', w.get('pool_allocs'))"
    done
  done
done
