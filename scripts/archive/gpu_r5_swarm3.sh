#!/bin/bash
# Round 5, third swarm call: config 6 with every piece SHA-1'd on the gfx950 PartHasher
# (--swarm-gpu-inflight 4096: no host overflow) and a piece pool big enough that no buffer is
# made or page-locked again after the first download (--swarm-pool-mb 4096), against the host
# SHA-1, on the 2 GB torrent and on an 8 GB one (--scale 4: the device's ~75 ms per piece is
# a smaller share of a longer job). 2 alternating rounds, 3 downloads per process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_swarm12}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
for sc in 1 4; do
  for i in 1 2; do
    for v in host gpu; do
      case $v in
        host) a="--swarm-verify cpu" ;;
        gpu) a="--swarm-verify gpu --swarm-gpu-inflight 4096 --swarm-pool-mb 4096" ;;
      esac
      step "$v x$sc $i"
      timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --reps 3 --scale $sc $a > $F/swarm_${v}_x${sc}_$i.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
      python -c "import json;j=json.loads(open('$F/swarm_${v}_x${sc}_$i.json').read().strip().splitlines()[-1]);w=j.get('wire_stats',{});print('$v x$sc', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB', [(t['name'], round(t['user_s']+t['sys_s'],2)) for t in j['leech_thread_cpu'][:6]], 'gpu', w.get('gpu_pieces'), 'overflow', w.get('gpu_overflow'), 'allocs', w.get('pool_allocs'), 'locks', w.get('pool_locks'))"
    done
  done
done
