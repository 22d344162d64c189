#!/bin/bash
# Round 5, fifth swarm call: config 6 with the device SHA-1 handing the last GB to the host
# (download.swarm_gpu_tail_mb, default 1024, at most a quarter of the torrent) vs all on the
# device (--swarm-gpu-tail-mb 0) vs the host, at 2, 8 and 16 GB, with a piece pool big enough
# (POOL=8192: --swarm-pool-mb 8192) that no download after the first makes or page-locks
# buffers; without POOL the defaults (4 GB pool, 4 GB verify backlog).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_swarm18}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
for sc in ${SCALES:-1 4 8}; do
  for i in 1 2; do
    for v in ${VARIANTS:-cpu tail gpu}; do
      case $v in
        cpu) a="--swarm-verify cpu" ;;
        tail) a="--swarm-verify gpu ${POOL:+--swarm-pool-mb $POOL}" ;;
        gpu) a="--swarm-verify gpu ${POOL:+--swarm-pool-mb $POOL} --swarm-gpu-tail-mb 0" ;;
      esac
      step "$v x$sc $i"
      timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --reps 3 --scale $sc $a > $F/swarm_${v}_x${sc}_$i.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
      python -c "import json;j=json.loads(open('$F/swarm_${v}_x${sc}_$i.json').read().strip().splitlines()[-1]);w=j.get('wire_stats',{});print('$v x$sc', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB', [(t['name'], round(t['user_s']+t['sys_s'],2)) for t in j['leech_thread_cpu'][:5]], 'gpu', w.get('gpu_pieces'), 'allocs', w.get('pool_allocs'))"
    done
  done
done
