#!/bin/bash
# Round 6: config 6 at 2 GB - the gfx950 arm with the auto tail (rate x measured device
# latency) at its defaults (x 2, at most 3/4 of the torrent) and at x 3 / at most 0.85, and the
# host arm, alternating.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_tailx4}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
step() { echo "== $1 $(date +%T)"; }
for r in 1 2; do
  for v in gpu gpu75 cpu; do
    step "config6 $v #$r"
    case $v in
      cpu) a="--swarm-verify cpu";;
      gpu) a="--swarm-verify gpu";;
      gpu75) a="--swarm-verify gpu --swarm-gpu-tail-x 3 --swarm-gpu-tail-max 0.85";;
    esac
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 6 --reps 4 --scale ${SCALE:-1} $a > $F/swarm_${v}_$r.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
    python -c "import json;j=json.loads(open('$F/swarm_${v}_$r.json').read().strip().splitlines()[-1]);w=j.get('wire_stats',{});print('$v', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB', 'tail', [round(b/2**20) for b in j.get('gpu_host_tail_bytes_reps',[])], 'MiB', 'gpu', w.get('gpu_pieces'), 'lat ms', round(w.get('gpu_latency_ms_mean',0),1), 'locks', j.get('pool_locks_reps'))"
  done
done
