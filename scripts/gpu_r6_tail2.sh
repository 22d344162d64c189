#!/bin/bash
# Round 6: config 6 with the gfx950 SHA-1 and the auto tail at its defaults (x 2 the measured
# device latency, at most 3/4 of the torrent) vs the host, alternating, at 2 and 16 GB.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_tail2}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
step() { echo "== $1 $(date +%T)"; }
for sc in ${SCALES:-1 8}; do
  for r in 1 2; do
    for v in ${VERIFY:-gpu cpu}; do
      step "config6 $v x$sc #$r"
      timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --reps ${REPS:-4} --scale $sc --swarm-verify $v > $F/swarm_${v}_x${sc}_$r.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
      python -c "import json;j=json.loads(open('$F/swarm_${v}_x${sc}_$r.json').read().strip().splitlines()[-1]);w=j.get('wire_stats',{});print('$v x$sc', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB', 'tail', [round(b/2**20) for b in j.get('gpu_host_tail_bytes_reps',[])], 'MiB', 'gpu', w.get('gpu_pieces'), 'lat ms', round(w.get('gpu_latency_ms_mean',0),1))"
    done
  done
done
