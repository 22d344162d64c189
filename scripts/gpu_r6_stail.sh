#!/bin/bash
# Round 6: the streamed torrent's host-hashed tail (stream_gpu_tail parts) with the split-wave
# kernel's 57 ms per piece: 96 (default) / 64 / 48 / 96 again, 5 pairs each (config 4, 20 GB).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_stail}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
n=0
for t in ${TAILS:-96 64 48 96}; do
  n=$((n+1))
  echo "== tail $t $(date +%T)"
  timeout -k 10 400 python -m downloader_amd.bench.torrent_ab --gb 20 --pairs ${PAIRS:-5} --set stream_gpu_tail=$t > $F/ab_t${t}_$n.json 2>> $F/ab.err || { tail -20 $F/ab.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/ab_t${t}_$n.json').read().strip().splitlines()[-1]);print('tail $t', {k: j.get(k) for k in ('torrent_gpu_MBps','torrent_host_MBps','gpu_part_share','gpu_lanes_per_launch','torrent_gpu_MBps_runs','torrent_host_MBps_runs','torrent_gpu_worker_cpu_s_per_GB','torrent_host_worker_cpu_s_per_GB')})"
done
