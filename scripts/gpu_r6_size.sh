#!/bin/bash
# Round 6: torrent A/B at 10 / 20 / 40 GB (per-job fixed costs vs the steady rate), pinned,
# alternating on one box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_size}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
n=0
for g in ${SIZES:-10 20 40 10 20 40}; do
  n=$((n+1))
  echo "== gb $g #$n $(date +%T)"
  timeout -k 10 400 python -m downloader_amd.bench.torrent_ab --gb $g --pairs ${PAIRS:-3} > $F/ab_g${g}_$n.json 2>> $F/ab.err || { tail -20 $F/ab.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/ab_g${g}_$n.json').read().strip().splitlines()[-1]);g,h=j['torrent_gpu_MBps'],j['torrent_host_MBps'];print('gb $g', g, h, round(g/h,3), j['gpu_part_share'], j['torrent_gpu_MBps_runs'], j['torrent_host_MBps_runs'], j['torrent_gpu_worker_cpu_s_per_GB'], j['torrent_host_worker_cpu_s_per_GB'])"
done
