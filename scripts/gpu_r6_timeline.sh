#!/bin/bash
# Round 6: where a streamed torrent job's time goes on each arm (torrent/stream.py timeline),
# pinned torrent A/B at 20 and 40 GB on one box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_timeline}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
n=0
for g in ${SIZES:-20 40 20}; do
  n=$((n+1))
  echo "== gb $g #$n $(date +%T)"
  timeout -k 10 400 python -m downloader_amd.bench.torrent_ab --gb $g --pairs ${PAIRS:-4} > $F/ab_g${g}_$n.json 2>> $F/ab.err || { tail -20 $F/ab.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/ab_g${g}_$n.json').read().strip().splitlines()[-1]);g,h=j['torrent_gpu_MBps'],j['torrent_host_MBps'];print('gb $g', g, h, round(g/h,3));print(' gpu ', j['torrent_gpu_timeline_s']);print(' host', j['torrent_host_timeline_s'])"
done
