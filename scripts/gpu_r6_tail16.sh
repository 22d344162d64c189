#!/bin/bash
# Round 6: host tail of the streamed torrent's relayed parts (stream_gpu_tail 32 / 16 / 24)
# with parts staged in L2 + streamed (STAGER_PART_NT=1), pinned torrent A/B (config 4, 20 GB),
# alternating on one box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_tail16}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
n=0
for t in ${TAILS:-32 16 24 32 16 24 32 16 24 32 16 24}; do
  n=$((n+1))
  echo "== tail $t #$n $(date +%T)"
  timeout -k 10 400 python -m downloader_amd.bench.torrent_ab --gb 20 --pairs ${PAIRS:-4} --set stream_gpu_tail=$t > $F/ab_t${t}_$n.json 2>> $F/ab.err || { tail -20 $F/ab.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/ab_t${t}_$n.json').read().strip().splitlines()[-1]);g,h=j['torrent_gpu_MBps'],j['torrent_host_MBps'];print('tail $t', g, h, round(g/h,3), j['gpu_part_share'], j['torrent_gpu_MBps_runs'], j['torrent_host_MBps_runs'], j['torrent_gpu_worker_cpu_s_per_GB'], j['torrent_host_worker_cpu_s_per_GB'], j.get('gpu_lanes_per_launch'))"
done
