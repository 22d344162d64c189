#!/bin/bash
# Round 6: with sha1_lanes_split - the streamed torrent's host tail (32 / 16 parts) x the
# PartHasher's stream split (2 copy + 2 compute, or 1 copy + 3 compute: a part's launch waits
# less for a stream), 4 pairs each (config 4, 20 GB).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_stail3}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
for c in "32 2" "32 1" "16 2" "16 1"; do
  set -- $c
  echo "== tail $1 copy $2 $(date +%T)"
  timeout -k 10 400 python -m downloader_amd.bench.torrent_ab --gb 20 --pairs ${PAIRS:-4} --set stream_gpu_tail=$1 --set stream_gpu_copy_streams=$2 > $F/ab_t$1_c$2.json 2>> $F/ab.err || { tail -20 $F/ab.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/ab_t$1_c$2.json').read().strip().splitlines()[-1]);g,h=j['torrent_gpu_MBps'],j['torrent_host_MBps'];print('tail $1 copy $2', g, h, round(g/h,3), j['gpu_part_share'], j['torrent_gpu_MBps_runs'], j['torrent_host_MBps_runs'], j['torrent_gpu_worker_cpu_s_per_GB'], j['torrent_host_worker_cpu_s_per_GB'])"
done
