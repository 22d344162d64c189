#!/bin/bash
# Round 6: parts relayed at once per streamed torrent job (torrent_stream_parallel 16 / 24 /
# 32), pinned torrent A/B (config 4, 20 GB), 4 pairs each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_spar}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
for p in ${PARS:-16 24 32 16}; do
  echo "== parallel $p $(date +%T)"
  timeout -k 10 400 python -m downloader_amd.bench.torrent_ab --gb 20 --pairs ${PAIRS:-4} --set torrent_stream_parallel=$p > $F/ab_p$p.json 2>> $F/ab.err || { tail -20 $F/ab.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/ab_p$p.json').read().strip().splitlines()[-1]);g,h=j['torrent_gpu_MBps'],j['torrent_host_MBps'];print('parallel $p', g, h, round(g/h,3), j['gpu_part_share'], j['torrent_gpu_MBps_runs'], j['torrent_host_MBps_runs'], j['torrent_gpu_worker_cpu_s_per_GB'], j['torrent_host_worker_cpu_s_per_GB'])"
done
