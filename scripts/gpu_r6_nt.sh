#!/bin/bash
# Round 6: how a hashed relay fills its 64 MiB part buffer (STAGER_PART_NT 0: peek into it;
# 1: device-bound parts staged in L2 and streamed with non-temporal stores; 2: every part),
# pinned torrent A/B (config 4, 20 GB), alternating on one box. Then the checked headline with
# a cache-missing 8 MiB peek buffer vs the default 512 KiB (the memory-traffic hypothesis).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_nt}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
n=0
for m in ${MODES:-0 1 2 0 1 2}; do
  n=$((n+1))
  echo "== part_nt $m #$n $(date +%T)"
  STAGER_PART_NT=$m timeout -k 10 400 python -m downloader_amd.bench.torrent_ab --gb 20 --pairs ${PAIRS:-3} > $F/ab_nt${m}_$n.json 2>> $F/ab.err || { tail -20 $F/ab.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/ab_nt${m}_$n.json').read().strip().splitlines()[-1]);g,h=j['torrent_gpu_MBps'],j['torrent_host_MBps'];print('part_nt $m', g, h, round(g/h,3), j['gpu_part_share'], j['torrent_gpu_MBps_runs'], j['torrent_host_MBps_runs'], j['torrent_gpu_worker_cpu_s_per_GB'], j['torrent_host_worker_cpu_s_per_GB'])"
done
[ -n "${SKIP_PEEK:-}" ] && exit 0
for k in 512 8192 512 8192; do
  n=$((n+1))
  echo "== peek $k #$n $(date +%T)"
  STAGER_PEEK_KB=$k timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-compare-unchecked --no-compare-reference --workers-curve "" --no-config1 --torrent-gb 0 > $F/peek_${k}_$n.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/peek_${k}_$n.json').read().strip().splitlines()[-1]);print('peek $k', j['value'], j['p50_job_latency_s'], j['cpu_utilisation'], j.get('worker_cpu_s_per_GB'), j.get('peer_cpu_s_per_GB'))"
done
