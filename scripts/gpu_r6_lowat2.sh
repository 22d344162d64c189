#!/bin/bash
# Round 6: SO_RCVLOWAT mark of the relay's peek and the sink (256 KiB default vs 384 / 512),
# checked headline only (no extras), alternating, on one box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_lowat2}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
n=0
for k in 256 512 384 256 512 384; do
  n=$((n+1))
  echo "== lowat $k #$n $(date +%T)"
  STAGER_RCVLOWAT_KB=$k STAGER_BLOBD_RCVLOWAT_KB=$k timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-compare-unchecked --no-compare-reference --workers-curve "" --no-config1 --torrent-gb 0 > $F/lowat_${k}_$n.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/lowat_${k}_$n.json').read().strip().splitlines()[-1]);print('lowat $k', j['value'], j['p50_job_latency_s'], j['cpu_utilisation'], j.get('worker_cpu_s_per_GB'), j.get('peer_cpu_s_per_GB'))"
done
