#!/bin/bash
# Round 6: the checked headline alone (no extras), four back-to-back runs on one box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_head}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
for i in 1 2 3 4; do
  echo "== headline $i $(date +%T)"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-compare-unchecked --no-compare-reference --workers-curve "" --no-config1 --torrent-gb 0 > $F/head_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/head_$i.json').read().strip().splitlines()[-1]);print('headline', j['value'], j['p50_job_latency_s'], j['cpu_utilisation'], j.get('worker_cpu_s_per_GB'), j.get('peer_cpu_s_per_GB'))"
done
