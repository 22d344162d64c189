#!/bin/bash
# Round 6: the driver's bench command three times back to back on one box (the headline's
# spread on the round's last tree).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_reps}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
for i in 1 2 3; do
  echo "== bench $i $(date +%T)"
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python3 -c "import json;j=json.loads(open('$F/bench_$i.json').read().strip().splitlines()[-1]);print({k: j.get(k) for k in ('value','p50_job_latency_s','vs_baseline','unchecked_MBps','reference_mode_MBps','torrent_gpu_MBps','torrent_host_MBps','gpu_part_share','cpu_utilisation')})"
done
