#!/bin/bash
# Round 6: config 6 with the gfx950 SHA-1 and the adaptive host tail (rate x measured device
# latency) against the host, alternating, at 2 GB and 16 GB; and the split kernel's GPU tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_tail}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_hash.py tests/test_torrent.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $F/pytest.txt 2>&1 || { tail -30 $F/pytest.txt; exit 1; }
tail -1 $F/pytest.txt
for sc in ${SCALES:-1 8}; do
  for r in 1 2; do
    for v in gpu cpu; do
      step "config6 $v x$sc #$r"
      timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --reps 3 --scale $sc --swarm-verify $v ${EXTRA} > $F/swarm_${v}_x${sc}_$r.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
      python -c "import json;j=json.loads(open('$F/swarm_${v}_x${sc}_$r.json').read().strip().splitlines()[-1]);w=j.get('wire_stats',{});print('$v x$sc', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB', 'tail', [round(b/2**20) for b in j.get('gpu_host_tail_bytes_reps',[])], 'MiB', 'gpu pieces', w.get('gpu_pieces'), 'lat ms', round(w.get('gpu_latency_ms_mean',0),1), round(w.get('gpu_latency_ms_max',0),1))"
    done
  done
done
