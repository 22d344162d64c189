#!/bin/bash
# Round 5, second swarm call: config 6 (4 seeders in their own processes, 2 GB, 4 MiB pieces,
# loopback) with the native wire requesting whole pieces by itself (--wire-requests native,
# the default now) against every block requested and booked in Python (--wire-requests
# python, the first round-5 wire) and the all-Python wire, host-verified; then the native
# requests with pieces SHA-1'd on the gfx950 PartHasher. 3 alternating rounds, 3 downloads per
# process (the first is its cold one). The GPU test of the wire's device mode first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_swarm9}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
step gpu; timeout -k 10 300 python -u -m pytest tests/test_gpu_hash.py -m gpu -x -v --timeout 120 --timeout-method thread -k swarm > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
for i in 1 2 3; do
  for v in ${VARIANTS:-python blocks owned owned_gpu}; do
    case $v in
      python) a="--wire python" ;;
      blocks) a="--wire native --swarm-verify cpu --wire-requests python" ;;
      owned) a="--wire native --swarm-verify cpu --wire-requests native" ;;
      owned_gpu) a="--wire native --swarm-verify gpu --wire-requests native" ;;
    esac
    step "$v $i"
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 6 --reps 3 $a > $F/swarm_${v}_$i.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
    python -c "import json;j=json.loads(open('$F/swarm_${v}_$i.json').read().strip().splitlines()[-1]);w=j.get('wire_stats',{});print('$v', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB', [(t['name'], round(t['user_s']+t['sys_s'],2)) for t in j['leech_thread_cpu'][:6]], 'gpu', w.get('gpu_pieces'), 'assigned', w.get('assigned'), 'requests', w.get('requests'))"
  done
done
