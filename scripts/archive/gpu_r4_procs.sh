#!/bin/bash
# Round 4: worker processes x jobs per process for one 16-CPU rank (16 relays in flight in
# each layout but 3x3), alternating, 3 rounds - the headline's default is 2 x 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_procs}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
for r in 1 2 3; do
  for v in "p2c4 --procs-per-rank 2 --concurrency 4" "p4c2 --procs-per-rank 4 --concurrency 2" "p3c3 --procs-per-rank 3 --concurrency 3" "p8c1 --procs-per-rank 8 --concurrency 1"; do
    set -- $v; n=$1; shift
    timeout -k 10 300 python bench.py --no-compare-single-put --no-compare-crc "$@" > $F/${n}_$r.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
    python -c "import json;j=json.load(open('$F/${n}_$r.json'));print('$n $r', j['value'], j['p50_job_latency_s'], j['worker_cpu_s_per_GB'], j['peer_cpu_s_per_GB'], j['event_loop_busy'], j['pipe_kb'])"
  done
done
