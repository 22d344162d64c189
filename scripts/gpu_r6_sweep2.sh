#!/bin/bash
# Round 6: worker processes x jobs in flight x peek size for the checked headline, headline only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r6_sweep2}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
X="--no-compare-unchecked --no-compare-reference --workers-curve= --torrent-gb 0"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py "$@" $X > $F/$n.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
  python3 -c "
import json; j=json.load(open('$F/$n.json'))
print('$n', 'procs', j['procs_per_rank'], 'conc', j['concurrency_per_worker'], 'pipe', j['pipe_kb'], 'MB/s', j['value'], 'p50', j['p50_job_latency_s'], 'util', j['cpu_utilisation'], 'w', j['worker_cpu_s_per_GB'], 'peer', j['peer_cpu_s_per_GB'], 'relay', j['worker_breakdown']['relay_threads_cpu_s_per_GB'], 'other', j['worker_breakdown']['other_worker_cpu_s_per_GB'])"
}
for rep in 1 2; do
  for pc in 4:2 4:3 4:4 5:3 6:2 6:3 8:2; do
    p=${pc%:*}; c=${pc#*:}
    run p${p}_c${c}_$rep --procs-per-rank $p --concurrency $c
  done
  for kb in 256 1024; do
    STAGER_PEEK_KB=$kb run p4_c3_peek${kb}_$rep --procs-per-rank 4 --concurrency 3
  done
done
