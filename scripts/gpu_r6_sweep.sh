#!/bin/bash
# Round 6: concurrency x worker processes sweep of the checked headline (CRC32C on every part),
# headline only (no extras), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r6_sweep}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
X="--no-compare-unchecked --no-compare-reference --workers-curve= --torrent-gb 0"
for rep in 1 2; do
for p in ${PROCS:-2 3 4}; do
  for c in ${CONCS:-4 6 8}; do
    timeout -k 10 120 python bench.py --procs-per-rank $p --concurrency $c $X $EXTRA > $F/p${p}_c${c}_$rep.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
    python3 -c "
import json; j=json.load(open('$F/p${p}_c${c}_$rep.json'))
print('procs $p conc', j['concurrency_per_worker'], 'pipe', j['pipe_kb'], 'MB/s', j['value'], 'p50', j['p50_job_latency_s'], 'util', j['cpu_utilisation'], 'w', j['worker_cpu_s_per_GB'], 'peer', j['peer_cpu_s_per_GB'], 'loop', j['event_loop_busy'])"
  done
done
done
