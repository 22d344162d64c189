#!/bin/bash
# Round-3: splice pipe capacity vs throughput on one rank, to price the smaller pipes a node
# of 8 ranks gets from the uid's 64 MiB pipe budget (bench.py sizes them per worker: 1 MiB at
# 1-2 ranks, 512 KiB at 4, 256 KiB at 8). Headline and config 4 at 1024 / 256 / 128 KiB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_pipes}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
summ() { python -c "import json,sys
for l in open(sys.argv[1]):
  j=json.loads(l); print(sys.argv[1].split('/')[-1], {k:j.get(k) for k in sys.argv[2].split(',')})" "$@"; }
for round in 1 2; do
  for kb in 1024 256 128; do
    timeout -k 10 200 python bench.py --pipe-kb $kb --no-compare-single-put > $F/c2_${kb}_${round}.json 2>> $F/err.txt || exit 1
    summ $F/c2_${kb}_${round}.json value,p50_job_latency_s,worker_cpu_s_per_GB,peer_cpu_s_per_GB,pipe_kb,pipes_short
  done
done
timeout -k 10 200 python bench.py --no-compare-single-put > $F/c2_auto.json 2>> $F/err.txt || exit 1
summ $F/c2_auto.json value,p50_job_latency_s,pipe_kb,pipes_short
