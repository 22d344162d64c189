#!/bin/bash
# Round-3: config 9 (control-plane ceiling) with tracing off vs on after the span exporter
# moved to an interval-batched writer thread, and the headline with CRC32C on the plain relay
# (tee'd pipe, one user-space copy) vs the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_trace}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
summ() { python -c "import json,sys
for l in open(sys.argv[1]):
  j=json.loads(l); print(sys.argv[1].split('/')[-1], {k:j.get(k) for k in sys.argv[2].split(',')})" "$@"; }
for round in 1 2; do
  for tr in off on; do
    flag=""; [ $tr = on ] && flag="--trace"
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 9 --jobs 5000 --concurrency 64 $flag > $F/c9_${tr}_${round}.json 2>> $F/err.txt || exit 1
    summ $F/c9_${tr}_${round}.json trace,jobs_per_s,worker_cpu_ms_per_job,p50_latency_s,spans_written
  done
done
for round in 1 2; do
  for ck in auto always; do
    timeout -k 10 200 python bench.py --checksum $ck --no-compare-single-put > $F/c2_${ck}_${round}.json 2>> $F/err.txt || exit 1
    summ $F/c2_${ck}_${round}.json value,p50_job_latency_s,worker_cpu_s_per_GB,peer_cpu_s_per_GB,sink_mismatches
  done
done
