#!/bin/bash
# Round-3 validation of the current tree: GPU tier, smoke, the driver's default headline
# twice, and config 5 with one job in flight per worker (the reference's prefetch 1) at
# retry backoff 0.5 vs 5 s, broker-held delay vs in-consumer sleep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_quick}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $F/bench_1.json 2> $F/bench.err && \
timeout -k 10 300 python bench.py > $F/bench_2.json 2>> $F/bench.err || exit 1
tail -1 $F/pytest_gpu.txt; tail -1 $F/smoke.txt; cat $F/bench_1.json $F/bench_2.json
for delay in queue sleep; do
  for b in 0.5 5; do
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 5 --concurrency 1 --retry-backoff-s $b \
      --retry-delay $delay > $F/c5_c1_${delay}_${b}.json 2>> $F/err.txt || exit 1
    python -c "import json;j=json.load(open('$F/c5_c1_${delay}_${b}.json'));print('$delay', $b, {k:j[k] for k in ('healthy_p50_s','healthy_p99_s','p99_latency_s','jobs_per_s')})"
  done
done
