#!/bin/bash
# Quick re-validation: GPU tier, smoke, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_quick}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $F/bench_default.json 2> $F/bench.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $F/bench_20_5.json 2>> $F/bench.err
rc=$?
tail -2 $F/pytest_gpu.txt
tail -1 $F/smoke.txt
cat $F/bench_default.json $F/bench_20_5.json
exit $rc
