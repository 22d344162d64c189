#!/bin/bash
# Round-2 first validation on a fresh box: GPU tier, smoke, headline bench, rocprof of the
# gfx950 verifier, one config-4 run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=gpurun_out/r2_first
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $F/bench_default.json 2> $F/bench.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $F/bench_20_5.json 2>> $F/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $F/prof -o verify -- python3 -m downloader_amd.bench.verify_bench > $F/verify_bench.txt 2>&1
rc=$?
tail -3 $F/pytest_gpu.txt
cat $F/bench_default.json $F/bench_20_5.json
exit $rc
