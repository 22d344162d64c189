#!/bin/bash
# GPU tests + verification benchmark + rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python -m downloader_amd.bench.verify_bench --gib 4 --piece-mb 1 > gpurun_out/verify_bench.jsonl 2> gpurun_out/verify_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_verify -o run --output-format csv -- python -m downloader_amd.bench.verify_bench --kernel-only > gpurun_out/prof_verify.log 2>&1
echo "exit $?"
