#!/bin/bash
# What the driver runs at round end, plus the torrent/swarm configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
timeout -k 10 300 python -m pytest tests -m gpu -q > gpurun_out/r_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r_bench_default.json 2> gpurun_out/r_bench_default.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 3 --config 4 > gpurun_out/r_configs34.jsonl 2>> gpurun_out/r_configs.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 6 --piece-mb 1 > gpurun_out/r_swarm.jsonl 2>> gpurun_out/r_configs.err
echo "exit $?"
