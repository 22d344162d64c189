#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
timeout -k 10 600 python -m downloader_amd.bench.configs --config 3 --config 4 > gpurun_out/c34b.jsonl 2> gpurun_out/c34b.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 4 --piece-mb 16 >> gpurun_out/c34b.jsonl 2>> gpurun_out/c34b.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 4 --stage-dir /dev/shm >> gpurun_out/c34b.jsonl 2>> gpurun_out/c34b.err
echo "exit $?"
