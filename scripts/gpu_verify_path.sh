#!/bin/bash
# GPU tier + configs 3/4 with webseed runs verified on the host vs on the GPU (batcher).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
O=gpurun_out/vp.jsonl; : > $O
s() { echo "== $*" >&2; echo "{\"args\": \"$*\"}" >> $O; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $O 2>> gpurun_out/vp.err || exit 1; }
s --config 4 --verify-backend cpu
s --config 4 --verify-backend gpu --webseed-verify-depth 8
s --config 4 --verify-backend gpu --webseed-verify-depth 16
s --config 4 --verify-backend gpu --webseed-streams 8 --webseed-verify-depth 8
s --config 3 --verify-backend cpu
s --config 3 --verify-backend gpu --webseed-verify-depth 8
s --config 3 --verify-backend gpu --webseed-verify-depth 16
cat $O
