#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
OUT=gpurun_out/configs34.jsonl
: > $OUT
step() { echo "== $*" >&2; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $OUT 2>>gpurun_out/configs.err || exit 1; }
step --config 3 --mode tuned --verify-backend cpu
step --config 3 --mode tuned --verify-backend gpu
step --config 4 --mode tuned --verify-backend cpu
cat $OUT
