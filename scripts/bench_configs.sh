#!/bin/bash
# BASELINE.json configs 1,3,4,5 (config 2 = bench.py), tuned vs reference-equivalent mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
OUT=gpurun_out/configs.jsonl
: > $OUT
step() { echo "== $*" >&2; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $OUT 2>>gpurun_out/configs.err || exit 1; }
step --config 1 --mode reference
step --config 1 --mode tuned
step --config 3 --mode reference
step --config 3 --mode tuned --verify-backend cpu
step --config 3 --mode tuned --verify-backend gpu
step --config 4 --mode tuned --verify-backend auto
step --config 4 --mode reference
step --config 5 --mode tuned --workers 4 --qps 50
step --config 5 --mode reference --workers 4 --qps 50
cat $OUT
