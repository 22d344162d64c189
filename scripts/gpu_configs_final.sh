#!/bin/bash
# All BASELINE configs, tuned vs reference-equivalent mode, current defaults.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/cf.jsonl; : > $O
s() { echo "== $*" >&2; timeout -k 10 900 python -m downloader_amd.bench.configs "$@" >> $O 2>> gpurun_out/cf.err || exit 1; }
s --config 1 --config 3 --config 4
s --config 1 --config 3 --config 4 --mode reference
s --config 4 --verify-backend cpu
s --config 5
s --config 5 --mode reference
timeout -k 10 600 python bench.py --steps 16 --jobs-per-step 8 --compare-reference > gpurun_out/cf_headline.json 2>> gpurun_out/cf.err || exit 1
cat $O gpurun_out/cf_headline.json
