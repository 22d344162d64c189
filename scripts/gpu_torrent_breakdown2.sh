#!/bin/bash
# Configs 3/4 after moving job-dir removal off the critical path; reference mode for A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/tb2.jsonl; : > $O
s() { echo "== $*" >&2; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $O 2>> gpurun_out/tb2.err || exit 1; }
s --config 3
s --config 3
s --config 4
s --config 4
s --config 3 --mode reference
s --config 4 --mode reference
cat $O
