#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/cws2.jsonl; : > $O
s() { echo "== $*" >&2; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $O 2>> gpurun_out/cws2.err || exit 1; }
s --config 3
s --config 4
s --config 4 --webseed-streams 12
s --config 4 --webseed-chunk-mb 128
s --config 3 --webseed-streams 12 --webseed-chunk-mb 128
cat $O
