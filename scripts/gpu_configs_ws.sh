#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/cws.jsonl; : > $O
s() { echo "== $*" >&2; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $O 2>> gpurun_out/cws.err || exit 1; }
s --config 4 --webseed-streams 8
s --config 4 --webseed-streams 8 --webseed-chunk-mb 64
s --config 4 --webseed-streams 16 --webseed-chunk-mb 16
s --config 4 --webseed-streams 4 --webseed-chunk-mb 64
s --config 1 --mode reference
s --config 3 --mode reference
s --config 4 --mode reference
cat $O
