#!/bin/bash
# Webseed streams with fetch/verify overlap + file spreading (config 4 is 50 files).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/wp2.jsonl; : > $O
s() { echo "== $*" >&2; echo "{\"args\": \"$*\"}" >> $O; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $O 2>> gpurun_out/wp2.err || exit 1; }
for st in 4 8 16; do s --config 4 --webseed-streams $st; done
s --config 4 --webseed-streams 8 --webseed-chunk-mb 32
s --config 3 --webseed-streams 2 --webseed-verify-depth 4
s --config 3 --webseed-streams 4 --webseed-verify-depth 4
s --config 3
cat $O
