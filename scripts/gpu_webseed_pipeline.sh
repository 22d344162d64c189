#!/bin/bash
# Webseed streams sweep after pipelining fetch and verify inside each stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/wp.jsonl; : > $O
s() { echo "== $*" >&2; echo "{\"args\": \"$*\"}" >> $O; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $O 2>> gpurun_out/wp.err || exit 1; }
for st in 1 2 4 8; do s --config 3 --webseed-streams $st; done
s --config 3 --webseed-streams 4 --webseed-verify-depth 1
s --config 3 --webseed-streams 2 --webseed-verify-depth 4
for st in 2 4 8; do s --config 4 --webseed-streams $st; done
cat $O
