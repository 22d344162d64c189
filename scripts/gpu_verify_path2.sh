#!/bin/bash
# Configs 3/4: host vs GPU (prewarmed verifier) incremental piece verification.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/vp2.jsonl; : > $O
s() { echo "== $*" >&2; echo "{\"args\": \"$*\"}" >> $O; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $O 2>> gpurun_out/vp2.err || exit 1; }
s --config 4 --verify-backend cpu
s --config 4 --verify-backend auto --gpu-prewarm --webseed-verify-depth 16
s --config 4 --verify-backend auto --gpu-prewarm --webseed-verify-depth 32
s --config 4 --verify-backend cpu --webseed-verify-depth 16
s --config 3 --verify-backend cpu
s --config 3 --verify-backend auto --gpu-prewarm --webseed-verify-depth 16
s --config 3 --verify-backend auto --gpu-prewarm --webseed-verify-depth 32
s --config 3 --verify-backend auto --gpu-prewarm --webseed-verify-depth 32 --webseed-chunk-mb 32
cat $O
