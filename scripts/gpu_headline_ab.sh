#!/bin/bash
# Headline repeatability on one box + reference-mode torrent configs (serial webseed verify).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/hab.jsonl; : > $O
b() { echo "== $*" >&2; timeout -k 10 300 python bench.py "$@" >> $O 2>> gpurun_out/hab.err || exit 1; }
b --steps 16 --jobs-per-step 8
b
b --steps 16 --jobs-per-step 8
b
b --steps 16 --jobs-per-step 8 --concurrency 3
b --steps 16 --jobs-per-step 8 --concurrency 6
timeout -k 10 900 python -m downloader_amd.bench.configs --config 3 --config 4 --mode reference > gpurun_out/hab_ref34.jsonl 2>> gpurun_out/hab.err || exit 1
cat $O
