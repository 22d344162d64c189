#!/bin/bash
# Is the event-loop thread the limit? Headline variants + configs 3/4 with 64 MiB parts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/lb.jsonl; : > $O
b() { echo "== $*" >&2; echo "{\"args\": \"$*\"}" >> $O; timeout -k 10 300 python bench.py --steps 16 --jobs-per-step 8 "$@" >> $O 2>> gpurun_out/lb.err || exit 1; }
b
b --concurrency 8
b --concurrency 8 --jobs-per-step 16
b --threshold-mb 128 --concurrency 8
b --threshold-mb 128 --concurrency 12 --jobs-per-step 12
timeout -k 10 900 python -m downloader_amd.bench.configs --config 3 --config 4 > gpurun_out/lb_c34.jsonl 2>> gpurun_out/lb.err || exit 1
cat $O gpurun_out/lb_c34.jsonl
