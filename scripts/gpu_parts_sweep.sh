#!/bin/bash
# Headline with quota-share pinning: part size x jobs in flight (Python per-request overhead).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/ps.jsonl; : > $O
b() { echo "== $*" >&2; echo "{\"args\": \"$*\"}" >> $O; timeout -k 10 300 python bench.py --steps 16 --jobs-per-step 8 "$@" >> $O 2>> gpurun_out/ps.err || exit 1; }
b
b --part-mb 32
b --part-mb 50
b --concurrency 8
b --part-mb 32 --concurrency 8
b --part-mb 50 --concurrency 8
b --concurrency 8 --jobs-per-step 16
b --part-mb 8
b
cat $O
