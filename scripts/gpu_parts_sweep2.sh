#!/bin/bash
# Fewer, bigger requests per job: part size / single-PUT threshold x jobs in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/ps2.jsonl; : > $O
b() { echo "== $*" >&2; echo "{\"args\": \"$*\"}" >> $O; timeout -k 10 300 python bench.py --steps 16 --jobs-per-step 8 "$@" >> $O 2>> gpurun_out/ps2.err || exit 1; }
for r in 1 2; do
b --part-mb 50
b --part-mb 64
b --part-mb 100 --threshold-mb 64
b --threshold-mb 128
b --threshold-mb 128 --concurrency 8
b --part-mb 34
done
b --part-mb 50 --concurrency 6
b --part-mb 25
cat $O
