#!/bin/bash
# N=1 headline: unpinned vs pinned to 16 / 32 contiguous CPUs (quota is 16), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/pin.jsonl; : > $O
lscpu > gpurun_out/pin_lscpu.txt 2>&1 || true
b() { echo "== $*" >&2; echo "{\"args\": \"$*\"}" >> $O; timeout -k 10 300 python bench.py --steps 16 --jobs-per-step 8 "$@" >> $O 2>> gpurun_out/pin.err || exit 1; }
for r in 1 2 3; do
  b --cpus-per-rank -1
  b --cpus-per-rank 16
  b --cpus-per-rank 32
done
b --cpus-per-rank 16 --concurrency 6
b --cpus-per-rank 24
cat $O
