#!/bin/bash
# Current defaults: bench default, headline vs reference, jobs-in-flight variants, N=2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
O=gpurun_out/bd.jsonl; : > $O
b() { echo "== $*" >&2; echo "{\"args\": \"$*\"}" >> $O; timeout -k 10 600 python bench.py "$@" >> $O 2>> gpurun_out/bd.err || exit 1; }
b
b --steps 16 --jobs-per-step 8 --compare-reference
b --steps 16 --jobs-per-step 8 --concurrency 6
b --steps 16 --jobs-per-step 8 --concurrency 8
b
echo '{"args": "N=2"}' >> $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 >> $O 2>> gpurun_out/bd.err || exit 1
cat $O
