#!/bin/bash
# Default bench (auto quota-share pinning), headline vs reference, and a 2-rank run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
timeout -k 10 300 python bench.py > gpurun_out/pb_default.json 2> gpurun_out/pb.err && \
timeout -k 10 600 python bench.py --steps 16 --jobs-per-step 8 --compare-reference > gpurun_out/pb_headline.json 2>> gpurun_out/pb.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/pb_n2.json 2>> gpurun_out/pb.err
rc=$?
cat gpurun_out/pb_default.json gpurun_out/pb_headline.json gpurun_out/pb_n2.json
exit $rc
