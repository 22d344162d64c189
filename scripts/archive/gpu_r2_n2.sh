#!/bin/bash
# Rehearsal of the driver's multi-rank bench on the 1-GPU box: N=2 ranks via torch.distributed.run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_n2}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $F/bench_n2.json 2> $F/bench_n2.err && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $F/bench_n1.json 2>> $F/bench_n2.err
rc=$?
cat $F/bench_n2.json $F/bench_n1.json
tail -5 $F/bench_n2.err
exit $rc
