#!/bin/bash
# End-of-round re-validation of the committed tree: GPU tier, smoke, headline bench x2, N=2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/close}
mkdir -p $F
export LOG_LEVEL=error
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $F/bench_default.json 2> $F/bench.err && \
timeout -k 10 300 python bench.py --compare-reference > $F/bench_vs_reference.json 2>> $F/bench.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 > $F/bench_n2.json 2>> $F/bench.err
rc=$?
tail -3 $F/pytest_gpu.txt
tail -2 $F/smoke.txt
cat $F/bench_*.json
exit $rc
