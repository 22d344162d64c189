#!/bin/bash
# Round-end numbers with the current defaults (GPU tier, smoke, bench, configs, N=2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export LOG_LEVEL=error
F=gpurun_out/final
timeout -k 10 300 python -m pytest tests -m gpu -q > $F/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $F/bench_default.json 2> $F/bench.err && \
timeout -k 10 300 python bench.py > $F/bench_default2.json 2>> $F/bench.err && \
timeout -k 10 600 python bench.py --compare-reference > $F/bench_vs_reference.json 2>> $F/bench.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 > $F/bench_n2.json 2>> $F/bench.err && \
timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 > $F/configs134.jsonl 2>> $F/configs.err && \
timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --mode reference > $F/configs134_ref.jsonl 2>> $F/configs.err
rc=$?
tail -1 $F/pytest_gpu.txt
cat $F/bench_default.json $F/bench_default2.json $F/bench_vs_reference.json $F/bench_n2.json
exit $rc
