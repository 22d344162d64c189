#!/bin/bash
# Session-2 validation: GPU tier, smoke, headline bench, BASELINE configs 1/3/4/5 tuned and
# reference-equivalent, N=2 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/s2final
mkdir -p $F
export LOG_LEVEL=error
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $F/bench_default.json 2> $F/bench.err && \
timeout -k 10 300 python bench.py > $F/bench_default2.json 2>> $F/bench.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 > $F/bench_n2.json 2>> $F/bench.err && \
timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 > $F/configs.jsonl 2> $F/configs.err && \
timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 --mode reference > $F/configs_ref.jsonl 2>> $F/configs.err
rc=$?
tail -1 $F/pytest_gpu.txt; tail -1 $F/smoke.txt
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/s2final/bench_*.json")):
    for l in open(f):
        j = json.loads(l); print(f.split("/")[-1], j["value"], j["p50_job_latency_s"], j["config"]["parallelism"])
for f in ("configs", "configs_ref"):
    try:
        for l in open(f"gpurun_out/s2final/{f}.jsonl"):
            j = json.loads(l); print(f, {k: j[k] for k in list(j)[:9]})
    except FileNotFoundError:
        pass
PY
exit $rc
