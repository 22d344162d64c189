#!/bin/bash
# Round-2 validation after the ADVICE fixes (pooled relay part buffers, verify-task error
# handling): GPU tier, smoke, headline x2, configs 3/4 x3 reps with worker RSS, and a
# rocprofv3 kernel trace (CSV stats) of the gfx950 verifier bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_validate}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $F/bench_default.json 2> $F/bench.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $F/bench_20_5.json 2>> $F/bench.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 3 --config 4 --reps 3 > $F/configs34_tuned.jsonl 2> $F/configs.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $F/prof -o verify -- python3 -m downloader_amd.bench.verify_bench > $F/verify_bench.txt 2>&1
rc=$?
tail -2 $F/pytest_gpu.txt
cat $F/bench_default.json $F/bench_20_5.json
python3 - <<PY
import json
for l in open("$F/configs34_tuned.jsonl"):
    j = json.loads(l)
    print(j["config"], j["MBps"], j["MBps_reps"], j["worker_cpu_s"], j.get("worker_rss_after_MB"), j.get("worker_rss_peak_MB"), j.get("relay_pool_after"))
PY
exit $rc
