#!/bin/bash
# Round-end style validation + refreshed config numbers with the current defaults.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
timeout -k 10 300 python -m pytest tests -m gpu -q > gpurun_out/r_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r_bench_default.json 2> gpurun_out/r_bench_default.err && \
timeout -k 10 600 python bench.py --steps 16 --jobs-per-step 8 --compare-reference > gpurun_out/r_bench_headline.json 2> gpurun_out/r_bench_headline.err && \
timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 > gpurun_out/r_configs134.jsonl 2>> gpurun_out/r_configs.err && \
timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --mode reference > gpurun_out/r_configs134_ref.jsonl 2>> gpurun_out/r_configs.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 4 --verify-backend cpu > gpurun_out/r_config4_cpuverify.jsonl 2>> gpurun_out/r_configs.err
rc=$?
tail -1 gpurun_out/r_pytest_gpu.log; cat gpurun_out/r_bench_default.json gpurun_out/r_bench_headline.json
echo "exit $rc"
