#!/bin/bash
# Round 4: GPU tier, then the part-budget A/B (scripts/archive/gpu_r4_budget.sh) then the rocprofv3 trace of config 4
# (scripts/archive/gpu_r4_prof.sh), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4_budget
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_budget/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r4_budget/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/r4_budget/pytest_gpu.txt
bash scripts/archive/gpu_r4_budget.sh && bash scripts/archive/gpu_r4_prof.sh
