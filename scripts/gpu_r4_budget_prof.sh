#!/bin/bash
# Round 4: the part-budget A/B (scripts/gpu_r4_budget.sh) then the rocprofv3 trace of config 4
# (scripts/gpu_r4_prof.sh), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r4_budget.sh && bash scripts/gpu_r4_prof.sh
