#!/bin/bash
# Round 6: the check call (GPU tier, smoke, bench line, torrent A/B + trace) then the swarm call
# (heterogeneous swarm on both wires, config 6 host vs gfx950 at 2 and 16 GB), one box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
bash scripts/gpu_r6_check.sh && OUT=gpurun_out/r6_swarm2 bash scripts/gpu_r6_swarm.sh
