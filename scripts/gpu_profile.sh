#!/bin/bash
# Kernel PMC counters + verify bench reader sweep + bench CPU accounting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp LOG_LEVEL=error
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc -o pmc -- python -m downloader_amd.bench.verify_bench --kernel-only > gpurun_out/pmc.log 2>&1 && \
timeout -k 10 600 python -m downloader_amd.bench.verify_bench --gib 4 --piece-mb 1 --readers 16 --repeat 2 > gpurun_out/verify_r16.jsonl 2>&1 && \
timeout -k 10 600 python -m downloader_amd.bench.verify_bench --gib 4 --piece-mb 4 --readers 12 --repeat 2 > gpurun_out/verify_p4_r12.jsonl 2>&1 && \
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --compare-reference > gpurun_out/bench_cpu.json 2>gpurun_out/bench_cpu.err
echo "exit $?"
