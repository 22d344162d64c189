#!/bin/bash
# Where does a torrent job's time go? Config 3/4 with per-phase timers, staging on the
# default tmp dir vs tmpfs, plus the GPU test tier.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export LOG_LEVEL=error
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1 || { tail -20 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
O=gpurun_out/tb.jsonl; : > $O
s() { echo "== $*" >&2; timeout -k 10 600 python -m downloader_amd.bench.configs "$@" >> $O 2>> gpurun_out/tb.err || exit 1; }
s --config 3
s --config 3 --stage-dir /dev/shm
s --config 4
s --config 4 --stage-dir /dev/shm
df -hT /tmp /dev/shm >> gpurun_out/tb.err 2>&1
cat $O
