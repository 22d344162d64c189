#!/bin/bash
# Kernel A/B: SHA-1 block prefetch (load block k+1 while block k is hashed) vs none, plus
# bitop3 vs plain, then the GPU tier (correctness of the rebuilt kernels) and a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_kpf}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 300 python -u -m downloader_amd.bench.verify_bench --kernel-only > $F/kernel.jsonl 2> $F/kernel.err && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_hash.py -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu_hash.txt 2>&1 && \
timeout -k 10 300 python -u -m downloader_amd.bench.verify_bench --gib 2 --repeat 1 > $F/verify.jsonl 2> $F/verify.err
rc=$?
cat $F/kernel.jsonl
tail -2 $F/pytest_gpu_hash.txt
tail -3 $F/verify.jsonl
exit $rc
