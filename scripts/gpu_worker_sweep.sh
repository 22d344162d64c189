#!/bin/bash
# BASELINE.md's results table: MB/s and p50 job latency at 1/2/4/8 worker processes, tuned vs
# reference-equivalent mode, on one GPU slot's host share (16 CPUs on the build box).
#   config 2 (headline): bench.py with --procs-per-rank N (N worker processes, one rank)
#   config 5 (mixed queue, fixed QPS, retry path): configs.py --workers N
# Configs 1/3/4 are single-job configs (one worker does all the work): see configs.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/sweep
mkdir -p $F
export LOG_LEVEL=error
: > $F/config2.jsonl
: > $F/config5.jsonl
for n in 1 2 4 8; do
  timeout -k 10 240 python bench.py --procs-per-rank $n >> $F/config2.jsonl 2>> $F/bench.err || exit $?
  timeout -k 10 240 python bench.py --procs-per-rank $n --mode reference --jobs-per-step 8 \
      --steps 4 --warmup 1 >> $F/config2.jsonl 2>> $F/bench.err || exit $?
  echo "config2 n=$n done"
done
for n in 1 2 4 8; do
  for m in tuned reference; do
    timeout -k 10 240 python -m downloader_amd.bench.configs --config 5 --workers $n --mode $m \
        >> $F/config5.jsonl 2>> $F/configs.err || exit $?
    echo "config5 n=$n $m done"
  done
done
cat $F/config2.jsonl $F/config5.jsonl
