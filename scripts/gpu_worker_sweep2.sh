#!/bin/bash
# Second half of the worker sweep (gpu_worker_sweep.sh): config 2 in reference mode with N
# reference workers (N serial consumers, like N reference containers), and config 5 with an
# offered rate no worker count keeps up with (1000 jobs/s), so its MB/s measures capacity.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/sweep2
mkdir -p $F
export LOG_LEVEL=error
: > $F/config2_ref.jsonl
: > $F/config5_sat.jsonl
for n in 1 2 4 8; do
  timeout -k 10 240 python bench.py --procs-per-rank $n --mode reference --jobs-per-step 8 \
      --steps 4 --warmup 1 >> $F/config2_ref.jsonl 2>> $F/bench.err || exit $?
  echo "config2 ref n=$n done"
done
for n in 1 2 4 8; do
  for m in tuned reference; do
    timeout -k 10 240 python -m downloader_amd.bench.configs --config 5 --workers $n --mode $m \
        --qps 1000 >> $F/config5_sat.jsonl 2>> $F/configs.err || exit $?
    echo "config5 n=$n $m done"
  done
done
cat $F/config2_ref.jsonl $F/config5_sat.jsonl
