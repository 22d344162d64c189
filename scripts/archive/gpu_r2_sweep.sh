#!/bin/bash
# Round-2 worker sweep (BASELINE.md's table: MB/s and p50 at 1/2/4/8 worker processes,
# tuned vs reference-equivalent mode, one GPU slot's 16 CPUs):
#   config 2: bench.py --procs-per-rank N (reference: N serial consumers)
#   config 5: 1000 mixed jobs offered at 1000 jobs/s (capacity), --workers N
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_sweep}
mkdir -p $F
export LOG_LEVEL=error
: > $F/config2.jsonl
: > $F/config5_sat.jsonl
for n in 1 2 4 8; do
  timeout -k 10 240 python bench.py --procs-per-rank $n >> $F/config2.jsonl 2>> $F/bench.err || exit $?
  timeout -k 10 240 python bench.py --procs-per-rank $n --mode reference --jobs-per-step 8 \
      --steps 4 --warmup 1 >> $F/config2.jsonl 2>> $F/bench.err || exit $?
  echo "config2 n=$n done"
done
for n in 1 2 4 8; do
  for m in tuned reference; do
    timeout -k 10 240 python -m downloader_amd.bench.configs --config 5 --workers $n --mode $m \
        --qps 1000 >> $F/config5_sat.jsonl 2>> $F/configs.err || exit $?
    echo "config5 n=$n $m done"
  done
done
python3 - <<PY
import json
for l in open("$F/config2.jsonl"):
    j = json.loads(l)
    print("c2", j["mode"], j["procs_per_rank"], j["value"], j["p50_job_latency_s"])
for l in open("$F/config5_sat.jsonl"):
    j = json.loads(l)
    print("c5", j.get("mode"), j.get("workers"), j.get("jobs_per_s"), j.get("MBps"), j.get("p50_latency_s"))
PY
