#!/bin/bash
# Slot pinning check + timed-region length A/B (jobs per step 16 vs 32 vs 64), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/s2ab
mkdir -p $F
export LOG_LEVEL=error
for r in 1 2; do
  for j in 16 32 64; do
    timeout -k 10 300 python bench.py --jobs-per-step $j >> $F/jobs_ab.jsonl 2>> $F/bench.err || exit $?
  done
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --jobs-per-step 64 > $F/bench_n2_j64.json 2>> $F/bench.err
rc=$?
python3 - <<'EOF'
import json
for l in open("gpurun_out/s2ab/jobs_ab.jsonl"):
    j = json.loads(l)
    print(j["config"]["jobs_per_step_per_worker"], j["value"], j["p50_job_latency_s"], j["cpus_per_rank"], j["procs_per_rank"], j["ms_per_step"])
EOF
cat $F/bench_n2_j64.json
exit $rc
