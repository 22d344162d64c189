#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep3.jsonl
: > $OUT
run() {
  echo "== $*" >&2
  timeout -k 10 300 python bench.py --steps 16 --warmup 2 "$@" | tail -1 | python -c "import sys,json; j=json.loads(sys.stdin.read()); j['args']='$*'; print(json.dumps(j))" >> $OUT || exit 1
}
runN() {
  n=$1; shift
  echo "== N=$n $*" >&2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus $n --steps 16 --warmup 2 "$@" 2>gpurun_out/torchrun_err.log | grep '^{' | tail -1 | python -c "import sys,json; j=json.loads(sys.stdin.read()); j['args']='N=$n $*'; print(json.dumps(j))" >> $OUT || exit 1
}
cat /sys/fs/cgroup/cpu.max > gpurun_out/cpu_max.txt 2>&1 || true
run --mode reference --jobs-per-step 2
run --concurrency 4
run --concurrency 8
run --concurrency 8 --sink checksum
run --concurrency 8 --peers shared
runN 2 --concurrency 4
runN 2 --concurrency 8
runN 4 --concurrency 4
python - <<'PY'
import json
for l in open("gpurun_out/sweep3.jsonl"):
    j=json.loads(l); print(f"{j['args']:40s} {j['value']:10.1f} MB/s  p50 {j['p50_job_latency_s']:.4f}s  ms/step {j['ms_per_step']}")
PY
