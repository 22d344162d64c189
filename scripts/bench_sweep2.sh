#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep2.jsonl
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
run --concurrency 6
run --concurrency 8
run --concurrency 12
run --concurrency 8 --part-mb 32
run --concurrency 12 --part-mb 32
run --concurrency 16 --part-mb 32
runN 2 --concurrency 8 --part-mb 32
runN 4 --concurrency 8 --part-mb 32
python - <<'PY'
import json
for l in open("gpurun_out/sweep2.jsonl"):
    j=json.loads(l); print(f"{j['args']:40s} {j['value']:10.1f} MB/s  p50 {j['p50_job_latency_s']:.4f}s  ms/step {j['ms_per_step']}")
PY
