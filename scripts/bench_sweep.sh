#!/bin/bash
# Single-worker parameter sweep of bench.py on the GPU box (CPU/NIC-path knobs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep.jsonl
: > $OUT
run() {
  echo "== $*" >&2
  timeout -k 10 240 python bench.py --steps 8 --warmup 1 "$@" | tail -1 | python -c "import sys,json; j=json.loads(sys.stdin.read()); j['args']='$*'; print(json.dumps(j))" >> $OUT || exit 1
}
for a in "${@}"; do :; done
run --mode reference --jobs-per-step 2
run --staging disk --concurrency 4
run --staging disk --concurrency 6
run --staging stream --concurrency 2
run --staging stream --concurrency 4
run --staging stream --concurrency 8
run --staging stream --concurrency 4 --inflight-parts 16
run --staging stream --concurrency 4 --part-mb 32
run --staging stream --concurrency 4 --part-mb 8
python - <<'PY'
import json
for l in open("gpurun_out/sweep.jsonl"):
    j=json.loads(l); print(f"{j['args']:55s} {j['value']:10.1f} MB/s  p50 {j['p50_job_latency_s']:.4f}s  ms/step {j['ms_per_step']}")
PY
