#!/bin/bash
# Config 4 (20 GB, 50 files) with disk staging and every webseed run verified by the gfx950
# SHA-1 kernel (verify_backend=gpu), 3 reps, under rocprofv3 kernel trace + stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
F=gpurun_out/s4_verify_prof
mkdir -p $F
export LOG_LEVEL=error
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $F/rocprof -o run -- python3 -m downloader_amd.bench.configs --config 4 --verify-backend gpu --torrent-stream off --reps 3 > $F/config4_gpu_verify.jsonl 2> $F/run.err
rc=$?
find $F -name "*stats*.csv" | head -5
python3 - <<'PY'
import json
for l in open("gpurun_out/s4_verify_prof/config4_gpu_verify.jsonl"):
    j = json.loads(l); print(j["config"], j["MBps"], j["MBps_reps"], j["torrent"].get("staging"), j["worker_cpu_s"])
PY
exit $rc
