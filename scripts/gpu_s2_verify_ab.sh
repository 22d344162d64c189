#!/bin/bash
# Disk-staged torrent config 4 (20 GB, incremental webseed verification): host multi-buffer
# SHA-1 vs GPU batcher, A/B in one call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/s2vab
mkdir -p $F
export LOG_LEVEL=error
C="timeout -k 10 300 python -m downloader_amd.bench.configs --torrent-stream off"
for r in 1 2; do
  $C --config 3 --config 4 --verify-backend cpu >> $F/cpu.jsonl 2>> $F/err.txt || exit $?
  $C --config 3 --config 4 --verify-backend gpu >> $F/gpu.jsonl 2>> $F/err.txt || exit $?
done
python3 - <<'PY'
import json
for f in ("cpu", "gpu"):
    for l in open(f"gpurun_out/s2vab/{f}.jsonl"):
        j = json.loads(l)
        print(f, j["config"], j["MBps"], j["job_s"], "cpu", j["worker_cpu_s"], j["peer_cpu_s"])
PY
