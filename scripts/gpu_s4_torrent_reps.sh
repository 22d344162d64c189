#!/bin/bash
# Configs 3/4 (4 GB / 20 GB webseed torrents) staged 5x each on one setup, tuned vs
# reference-equivalent mode: median + per-rep MB/s instead of one sub-second sample.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/s4_reps}
mkdir -p $F
export LOG_LEVEL=error
timeout -k 10 600 python -m downloader_amd.bench.configs --config 3 --config 4 --reps 5 > $F/configs34_tuned.jsonl 2> $F/configs.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 3 --config 4 --reps 3 --mode reference > $F/configs34_ref.jsonl 2>> $F/configs.err
rc=$?
python3 - <<'PY'
import json, os
out = os.environ.get("OUT", "gpurun_out/s4_reps")
for f in ("configs34_tuned", "configs34_ref"):
    try:
        for l in open(f"{out}/{f}.jsonl"):
            j = json.loads(l); print(f, j["config"], j["MBps"], j["MBps_reps"], j["worker_cpu_s"], j["peer_cpu_s"])
    except FileNotFoundError:
        pass
PY
exit $rc
