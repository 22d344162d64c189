#!/bin/bash
# Round-1 close: BASELINE configs 1/3/4/5 tuned and reference-equivalent on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/close_configs
mkdir -p $F
export LOG_LEVEL=error
timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 > $F/configs.jsonl 2> $F/configs.err && \
timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 --mode reference > $F/configs_ref.jsonl 2>> $F/configs.err
rc=$?
python3 - <<'PY'
import json
for f in ("configs", "configs_ref"):
    try:
        for l in open(f"gpurun_out/close_configs/{f}.jsonl"):
            j = json.loads(l); print(f, {k: j[k] for k in list(j)[:9]})
    except FileNotFoundError:
        pass
PY
exit $rc
