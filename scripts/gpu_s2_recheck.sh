#!/bin/bash
# Re-validation after the stream-stager state fix: GPU tier, smoke, headline, configs 3/4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/s2re
mkdir -p $F
export LOG_LEVEL=error
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $F/bench.json 2> $F/bench.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 3 --config 4 > $F/configs34.jsonl 2> $F/configs.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 3 --config 4 >> $F/configs34.jsonl 2>> $F/configs.err
rc=$?
tail -1 $F/pytest_gpu.txt; tail -1 $F/smoke.txt; cat $F/bench.json
python3 -c "
import json
for l in open('$F/configs34.jsonl'):
    j=json.loads(l); print(j['config'], j['MBps'], j['job_s'], j['torrent'].get('staging'), j['torrent']['hash_fails'])
"
exit $rc
