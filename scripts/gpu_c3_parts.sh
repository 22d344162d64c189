#!/bin/bash
# Config 3 (4 GB single-file webseed torrent, stream staging): parts in flight x part size,
# interleaved A/B in one call (box-to-box variance is larger than the effects).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/c3parts
mkdir -p $F
export LOG_LEVEL=error
: > $F/c3.jsonl
for rep in 1 2; do
  for v in 16:64 16:32 24:32 32:32 24:64 32:64 32:16; do
    p=${v%%:*}; m=${v##*:}
    timeout -k 10 120 python -m downloader_amd.bench.configs --config 3 --stream-parallel $p \
        --part-mb $m > $F/one.json 2>> $F/err.txt || exit $?
    python -c "import json,sys; d=json.load(open('$F/one.json')); d['parallel']=$p; d['part_mb']=$m; print(json.dumps(d))" >> $F/c3.jsonl
    echo "rep $rep p=$p part=$m done"
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/c3parts/c3.jsonl"):
    d = json.loads(l)
    print(d["parallel"], d["part_mb"], d["MBps"], d["worker_cpu_s"], d["peer_cpu_s"])
PY
