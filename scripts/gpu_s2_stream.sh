#!/bin/bash
# Torrent configs 3/4: stream staging (webseed -> S3 relay, in-flight SHA-1) vs disk staging,
# A/B in one call; then a parallelism sweep for the stream path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/s2stream
mkdir -p $F
export LOG_LEVEL=error
C="timeout -k 10 300 python -m downloader_amd.bench.configs"
for r in 1 2; do
  $C --config 3 --config 4 >> $F/stream.jsonl 2>> $F/err.txt || exit $?
  $C --config 3 --config 4 --torrent-stream off >> $F/disk.jsonl 2>> $F/err.txt || exit $?
done
for p in 8 32; do
  $C --config 3 --config 4 --stream-parallel $p | sed "s/^{/{\"stream_parallel\": $p, /" >> $F/sweep.jsonl 2>> $F/err.txt || exit $?
done
python3 - <<'PY'
import json
for f in ("stream", "disk", "sweep"):
    for l in open(f"gpurun_out/s2stream/{f}.jsonl"):
        j = json.loads(l)
        t = j["torrent"]
        print(f, j.get("stream_parallel", ""), j["config"], j["MBps"], j["job_s"], t.get("staging"),
              "fetch_s", t["webseed_fetch_s"], "hash_fails", t["hash_fails"],
              "cpu", j["worker_cpu_s"], j["peer_cpu_s"])
PY
