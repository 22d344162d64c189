#!/bin/bash
# Torrent configs 3/4: job dir on the container overlay (default temp dir) vs tmpfs (/dev/shm).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/s2fs
mkdir -p $F /dev/shm/stage-ab
export LOG_LEVEL=error
df -h /tmp /dev/shm > $F/df.txt; mount | grep -E ' / | /tmp | /dev/shm ' >> $F/df.txt
for r in 1 2; do
  timeout -k 10 300 python -m downloader_amd.bench.configs --config 3 --config 4 >> $F/overlay.jsonl 2>> $F/err.txt || exit $?
  timeout -k 10 300 python -m downloader_amd.bench.configs --config 3 --config 4 --stage-dir /dev/shm/stage-ab >> $F/tmpfs.jsonl 2>> $F/err.txt || exit $?
done
rm -rf /dev/shm/stage-ab
python3 - <<'EOF'
import json
for f in ("overlay", "tmpfs"):
    for l in open(f"gpurun_out/s2fs/{f}.jsonl"):
        j = json.loads(l)
        t = j["torrent"]
        print(f, j["config"], j["MBps"], j["job_s"], "fetch", t["webseed_fetch_s"], "verify", t["webseed_verify_s"], "eager", j["eager_upload_s"], "cleanup", j["cleanup_after_job_s"])
EOF
cat $F/df.txt
