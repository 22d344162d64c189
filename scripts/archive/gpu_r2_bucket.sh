#!/bin/bash
# Config 8: bucket:// season (10 x 1 GB episodes + 2 GB extras): stream vs disk vs reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_bucket}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 300 python -m downloader_amd.bench.configs --config 8 > $F/bucket.jsonl 2> $F/bucket.err && \
timeout -k 10 300 python -m downloader_amd.bench.configs --config 8 > $F/bucket2.jsonl 2>> $F/bucket.err && \
timeout -k 10 300 python -m downloader_amd.bench.configs --config 8 --torrent-stream off >> $F/bucket.jsonl 2>> $F/bucket.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 8 --mode reference >> $F/bucket.jsonl 2>> $F/bucket.err
rc=$?
cat $F/bucket.jsonl $F/bucket2.jsonl | cut -c1-330
exit $rc
