#!/bin/bash
# Long soak for leaks: 4 workers, 40 jobs/s for ~5 min, AMQP connection drops every 2 s and
# 1 % S3 503s but no worker kills, so each worker lives the whole run (RSS / fd series).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_soak}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 900 python -m downloader_amd.bench.configs --config 7 --scale 20 --workers 4 --concurrency 4 --qps 40 --chaos-interval 2.0 --no-chaos-kill --s3-fail-rate 0.01 --chaos-timeout 700 > $F/soak.jsonl 2> $F/soak.err
rc=$?
cat $F/soak.jsonl
grep '^\[chaos\]' $F/soak.err | tail -3
exit $rc
