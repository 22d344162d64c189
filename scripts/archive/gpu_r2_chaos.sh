#!/bin/bash
# Config 7 chaos soak on the box: supervised workers over AMQP, SIGKILLs + connection drops.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_chaos}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 600 python -m downloader_amd.bench.configs --config 7 --scale 2 --workers 4 --concurrency 4 --qps 40 --chaos-interval 1.0 --s3-fail-rate 0.03 --chaos-timeout 400 > $F/chaos.jsonl 2> $F/chaos.err
rc=$?
cat $F/chaos.jsonl
grep -c '"level":50' $F/chaos.err || true
exit $rc
