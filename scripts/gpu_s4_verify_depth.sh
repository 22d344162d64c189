#!/bin/bash
# Config 4, disk staging, 3 reps each: host SHA-1 vs gfx950 verification at the default and
# a 4x deeper per-stream verify queue (more pieces per dispatch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/s4_verify_depth
mkdir -p $F
export LOG_LEVEL=error
C="python3 -m downloader_amd.bench.configs --config 4 --torrent-stream off --reps 3"
timeout -k 10 300 $C --verify-backend cpu > $F/host.jsonl 2> $F/run.err && \
timeout -k 10 300 $C --verify-backend gpu > $F/gpu_default.jsonl 2>> $F/run.err && \
timeout -k 10 300 $C --verify-backend gpu --webseed-verify-depth-gpu 128 > $F/gpu_depth128.jsonl 2>> $F/run.err
rc=$?
for f in host gpu_default gpu_depth128; do
  [ -f $F/$f.jsonl ] && python3 -c "
import json,sys
for l in open('$F/$f.jsonl'):
    j=json.loads(l); print('$f', j['MBps'], j['MBps_reps'], j['worker_cpu_s'])"
done
exit $rc
