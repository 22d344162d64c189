#!/bin/bash
# Probe: configs 1/3/4 in ONE process (as gpu_r3_full.sh runs them) with stream_verify auto
# (default) vs cpu, alternating, to see whether auto loses in a long-lived process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/probe_auto_multi}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD} STAGER_THREAD_CPU=1
for v in default cpu default cpu; do
  a=""; [ $v = cpu ] && a="--stream-verify cpu"
  timeout -k 10 400 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --reps 3 $a > $F/c134_$v.jsonl 2>> $F/err.txt || exit 1
  python -c "
import json
for l in open('$F/c134_$v.jsonl'):
    j=json.loads(l)
    if j.get('config') == 4:
        print('$v', j['MBps_reps'], [r['worker_cpu_s'] for r in j['reps_detail']], [r['peer_cpu_s'] for r in j['reps_detail']], j['torrent'].get('gpu_parts'), j.get('thread_cpu', [])[:4])"
done
