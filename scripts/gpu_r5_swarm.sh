#!/bin/bash
# Round 5: the peer-wire (swarm) path before / after the native wire, one call: config 6
# (4 seeders in their own processes, 2 GB, 4 MiB pieces, loopback) with every connection
# framed in Python (--wire python, round 4's path) or handed to csrc/peerwire.cpp (--wire
# native), 3 alternating pairs; leech CPU is the downloading process' own (RUSAGE_SELF) over
# the transfer.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_swarm2}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
for i in 1 2 3; do
  for w in python native; do
    step "$w $i"
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 6 --wire $w > $F/swarm_${w}_$i.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
    python -c "import json;j=json.loads(open('$F/swarm_${w}_$i.json').read().strip().splitlines()[-1]);print('$w', j['MBps'], 'MB/s', j['leech_cpu_s_per_GB'], 'CPU-s/GB', [(t['name'], round(t['user_s']+t['sys_s'],2)) for t in j['leech_thread_cpu'][:5]], j.get('wire_stats',{}).get('served_bytes'))"
  done
done
