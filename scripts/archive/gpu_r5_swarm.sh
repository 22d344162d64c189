#!/bin/bash
# Round 5: the peer-wire (swarm) path before / after the native wire, one call: config 6
# (4 seeders in their own processes, 2 GB, 4 MiB pieces, loopback) with every connection
# framed in Python (--wire python, round 4's path), handed to csrc/peerwire.cpp with pieces
# SHA-1'd on the host (--swarm-verify cpu) or on the gfx950 PartHasher (--swarm-verify gpu),
# 3 alternating rounds, each process downloading the torrent 3 times (the first is its cold
# one); leech CPU is the downloading process' own over the transfer, with its per-thread
# split (of the last download). GPU tier first (the wire's GPU mode shares the PartHasher).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_swarm5}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
for i in 1 2 3; do
  for v in python cpu gpu; do
    if [ $v = python ]; then a="--wire python"; else a="--wire native --swarm-verify $v"; fi
    step "$v $i"
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 6 --reps 3 $a > $F/swarm_${v}_$i.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
    python -c "import json;j=json.loads(open('$F/swarm_${v}_$i.json').read().strip().splitlines()[-1]);w=j.get('wire_stats',{});print('$v', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB', [(t['name'], round(t['user_s']+t['sys_s'],2)) for t in j['leech_thread_cpu'][:6]], 'gpu', w.get('gpu_pieces'), 'served', w.get('served_bytes'))"
  done
done
