#!/bin/bash
# Round 4: (1) the peek-based CRC relay (one copy, one pipe) vs the tee path, alternating,
# with relaybench's floor next to it; (2) what 8 ranks x 2 processes will get from a 64 MiB
# uid pipe budget: the headline at 1 MiB pipes (N=1 today), 256 KiB (the budget math at N=8)
# and 512 KiB with 12 instead of 16 relays per rank (3 jobs per process) - alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_pipes}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
show() { python -c "import json,sys;j=json.load(open('$F/$1.json'));print('$1', j['value'], j.get('crc_relay_MBps'), 'cpu/GB', j['worker_cpu_s_per_GB'], j['peer_cpu_s_per_GB'], j.get('crc_relay_worker_cpu_s_per_GB'), j.get('crc_relay_peer_cpu_s_per_GB'), 'pipe', j['pipe_kb'], 'short', j['pipes_short'])"; }
for i in 1 2 3; do
  for dup in peek tee; do
    STAGER_RELAY_DUP=$dup timeout -k 10 300 python bench.py --no-compare-single-put > $F/crc_${dup}_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
    show crc_${dup}_$i
  done
done
for i in 1 2; do
  for v in "p1024 --pipe-kb 1024" "p256 --pipe-kb 256" "c3p512 --pipe-kb 512 --concurrency 3" "p512 --pipe-kb 512"; do
    set -- $v
    n=$1; shift
    timeout -k 10 300 python bench.py --no-compare-single-put --no-compare-crc "$@" > $F/${n}_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
    show ${n}_$i
  done
done
