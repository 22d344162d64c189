#!/bin/bash
# Round 4: does anything accumulate across back-to-back bench runs (the driver runs N=1,2,4,8
# back to back)? The driver's bench line 5 times in a row with the host state in between:
# sockets (TIME_WAIT), /dev/shm and /tmp usage, free memory, pipe-using processes left.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_repeat}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
state() { echo "-- $1: $(ss -s | grep -E '^TCP:' ) | shm $(du -sm /dev/shm 2>/dev/null | cut -f1) MB | tmp $(du -sm /tmp 2>/dev/null | cut -f1) MB | $(grep -E 'MemAvailable' /proc/meminfo) | my procs $(ps -u $(id -u) --no-headers | wc -l)"; }
state start
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-compare-single-put --no-compare-crc > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python -c "import json;j=json.load(open('$F/bench_$i.json'));print('bench $i', j['value'], j['p50_job_latency_s'], j['worker_cpu_s_per_GB'], j['peer_cpu_s_per_GB'], j['event_loop_busy'])"
  state after_$i
done
