#!/bin/bash
# Round 5: rocprofv3 kernel + memory-copy trace of config 6 with every swarm piece SHA-1'd on
# the gfx950 PartHasher (4 GB, seeders on the leecher's event loop: no child processes under
# the profiler), to see why the device path runs below the host one.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r5_swarmprof}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $F/rocprof -o swarm -- \
  python3 -m downloader_amd.bench.configs --config 6 --reps 2 --scale 2 --swarm-verify gpu --seed-inproc \
  > $F/swarm_gpu.json 2>> $F/prof.err || { tail -20 $F/prof.err; exit 1; }
K=$(find $F/rocprof -name '*kernel_trace.csv' | head -1)
M=$(find $F/rocprof -name '*memory_copy_trace.csv' | head -1)
S=$(find $F/rocprof -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && cp "$S" $F/kernel_stats.csv
[ -n "$K" ] && python3 -m downloader_amd.bench.trace_summary "$K" ${M:+--copies "$M"} --json $F/trace_summary.json > /dev/null
python3 -c "import json; t=json.load(open('$F/trace_summary.json')); print(t)" | cut -c1-1500
python3 -c "import json; j=json.loads(open('$F/swarm_gpu.json').read().strip().splitlines()[-1]); print(j['MBps_reps'], j['leech_cpu_s_per_GB_reps'], j['wire_stats'])"
