#!/bin/bash
# Round 4: rocprofv3 kernel + memory-copy trace of the shipping PartHasher layout (2 copy + 2
# compute streams, 16 x 1 GiB slots) - config 4 with one job at a 1 GiB part budget and with
# two jobs at a 2 GiB budget: launches, lanes per launch, kernel time, copies.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r4_prof22}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd /tmp
for v in "j1 --relay-memory-mb 1024" "j2 --torrent-jobs 2 --relay-memory-mb 2048"; do
  set -- $v; n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $F/rocprof_$n -o c4 -- \
    python3 -m downloader_amd.bench.configs --config 4 --reps 2 --stream-verify gpu "$@" \
    > $F/prof_$n.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
  K=$(find $F/rocprof_$n -name '*kernel_trace.csv' | head -1)
  M=$(find $F/rocprof_$n -name '*memory_copy_trace.csv' | head -1)
  S=$(find $F/rocprof_$n -name '*kernel_stats.csv' | head -1)
  [ -n "$S" ] && cp "$S" $F/${n}_kernel_stats.csv
  python3 -m downloader_amd.bench.trace_summary "$K" --copies "$M" --json $F/trace_$n.json > /dev/null
  python3 -c "
import json; j=json.loads(open('$F/prof_$n.json').read().strip().splitlines()[-1]); t=json.load(open('$F/trace_$n.json'))
print('$n', j['MBps_reps'], j['part_pool_peak_MiB'], t.get('memory_copies'), {k: v for k, v in t.items() if k.startswith('sha1')})"
done
