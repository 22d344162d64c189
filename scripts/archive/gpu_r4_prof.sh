#!/bin/bash
# Round 4: rocprofv3 kernel trace of config 4 (two 20 GB jobs at once, GPU relay hashing,
# 2 GiB part budget): sha1_lanes launches, lanes (= grid threads) per launch, overlap.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r4_prof}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $F/rocprof -o c4 -- \
  python3 -m downloader_amd.bench.configs --config 4 --reps 2 --torrent-jobs 2 --stream-verify auto \
  --relay-memory-mb 2048 > $F/c4.json 2> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
python3 -c "
import json; j=json.loads(open('$F/c4.json').read().strip().splitlines()[-1])
print(j['MBps_reps'], j['torrent'].get('gpu_parts'), j['part_pool_peak_MiB'], j.get('gpu_relay'))"
T=$(find $F/rocprof -name '*kernel_trace.csv' | head -1)
python3 -m downloader_amd.bench.trace_summary "$T" --json $F/trace_summary.json
