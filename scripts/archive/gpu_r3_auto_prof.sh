#!/bin/bash
# Round-3: rocprofv3 kernel trace of config 4 with two jobs at once in stream_verify auto
# (the gfx950 sha1_lanes launches on the streamed-torrent hot path).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r3_auto_prof}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $F/rocprof -o c4 -- \
  python3 -m downloader_amd.bench.configs --config 4 --reps 2 --torrent-jobs 2 --stream-verify auto \
  > $F/c4.json 2> $F/err.txt || exit 1
python3 -c "
import json; j=json.loads(open('$F/c4.json').read().strip().splitlines()[-1])
print(j['MBps_reps'], j['torrent'].get('gpu_parts'), j.get('gpu_relay'))"
find $F/rocprof -name '*kernel_stats.csv' -exec cat {} \;
