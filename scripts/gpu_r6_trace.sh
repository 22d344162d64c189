#!/bin/bash
# Round 6: where the PartHasher's launches lose time in the torrent A/B - the kernel bench on
# this box, then a rocprofv3 kernel + copy trace of one A/B pair, raw kernel rows kept.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_trace}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
timeout -k 10 120 python -u -c "
from downloader_amd.ops import gpuhash
gv = gpuhash().GpuVerifier(0, 64 << 20, 8)
print('kernel bench 4 MiB x 512:', gv.kernel_bench_split(4 << 20, 512, 2))" > $F/kbench.txt 2>&1 || { cat $F/kbench.txt; exit 1; }
cat $F/kbench.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $F/rocprof -o ab -- \
  python3 -m downloader_amd.bench.torrent_ab --gb 20 --pairs ${PAIRS:-1} > $F/prof_ab.json 2>> $F/prof.err || { tail -20 $F/prof.err; exit 1; }
K=$(find $F/rocprof -name '*kernel_trace.csv' | head -1)
M=$(find $F/rocprof -name '*memory_copy_trace.csv' | head -1)
[ -n "$K" ] && cp "$K" $F/kernel_trace.csv && python3 -m downloader_amd.bench.trace_summary "$K" ${M:+--copies "$M"} --json $F/trace_summary.json > /dev/null
[ -n "$M" ] && cp "$M" $F/memory_copy_trace.csv
python3 -c "import json; t=json.load(open('$F/trace_summary.json')); print({k: v for k, v in t.items()})" | cut -c1-900
rm -rf $F/rocprof
