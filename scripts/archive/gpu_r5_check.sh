#!/bin/bash
# Round 5 check of the tree: GPU tier (incl. swarm pieces on the gfx950 PartHasher), smoke,
# the driver's bench line, then rocprofv3 kernel + memory-copy trace of the bench line's
# same-call torrent A/B (the PartHasher's sha1_lanes launches inside the driver's command).
# NOPROF=1: without the trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r5_check}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
step() { echo "== $1 $(date +%T)"; }
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || { tail -20 $F/smoke.txt; exit 1; }
step bench; timeout -k 10 300 python bench.py > $F/bench.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
python - <<PY
import json
j = json.load(open("$F/bench.json"))
print("bench", j["value"], "p50", j["p50_job_latency_s"], "crc", j.get("crc_relay_MBps"), "util", j["cpu_utilisation"], j.get("crc_relay_cpu_utilisation"))
print("torrent gpu", j.get("torrent_gpu_MBps"), j.get("torrent_gpu_MBps_runs"), "host", j.get("torrent_host_MBps"), j.get("torrent_host_MBps_runs"), "parts", j.get("gpu_parts"), "fallbacks", j.get("gpu_host_fallbacks"))
PY
[ -n "$NOPROF" ] && exit 0
step prof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $F/rocprof -o bench -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-compare-single-put --no-compare-crc --torrent-pairs 2 \
  > $F/prof_bench.json 2>> $F/prof.err || { tail -20 $F/prof.err; exit 1; }
K=$(find $F/rocprof -name '*kernel_trace.csv' | head -1)
M=$(find $F/rocprof -name '*memory_copy_trace.csv' | head -1)
S=$(find $F/rocprof -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && cp "$S" $F/bench_kernel_stats.csv
[ -n "$K" ] && python3 -m downloader_amd.bench.trace_summary "$K" ${M:+--copies "$M"} --json $F/trace_summary.json > /dev/null
python3 -c "import json; t=json.load(open('$F/trace_summary.json')); print({k: v for k, v in t.items()})" | cut -c1-600
