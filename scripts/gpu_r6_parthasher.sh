#!/bin/bash
# Round 6: the PartHasher with multi-slot launches (one sha1_lanes kernel spans every HBM slot
# closed while the compute streams were busy). GPU tier, then the streamed-torrent A/B (config
# 4 shape, 20 GB) at host-tail sizes 96 (old default) / 32 / 8, then a rocprofv3 kernel trace of
# one A/B for lanes per launch.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_parthasher}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
step() { echo "== $1 $(date +%T)"; }
summ() {
python3 - "$1" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: j.get(k) for k in ("download", "torrent_gpu_MBps", "torrent_gpu_MBps_runs", "torrent_host_MBps",
      "torrent_host_MBps_runs", "gpu_part_share", "gpu_parts", "gpu_host_fallbacks", "gpu_launches",
      "gpu_lanes_per_launch", "gpu_multi_slot_launches", "gpu_max_launch_lanes",
      "torrent_gpu_worker_cpu_s_per_GB", "torrent_host_worker_cpu_s_per_GB", "torrent_setup_s")})
PY
}
if [[ -z "$SKIP_GPU_TESTS" ]]; then
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
fi
for tail in ${TAILS:-96 32 8}; do
  step "ab tail $tail"
  timeout -k 10 300 python -m downloader_amd.bench.torrent_ab --gb 20 --set stream_gpu_tail=$tail > $F/ab_tail$tail.json 2>> $F/ab.err || { tail -20 $F/ab.err; exit 1; }
  summ $F/ab_tail$tail.json
done
[ -n "$NOPROF" ] && exit 0
step prof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $F/rocprof -o ab -- \
  python3 -m downloader_amd.bench.torrent_ab --gb 20 --pairs 2 ${PROF_SET:+--set $PROF_SET} > $F/prof_ab.json 2>> $F/prof.err || { tail -20 $F/prof.err; exit 1; }
K=$(find $F/rocprof -name '*kernel_trace.csv' | head -1)
M=$(find $F/rocprof -name '*memory_copy_trace.csv' | head -1)
S=$(find $F/rocprof -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && cp "$S" $F/ab_kernel_stats.csv
[ -n "$K" ] && python3 -m downloader_amd.bench.trace_summary "$K" ${M:+--copies "$M"} --json $F/trace_summary.json > /dev/null
python3 -c "import json; t=json.load(open('$F/trace_summary.json')); print({k: v for k, v in t.items()})" | cut -c1-900
rm -rf $F/rocprof
