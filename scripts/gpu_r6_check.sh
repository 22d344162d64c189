#!/bin/bash
# Round 6 check of the tree: GPU tier, smoke, the driver's bench line (checked headline +
# same-call extras), the torrent A/B alone at host tails 96 / 48 with the arena-based
# PartHasher, and a rocprofv3 kernel + copy trace of the A/B (lanes per launch, ms per launch).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_check}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
step() { echo "== $1 $(date +%T)"; }
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || { tail -20 $F/smoke.txt; exit 1; }
for i in ${BENCH_RUNS:-1}; do
  step bench$i; s0=$(date +%s)
  timeout -k 10 400 python bench.py > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  echo "wall $(( $(date +%s) - s0 )) s"
  python3 - $F/bench_$i.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ("value", "p50_job_latency_s", "integrity", "crc_parts", "media_parts", "crc_checked_parts", "bad_digests",
        "sink_mismatches", "cpu_utilisation", "procs_per_rank", "unchecked_MBps", "reference_mode_MBps",
        "reference_mode_p50_s", "vs_baseline", "torrent_gpu_MBps", "torrent_host_MBps", "gpu_part_share",
        "gpu_lanes_per_launch", "gpu_multi_slot_launches", "gpu_max_launch_lanes", "torrent_error")
print({k: j.get(k) for k in keys})
print("curve", [(c["procs"], c["MBps"], c["p50_s"]) for c in j.get("workers_curve", [])])
PY
done
if [[ -z "$SKIP_LOWAT" ]]; then
X="--no-compare-unchecked --no-compare-reference --workers-curve= --torrent-gb 0"
for rep in 1 2; do
  for lw in 0 256; do
    step "lowat $lw $rep"
    if [ $lw = 0 ]; then
      timeout -k 10 120 python bench.py $X > $F/lowat${lw}_$rep.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
    else
      STAGER_RCVLOWAT_KB=$lw STAGER_BLOBD_RCVLOWAT_KB=$lw timeout -k 10 120 python bench.py $X > $F/lowat${lw}_$rep.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
    fi
    python3 -c "
import json; j=json.load(open('$F/lowat${lw}_$rep.json'))
print('lowat $lw', j['value'], 'p50', j['p50_job_latency_s'], 'util', j['cpu_utilisation'], 'w', j['worker_cpu_s_per_GB'], 'peer', j['peer_cpu_s_per_GB'], j['worker_breakdown'])"
  done
done
fi
summ() {
python3 - "$1" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: j.get(k) for k in ("download", "torrent_gpu_MBps", "torrent_gpu_MBps_runs", "torrent_host_MBps",
      "torrent_host_MBps_runs", "gpu_part_share", "gpu_launches", "gpu_lanes_per_launch",
      "gpu_multi_slot_launches", "gpu_max_launch_lanes", "torrent_gpu_worker_cpu_s_per_GB",
      "torrent_host_worker_cpu_s_per_GB")})
PY
}
for tail in ${TAILS:-96 48}; do
  step "ab tail $tail"
  timeout -k 10 300 python -m downloader_amd.bench.torrent_ab --gb 20 --set stream_gpu_tail=$tail > $F/ab_tail$tail.json 2>> $F/ab.err || { tail -20 $F/ab.err; exit 1; }
  summ $F/ab_tail$tail.json
done
[ -n "$NOPROF" ] && exit 0
step prof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $F/rocprof -o ab -- \
  python3 -m downloader_amd.bench.torrent_ab --gb 20 --pairs 2 > $F/prof_ab.json 2>> $F/prof.err || { tail -20 $F/prof.err; exit 1; }
K=$(find $F/rocprof -name '*kernel_trace.csv' | head -1)
M=$(find $F/rocprof -name '*memory_copy_trace.csv' | head -1)
S=$(find $F/rocprof -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && cp "$S" $F/ab_kernel_stats.csv
[ -n "$K" ] && python3 -m downloader_amd.bench.trace_summary "$K" ${M:+--copies "$M"} --json $F/trace_summary.json > /dev/null
python3 -c "import json; t=json.load(open('$F/trace_summary.json')); print({k: v for k, v in t.items()})" | cut -c1-900
rm -rf $F/rocprof
