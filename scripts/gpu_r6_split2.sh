#!/bin/bash
# Round 6: sha1_lanes_split with one workgroup per CU - split tests, torrent A/B alternating the
# split and the old kernel twice each, a kernel trace of the A/B, config 6 at 2 GB (device vs
# host, twice), and the driver's bench line.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_split2}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_hash.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "split or kernels_match or part_hasher" > $F/pytest_split.txt 2>&1 || { tail -30 $F/pytest_split.txt; exit 1; }
tail -1 $F/pytest_split.txt
ab() {
  local name=$1; shift
  step "ab $name"
  env "$@" timeout -k 10 300 python -m downloader_amd.bench.torrent_ab --gb 20 --pairs 3 > $F/ab_$name.json 2>> $F/ab.err || { tail -20 $F/ab.err; return 1; }
  python3 -c "import json;j=json.loads(open('$F/ab_$name.json').read().strip().splitlines()[-1]);print('$name', {k: j.get(k) for k in ('torrent_gpu_MBps','torrent_host_MBps','gpu_part_share','gpu_lanes_per_launch','torrent_gpu_MBps_runs','torrent_host_MBps_runs','torrent_gpu_worker_cpu_s_per_GB','torrent_host_worker_cpu_s_per_GB')})"
}
ab split_1 STAGER_SHA1_KERNEL=split && ab lanes_1 STAGER_SHA1_KERNEL=lanes && ab split_2 STAGER_SHA1_KERNEL=split && ab lanes_2 STAGER_SHA1_KERNEL=lanes || exit 1
for r in 1 2; do
  for v in gpu cpu; do
    step "config6 $v $r"
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 6 --reps 3 --scale 1 --swarm-verify $v > $F/swarm_${v}_$r.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
    python -c "import json;j=json.loads(open('$F/swarm_${v}_$r.json').read().strip().splitlines()[-1]);print('$v', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB')"
  done
done
step prof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $F/rocprof -o ab -- \
  python3 -m downloader_amd.bench.torrent_ab --gb 20 --pairs 1 > $F/prof_ab.json 2>> $F/prof.err || { tail -20 $F/prof.err; exit 1; }
K=$(find $F/rocprof -name '*kernel_trace.csv' | head -1)
M=$(find $F/rocprof -name '*memory_copy_trace.csv' | head -1)
S=$(find $F/rocprof -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && cp "$S" $F/ab_kernel_stats.csv
[ -n "$K" ] && python3 -m downloader_amd.bench.trace_summary "$K" ${M:+--copies "$M"} --json $F/trace_summary.json > /dev/null
python3 -c "import json; t=json.load(open('$F/trace_summary.json')); print({k: v for k, v in t.items()})" | cut -c1-700
rm -rf $F/rocprof
cd $R
step bench
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench_1.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
python3 -c "import json;j=json.loads(open('$F/bench_1.json').read().strip().splitlines()[-1]);print({k: j.get(k) for k in ('value','vs_baseline','p50_job_latency_s','unchecked_MBps','torrent_gpu_MBps','torrent_host_MBps','gpu_part_share','gpu_lanes_per_launch')})"
