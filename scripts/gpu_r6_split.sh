#!/bin/bash
# Round 6: the split-wave PartHasher kernel (sha1_lanes_split: a schedule wave and a rounds wave
# per 64 pieces) against sha1_lanes<16> - kernel A/B, GPU tier, torrent A/B (config 4) with
# either kernel and shorter host tails, config 6 at 2 / 16 GB on the device, and a kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_split}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
step() { echo "== $1 $(date +%T)"; }
step new-tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_hash.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "split or kernels_match" > $F/pytest_split.txt 2>&1 || { tail -30 $F/pytest_split.txt; exit 1; }
tail -1 $F/pytest_split.txt
step kernel-ab
timeout -k 10 300 python -u - > $F/kernel_ab.jsonl 2>> $F/kernel.err <<'PY' || { tail -20 $F/kernel.err; exit 1; }
import json
from downloader_amd.ops import gpuhash
gv = gpuhash().GpuVerifier(0, 64 << 20, 8)
for plen in (4 << 20, 1 << 20):
    for lanes in (64, 256, 1024):
        s, l, same = gv.kernel_bench_split(plen, lanes, 3)
        print(json.dumps({"piece_len": plen, "lanes": lanes, "ms_split": round(s, 2), "ms_lanes": round(l, 2),
                          "speedup": round(l / s, 3), "same": same,
                          "split_MBps_per_lane": round(plen / s / 1e3, 1)}), flush=True)
PY
cat $F/kernel_ab.jsonl
step gpu-tier
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
ab() {   # name, env..., -- torrent_ab args
  local name=$1; shift
  step "ab $name"
  env "$@" timeout -k 10 300 python -m downloader_amd.bench.torrent_ab --gb 20 --pairs 3 ${ABSET} > $F/ab_$name.json 2>> $F/ab.err || { tail -20 $F/ab.err; return 1; }
  python3 -c "import json;j=json.loads(open('$F/ab_$name.json').read().strip().splitlines()[-1]);print('$name', {k: j.get(k) for k in ('torrent_gpu_MBps','torrent_host_MBps','gpu_part_share','gpu_lanes_per_launch','torrent_gpu_MBps_runs','torrent_host_MBps_runs','torrent_gpu_worker_cpu_s_per_GB','torrent_host_worker_cpu_s_per_GB')})"
}
ab split_t96 STAGER_SHA1_KERNEL=split || exit 1
ab lanes_t96 STAGER_SHA1_KERNEL=lanes || exit 1
ABSET="--set stream_gpu_tail=64" ab split_t64 STAGER_SHA1_KERNEL=split || exit 1
ABSET="--set stream_gpu_tail=48" ab split_t48 STAGER_SHA1_KERNEL=split || exit 1
for sc in 1 8; do
  for k in split lanes; do
    [[ $sc == 8 && $k == lanes ]] && continue
    step "config6 gpu $k x$sc"
    STAGER_SHA1_KERNEL=$k timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --reps 3 --scale $sc --swarm-verify gpu > $F/swarm_gpu_${k}_x${sc}.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
    python -c "import json;j=json.loads(open('$F/swarm_gpu_${k}_x${sc}.json').read().strip().splitlines()[-1]);print('$k x$sc', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB')"
  done
  step "config6 cpu x$sc"
  timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --reps 3 --scale $sc --swarm-verify cpu > $F/swarm_cpu_x${sc}.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
  python -c "import json;j=json.loads(open('$F/swarm_cpu_x${sc}.json').read().strip().splitlines()[-1]);print('cpu x$sc', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB')"
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
python3 -c "import json; t=json.load(open('$F/trace_summary.json')); print({k: v for k, v in t.items()})" | cut -c1-900
rm -rf $F/rocprof
