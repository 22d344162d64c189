#!/bin/bash
# Round 6 closing validation, one box: GPU tier, smoke, the driver's exact bench command twice,
# the 2-rank launch (torch.distributed.run, both ranks on the one device, 8 CPUs each), a
# rocprofv3 kernel + memory-copy trace of the bench line (its torrent A/B's sha1_lanes launches)
# and a counters-only PMC pass over the PartHasher's kernel. PART=a: up to the ranks; b: traces.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_final}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
step() { echo "== $1 $(date +%T)"; }
summ() {
python3 - "$1" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ("n_gpus", "value", "p50_job_latency_s", "integrity", "crc_parts", "media_parts", "crc_checked_parts",
        "bad_digests", "sink_mismatches", "cpu_utilisation", "procs_per_rank", "unchecked_MBps",
        "reference_mode_MBps", "reference_mode_p50_s", "vs_baseline", "config1_p50_s", "config1_reference_p50_s",
        "torrent_gpu_MBps", "torrent_host_MBps", "gpu_part_share", "gpu_lanes_per_launch",
        "gpu_multi_slot_launches", "gpu_max_launch_lanes", "torrent_ranks", "torrent_error")
print({k: j.get(k) for k in keys})
print("curve", [(c["procs"], c["MBps"], c["p50_s"]) for c in j.get("workers_curve", [])])
print("torrent breakdown gpu", j.get("torrent_gpu_breakdown"), "host", j.get("torrent_host_breakdown"))
PY
}
PART=${PART:-ab}
if [[ $PART == *a* ]]; then
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || { tail -20 $F/smoke.txt; exit 1; }
for i in 1 2; do
  step bench$i; s0=$(date +%s)
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  echo "wall $(( $(date +%s) - s0 )) s"; summ $F/bench_$i.json
done
step n2; s0=$(date +%s)
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 > $F/bench_n2.json 2> $F/n2.err || { tail -30 $F/n2.err; exit 1; }
echo "wall $(( $(date +%s) - s0 )) s"; summ $F/bench_n2.json
fi
if [[ $PART == *b* ]]; then
step prof
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $F/rocprof -o bench -- \
  python3 $R/bench.py --steps 5 --warmup 2 > $F/prof_bench.json 2>> $F/prof.err || { tail -20 $F/prof.err; exit 1; }
K=$(find $F/rocprof -name '*kernel_trace.csv' | head -1)
M=$(find $F/rocprof -name '*memory_copy_trace.csv' | head -1)
S=$(find $F/rocprof -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && cp "$S" $F/bench_kernel_stats.csv
[ -n "$K" ] && python3 -m downloader_amd.bench.trace_summary "$K" ${M:+--copies "$M"} --json $F/trace_summary.json > /dev/null
python3 -c "import json; t=json.load(open('$F/trace_summary.json')); print({k: v for k, v in t.items()})" | cut -c1-900
rm -rf $F/rocprof
step pmc
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $F/pmc -o pmc -- python3 -m downloader_amd.bench.torrent_ab --gb 20 --pairs 1 > $F/pmc_ab.json 2> $F/pmc.err || { tail -20 $F/pmc.err; exit 1; }
P=$(find $F/pmc -name '*counter_collection.csv' | head -1)
[ -n "$P" ] && python3 -m downloader_amd.bench.pmc_summary "$P" 4194304 > $F/pmc_summary.json && cat $F/pmc_summary.json
rm -rf $F/pmc/*/*.csv 2>/dev/null; true
fi
