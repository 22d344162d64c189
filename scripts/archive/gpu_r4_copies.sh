#!/bin/bash
# Round 4: the PartHasher's H2D copies. rocprofv3 kernel + memory-copy trace of config 4 (one
# 20 GB job, GPU relay hashing, 1 GiB part budget) with round 3's stream layout (1 copy + 4
# compute streams = 5 streams on GPU_MAX_HW_QUEUES 4) and the new one (1 copy + 3 compute);
# then alternating A/B of the layouts at the 1 GiB budget (copy-bound: parts wait for their
# DMA holding their buffers), incl. 2 copy + 2 compute.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r4_copies}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd /tmp
for v in "c1x4 --gpu-copy-streams 1 --gpu-compute-streams 4" "c1x3 --gpu-copy-streams 1"; do
  set -- $v; n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $F/rocprof_$n -o c4 -- \
    python3 -m downloader_amd.bench.configs --config 4 --reps 2 --stream-verify gpu --relay-memory-mb 1024 "$@" \
    > $F/prof_$n.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
  K=$(find $F/rocprof_$n -name '*kernel_trace.csv' | head -1)
  M=$(find $F/rocprof_$n -name '*memory_copy_trace.csv' | head -1)
  python3 -m downloader_amd.bench.trace_summary "$K" --copies "$M" --json $F/trace_$n.json > /dev/null
  python3 -c "
import json; j=json.loads(open('$F/prof_$n.json').read().strip().splitlines()[-1]); t=json.load(open('$F/trace_$n.json'))
print('$n', j['MBps_reps'], j['part_pool_peak_MiB'], t.get('memory_copies'), {k: (v['launches'], v['ms_mean'], v['max_concurrent']) for k, v in t.items() if k.startswith('sha1')})"
done
cd $R
for pair in 1 2 3; do
  for v in "c1x4 --gpu-copy-streams 1 --gpu-compute-streams 4" "c1x3 --gpu-copy-streams 1" "c2x2 --gpu-copy-streams 2"; do
    set -- $v; n=$1; shift
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 4 --reps 3 --stream-verify gpu --relay-memory-mb 1024 "$@" > $F/ab_${n}_$pair.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
    python -c "
import json; j=json.loads(open('$F/ab_${n}_$pair.json').read().strip().splitlines()[-1])
print('ab $n $pair', j['MBps_reps'], [r['worker_cpu_s'] for r in j['reps_detail']], j['part_pool_peak_MiB'], j['torrent'].get('gpu_parts'), j.get('gpu_relay', {}).get('device_compute_streams'))"
  done
done
