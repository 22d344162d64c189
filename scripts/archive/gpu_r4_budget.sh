#!/bin/bash
# Round 4, VERDICT item 6: GPU relay hashing (stream_verify_backend auto) vs host (cpu) for
# config 4 (20 GB, 50 files, webseed-streamed) under part-buffer budgets of 1 / 2 / 4 GiB per
# worker, one and two jobs at once. Per (budget, jobs): 3 alternating pairs of processes
# (auto, cpu, auto, cpu, ...), each staging the torrent 3 times; the first rep of a process is
# its cold one (HIP init for auto), so the medians use reps 2-3: 6 steady reps per cell.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_budget}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
# resident memory HIP itself adds to a worker: RSS before / after the PartHasher's set-up
timeout -k 10 120 python -c "
import resource
def rss(): return int(open('/proc/self/statm').read().split()[1]) * 4096 >> 20
from downloader_amd.ops import native, gpuhash
native(); a = rss()
g = gpuhash(); b = rss()
ph = g.PartHasher(0, 1 << 30, 16, 4, 16384); c = rss()
native().set_gpu_part_hasher(ph.api(), 8); d = rss()
print({'rss_MiB_modules': a, 'after_import_gpuhash': b, 'after_parthasher': c, 'after_install': d,
       'peak_MiB': resource.getrusage(resource.RUSAGE_SELF).ru_maxrss >> 10})
" > $F/hip_rss.txt 2>&1 || { cat $F/hip_rss.txt; exit 1; }
cat $F/hip_rss.txt
for mb in ${BUDGETS:-1024 2048 4096}; do
  for jobs in 1 2; do
    for pair in 1 2 3; do
      for mode in auto cpu; do
        n=c4_b${mb}_j${jobs}_${mode}_${pair}
        timeout -k 10 300 python -m downloader_amd.bench.configs --config 4 --reps 3 \
          --torrent-jobs $jobs --stream-verify $mode --relay-memory-mb $mb > $F/$n.json 2>> $F/err.txt \
          || { tail -20 $F/err.txt; exit 1; }
        python -c "
import json; j=json.loads(open('$F/$n.json').read().strip().splitlines()[-1])
print('$n', j['MBps_reps'], 'cpu', [r['worker_cpu_s'] for r in j['reps_detail']], 'rss', j['worker_rss_peak_MB'], 'pool_peak', j['part_pool_peak_MiB'], 'gpu_parts', j['torrent'].get('gpu_parts'))"
      done
    done
  done
done
