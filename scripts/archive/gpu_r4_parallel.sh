#!/bin/bash
# Round 4: parts in flight per streamed-torrent job (download.torrent_stream_parallel, 16 since
# round 2's config-4 sweep on host hashing) re-checked on today's paths: config 3 (4 GB, host
# multi-buffer SHA-1) and config 4 (20 GB, GPU PartHasher), 16 / 32 alternating, 3 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_parallel}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
for r in 1 2 3; do
  for c in 3 4; do
    for p in 16 32; do
      n=c${c}_p${p}_$r
      timeout -k 10 300 python -m downloader_amd.bench.configs --config $c --reps 3 --stream-parallel $p > $F/$n.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
      python -c "
import json; j=json.loads(open('$F/$n.json').read().strip().splitlines()[-1])
print('$n', j['MBps_reps'], [r['worker_cpu_s'] for r in j['reps_detail']], j.get('part_pool_peak_MiB'), j['worker_rss_peak_MB'])"
    done
  done
done
