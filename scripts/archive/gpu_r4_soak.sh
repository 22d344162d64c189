#!/bin/bash
# Round 4: memory over time under the part budget - one worker stages the 20 GB torrent
# (config 4, GPU relay hashing) 12 times back to back with two jobs at once, at a 2 GiB budget;
# RSS and the pool's leased + idle bytes after every rep must level off, not grow.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_soak}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 900 python -m downloader_amd.bench.configs --config 4 --reps 12 --torrent-jobs 2 \
  --stream-verify auto --relay-memory-mb 2048 > $F/c4_soak.json 2> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
python -c "
import json; j=json.loads(open('$F/c4_soak.json').read().strip().splitlines()[-1])
print('GB/s', j['MBps_reps']); print('rss', [r['rss_MB'] for r in j['reps_detail']]); print('pool', [r['pool_MiB'] for r in j['reps_detail']])
print('peak', j['worker_rss_peak_MB'], j['part_pool_peak_MiB'], j['relay_pool_after'])"
