#!/bin/bash
# Round 4: PartHasher slot size x stream layout for two 20 GB jobs at once (4 GiB budget) and
# one job (1 GiB): 2 copy + 2 compute with 1 GiB slots (256 lanes per launch at 4 MiB pieces)
# vs 2 GiB slots (512 lanes) vs 1 copy + 3 compute with 1 GiB slots, alternating, 3 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_slots}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
for r in 1 2 3; do
  for v in "j2_c2s1 --torrent-jobs 2 --relay-memory-mb 4096" "j2_c2s2 --torrent-jobs 2 --relay-memory-mb 4096 --gpu-slot-mb 2048" "j2_c1s1 --torrent-jobs 2 --relay-memory-mb 4096 --gpu-copy-streams 1" "j1_c2s1 --relay-memory-mb 1024" "j1_c2s2 --relay-memory-mb 1024 --gpu-slot-mb 2048"; do
    set -- $v; n=$1; shift
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 4 --reps 3 --stream-verify auto "$@" > $F/${n}_$r.json 2>> $F/err.txt || { tail -20 $F/err.txt; exit 1; }
    python -c "
import json; j=json.loads(open('$F/${n}_$r.json').read().strip().splitlines()[-1])
print('$n $r', j['MBps_reps'], [r['worker_cpu_s'] for r in j['reps_detail']], j['part_pool_peak_MiB'], j.get('gpu_relay', {}).get('device_max_batch_lanes'), j.get('gpu_relay', {}).get('device_launches'))"
  done
done
