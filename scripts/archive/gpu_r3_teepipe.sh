#!/bin/bash
# Round-3: size of the tee() duplicate pipe (main/4 = 256 KiB vs 1 MiB) for the CRC'd plain
# relay (headline --checksum always) and the hashed torrent relay (config 4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_teepipe}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
summ() { python -c "import json,sys
for l in open(sys.argv[1]):
  j=json.loads(l); print(sys.argv[1].split('/')[-1], {k:j.get(k) for k in sys.argv[2].split(',')})" "$@"; }
for round in 1 2; do
  for kb in 256 1024; do
    STAGER_TEE_PIPE_KB=$kb timeout -k 10 200 python bench.py --checksum always --no-compare-single-put > $F/c2_always_tee${kb}_${round}.json 2>> $F/err.txt || exit 1
    summ $F/c2_always_tee${kb}_${round}.json value,worker_cpu_s_per_GB,peer_cpu_s_per_GB,pipes_short
    STAGER_TEE_PIPE_KB=$kb timeout -k 10 300 python -m downloader_amd.bench.configs --config 4 --reps 3 > $F/c4_tee${kb}_${round}.jsonl 2>> $F/err.txt || exit 1
    summ $F/c4_tee${kb}_${round}.jsonl MBps_reps,worker_cpu_s,peer_cpu_s
  done
done
