#!/bin/bash
# Round-3: the tee()d user-space relays (one copy: splice the pages on, read a duplicate for
# CRC / piece SHA-1) vs recv + send (STAGER_RELAY_TEE=0), same call: configs 3/4 (hashed
# torrent relay, 3 reps each, twice), the headline with --checksum always, and config 4 with
# the pieces hashed on the GPU on top of the tee path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_tee}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
summ() { python -c "import json,sys
for l in open(sys.argv[1]):
  j=json.loads(l); print(sys.argv[1].split('/')[-1], {k:j.get(k) for k in sys.argv[2].split(',')})" "$@"; }
for round in 1 2; do
  for tee in 1 0; do
    STAGER_RELAY_TEE=$tee timeout -k 10 400 python -m downloader_amd.bench.configs --config 3 --config 4 --reps 3 > $F/c34_tee${tee}_${round}.jsonl 2>> $F/err.txt || exit 1
    summ $F/c34_tee${tee}_${round}.jsonl config,MBps_reps,worker_cpu_s,peer_cpu_s
  done
done
for tee in 1 0; do
  STAGER_RELAY_TEE=$tee timeout -k 10 200 python bench.py --checksum always --no-compare-single-put > $F/c2_always_tee${tee}.json 2>> $F/err.txt || exit 1
  summ $F/c2_always_tee${tee}.json value,p50_job_latency_s,worker_cpu_s_per_GB,peer_cpu_s_per_GB,sink_mismatches
done
timeout -k 10 400 python -m downloader_amd.bench.configs --config 4 --reps 3 --stream-verify gpu --stream-gpu-pending 160 > $F/c4_gpu_tee1.jsonl 2>> $F/err.txt || exit 1
summ $F/c4_gpu_tee1.jsonl config,MBps_reps,worker_cpu_s,peer_cpu_s,gpu_relay
