#!/bin/bash
# Round-3 A/Bs in one call: payload integrity (CRC32C) on vs off for configs 2/3/4, the
# reference-mode ratio, and config 5's healthy-job latency under retry backoff 0.5 vs 5 s
# with the broker-held (queue) vs in-consumer (sleep) delay.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_ab}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
summ() { python -c "import json,sys
for l in open(sys.argv[1]):
  j=json.loads(l); print(sys.argv[1].split('/')[-1], {k:j.get(k) for k in sys.argv[2].split(',')})" "$@"; }
for round in 1 2; do
  for ck in auto always; do
    timeout -k 10 200 python bench.py --checksum $ck --no-compare-single-put > $F/c2_${ck}_${round}.json 2>> $F/err.txt || exit 1
    summ $F/c2_${ck}_${round}.json value,p50_job_latency_s,worker_cpu_s_per_GB,peer_cpu_s_per_GB
  done
done
timeout -k 10 300 python bench.py --mode reference --steps 2 --warmup 1 --no-compare-single-put > $F/c2_reference.json 2>> $F/err.txt || exit 1
summ $F/c2_reference.json value,p50_job_latency_s
for ck in off auto; do
  timeout -k 10 400 python -m downloader_amd.bench.configs --config 3 --config 4 --reps 3 --checksum $ck > $F/c34_${ck}.jsonl 2>> $F/err.txt || exit 1
  summ $F/c34_${ck}.jsonl config,MBps_reps,worker_cpu_s,peer_cpu_s
done
for delay in queue sleep; do
  for b in 0.5 5; do
    timeout -k 10 300 python -m downloader_amd.bench.configs --config 5 --retry-backoff-s $b --retry-delay $delay > $F/c5_${delay}_${b}.json 2>> $F/err.txt || exit 1
    summ $F/c5_${delay}_${b}.json retry_delay,retry_backoff_s,healthy_p50_s,healthy_p99_s,p99_latency_s,jobs_per_s
  done
done
