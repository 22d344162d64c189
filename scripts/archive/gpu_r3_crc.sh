#!/bin/bash
# Round-3 re-measure after the AVX-512 VPCLMULQDQ CRC32C: the integrity tests on the box's
# CPU (EPYC, VPCLMULQDQ path), the headline with CRC32C on the plain relay (always) vs the
# default (auto: spliced, no CRC), and configs 3/4 with CRC32C off vs auto.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_crc}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
summ() { python -c "import json,sys
for l in open(sys.argv[1]):
  j=json.loads(l); print(sys.argv[1].split('/')[-1], {k:j.get(k) for k in sys.argv[2].split(',')})" "$@"; }
timeout -k 10 300 python -u -m pytest tests/test_integrity.py -x -q --timeout 120 > $F/pytest_integrity.txt 2>&1 || exit 1
tail -1 $F/pytest_integrity.txt
python -c "from downloader_amd.ops import native; import time, os
n = native(); b = os.urandom(256 << 20); n.crc32c(b, 0); t = time.perf_counter()
for _ in range(8): n.crc32c(b, 0)
print('crc32c GB/s per core', round(8 * len(b) / (time.perf_counter() - t) / 1e9, 1))" | tee $F/crc_rate.txt
for round in 1 2; do
  for ck in auto always; do
    timeout -k 10 200 python bench.py --checksum $ck --no-compare-single-put > $F/c2_${ck}_${round}.json 2>> $F/err.txt || exit 1
    summ $F/c2_${ck}_${round}.json value,p50_job_latency_s,worker_cpu_s_per_GB,peer_cpu_s_per_GB
  done
done
for ck in off auto; do
  timeout -k 10 400 python -m downloader_amd.bench.configs --config 3 --config 4 --reps 3 --checksum $ck > $F/c34_${ck}.jsonl 2>> $F/err.txt || exit 1
  summ $F/c34_${ck}.jsonl config,MBps_reps,worker_cpu_s,peer_cpu_s
done
