#!/bin/bash
# Multipart headline tuning: jobs in flight per worker x worker processes per rank, 100 MB
# objects as 2 x 64 MiB-part uploads, sampled sink check; single-PUT reference once.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_mp_sweep}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
rc=0
for c in 2 4 6 8; do
  for p in 1 2 4; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --concurrency $c --procs-per-rank $p \
      --no-compare-single-put > $F/c${c}_p${p}.json 2>> $F/bench.err || { rc=$?; break 2; }
    echo "c=$c p=$p $(python -c "import json;j=json.load(open('$F/c${c}_p${p}.json'));print(j['value'],j['p50_job_latency_s'],j['worker_cpu_s_per_GB'],j['peer_cpu_s_per_GB'])")"
  done
done
[ $rc -eq 0 ] && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --sink verify \
  --concurrency 4 --no-compare-single-put > $F/verify_c4.json 2>> $F/bench.err
rc=${rc:-$?}
cat $F/verify_c4.json
exit $rc
