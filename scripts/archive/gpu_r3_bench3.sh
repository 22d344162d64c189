#!/bin/bash
# Round-3: the driver's default bench (three same-call measurements: multipart headline, one
# PUT per object, CRC32C on every relayed PUT/part) with its wall time, after the GPU tier.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_bench3}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || exit 1
tail -1 $F/pytest_gpu.txt
for i in 1 2; do
  s=$(date +%s.%N)
  timeout -k 10 300 python bench.py > $F/bench_$i.json 2>> $F/bench.err || exit 1
  e=$(date +%s.%N)
  python -c "import json;j=json.loads(open('$F/bench_$i.json').read().strip().splitlines()[-1]);print('wall', round($e-$s,1), {k:j.get(k) for k in ('value','p50_job_latency_s','single_put_MBps','crc_relay_MBps','crc_relay_p50_s','crc_relay_worker_cpu_s_per_GB','crc_relay_sink_checked_puts','worker_cpu_s_per_GB','worker_kernel_share','peer_cpu_s_per_GB')})"
done
