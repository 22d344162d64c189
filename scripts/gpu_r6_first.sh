#!/bin/bash
# Round 6, first box call: GPU tier, then the driver's bench line (now: CRC32C on every part as
# the headline, unchecked / reference-mode / 1-2-4-8 worker curve / torrent A/B as same-call
# extras) twice, timed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r6_first}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
summ() {
python3 - "$1" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ("value", "p50_job_latency_s", "integrity", "crc_parts", "media_parts", "crc_checked_parts",
        "bad_digests", "sink_mismatches", "cpu_utilisation", "worker_cpu_s_per_GB", "peer_cpu_s_per_GB",
        "unchecked_MBps", "unchecked_worker_cpu_s_per_GB", "unchecked_peer_cpu_s_per_GB",
        "reference_mode_MBps", "reference_mode_p50_s", "vs_baseline", "torrent_gpu_MBps",
        "torrent_host_MBps", "gpu_parts", "gpu_lanes_per_launch", "torrent_setup_s", "torrent_error")
print({k: j.get(k) for k in keys})
print("curve", [(c["procs"], c["MBps"], c["p50_s"]) for c in j.get("workers_curve", [])])
print("breakdown", j.get("worker_breakdown"))
PY
}
if [[ -z "$SKIP_GPU_TESTS" ]]; then
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
fi
for i in 1 2; do
  step bench$i; s0=$(date +%s.%N)
  timeout -k 10 400 python bench.py > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  echo "wall $(python3 -c "print(round($(date +%s.%N) - $s0, 1))") s"
  summ $F/bench_$i.json
done
