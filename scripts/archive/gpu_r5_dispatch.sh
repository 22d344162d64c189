#!/bin/bash
# Round 5: the PartHasher now runs the shared PartDispatcher state machine (part_dispatch.h)
# over HipPartDevice. GPU tier (digests vs hashlib through the relay, faults, HBM release),
# smoke, then the driver's bench line (incl. the 20 GB torrent GPU vs host A/B) twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_dispatch}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 || { tail -20 $F/smoke.txt; exit 1; }
for i in 1 2; do
  step bench$i; timeout -k 10 300 python bench.py > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python - <<PY
import json
j = json.load(open("$F/bench_$i.json"))
print("bench", j["value"], "crc", j.get("crc_relay_MBps"), "util", j["cpu_utilisation"], j.get("crc_relay_cpu_utilisation"))
print("torrent gpu", j.get("torrent_gpu_MBps"), j.get("torrent_gpu_MBps_runs"), "host", j.get("torrent_host_MBps"), j.get("torrent_host_MBps_runs"),
      "parts", j.get("gpu_parts"), "fallbacks", j.get("gpu_host_fallbacks"), "lanes/launch", j.get("gpu_lanes_per_launch"))
PY
done
