#!/bin/bash
# Round 5, first call on the new tree: GPU tier, then the driver's bench line twice (timed-window
# CPU accounting, native relay breakdown, the same-call 20 GB torrent GPU vs host A/B), then
# relaybench's splice / peek+CRC floor at 8 relay threads on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_first}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
step gpu; timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 || { tail -30 $F/pytest_gpu.txt; exit 1; }
tail -1 $F/pytest_gpu.txt
for i in 1 2; do
  step bench$i; timeout -k 10 300 python bench.py > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python - <<PY
import json
j = json.load(open("$F/bench_$i.json"))
print("bench", j["value"], "crc", j.get("crc_relay_MBps"), "util", j["cpu_utilisation"], j.get("crc_relay_cpu_utilisation"),
      "cpu/GB", j["worker_cpu_s_per_GB"], j["peer_cpu_s_per_GB"], j.get("crc_relay_worker_cpu_s_per_GB"), j.get("crc_relay_peer_cpu_s_per_GB"))
print("breakdown", j["worker_breakdown"], j.get("crc_relay_worker_breakdown"))
print("torrent gpu", j.get("torrent_gpu_MBps"), j.get("torrent_gpu_MBps_runs"), "host", j.get("torrent_host_MBps"), j.get("torrent_host_MBps_runs"),
      "parts", j.get("gpu_parts"), "fallbacks", j.get("gpu_host_fallbacks"), "lanes/launch", j.get("gpu_lanes_per_launch"), "setup", j.get("torrent_setup_s"))
PY
done
for m in splice peekcrc; do
  timeout -k 5 120 taskset -c 0-15 ./downloader_amd/bin/relaybench --mode $m --gb 8 --threads 8 >> $F/relaybench.jsonl || exit 1
done
cat $F/relaybench.jsonl
