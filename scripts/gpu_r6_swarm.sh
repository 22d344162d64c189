#!/bin/bash
# Round 6 swarm call: the heterogeneous swarm (48 swarmd seeders,
# 0.2 - 50 MB/s, 20 - 200 ms, 10 % stalling, 10 % hanging up; 2 GB, 4 MiB pieces) on both wires,
# then config 6 (4 fast loopback seeders) on the epoll wire: host vs gfx950 SHA-1 at 2 GB and
# 16 GB (the small-torrent GPU tail, item 6).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r6_swarm}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
if [[ -z "$SKIP_HETERO" ]]; then
step hetero
timeout -k 10 500 python -m downloader_amd.bench.swarm_hetero --gb 2 --peers 48 --reps ${HREPS:-3} > $F/hetero.jsonl 2>> $F/hetero.err || { tail -20 $F/hetero.err; exit 1; }
python3 - <<PY
import json
for l in open("$F/hetero.jsonl"):
    j = json.loads(l)
    print(j["wire"], j["rep"], "MB/s", j["MBps"], "offered", j["offered_MBps"], "share", j["of_offered"], "idle", j["max_owned_idle_s"], "slow", j["slow_peers"], "threads", j["threads_before"], j["threads_peak"], "endgame", j["endgame_pieces"])
PY
fi
for sc in ${SCALES:-1 8}; do
  for v in ${VERIFY:-cpu gpu}; do
    step "config6 $v x$sc"
    timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --reps 3 --scale $sc --swarm-verify $v > $F/swarm_${v}_x${sc}.json 2>> $F/swarm.err || { tail -20 $F/swarm.err; exit 1; }
    python -c "import json;j=json.loads(open('$F/swarm_${v}_x${sc}.json').read().strip().splitlines()[-1]);w=j.get('wire_stats',{});print('$v x$sc', j['MBps_reps'], 'MB/s', j['leech_cpu_s_per_GB_reps'], 'CPU-s/GB', 'io threads', w.get('io_threads'), 'gpu', w.get('gpu_pieces'), 'overflow', w.get('gpu_overflow'))"
  done
done
