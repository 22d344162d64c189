#!/bin/bash
# Round 6: the heterogeneous swarm (48 swarmd seeders, 2 GB) on both wires, 3 seeds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_hetero4}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
timeout -k 10 700 python -m downloader_amd.bench.swarm_hetero --gb 2 --peers 48 --reps ${REPS:-3} > $F/hetero.jsonl 2> $F/hetero.err || { tail -20 $F/hetero.err; exit 1; }
python3 - "$F/hetero.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    j = json.loads(l)
    print(j["wire"], j["rep"], j["s"], j["MBps"], j["offered_MBps"], j["of_offered"], j.get("of_offered_incl_partial"),
          j["max_owned_idle_s"], j["threads_peak"] - j["threads_before"], j["endgame_pieces"])
PY
