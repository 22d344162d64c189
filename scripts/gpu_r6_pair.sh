#!/bin/bash
# Round 6: sha1_lanes_split with two blocks per barrier (sha1_lanes_split_pair) vs one, kernel
# bench in one process (digests checked against sha1_lanes<16> on lanes of varied lengths).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_pair}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
timeout -k 10 300 python -u - > $F/pair_ab.jsonl 2>> $F/pair.err <<'PY' || { tail -20 $F/pair.err; exit 1; }
import json
from downloader_amd.ops import gpuhash
gv = gpuhash().GpuVerifier(0, 64 << 20, 8)
for plen, lanes in ((65536 + 48, 200), (4 << 20, 16), (4 << 20, 64), (4 << 20, 1024), (1 << 20, 4096)):
    for rep in range(2):
        for pair in (False, True):
            s, l, same = gv.kernel_bench_split(plen, lanes, 2, True, pair)
            print(json.dumps({"piece_len": plen, "lanes": lanes, "pair": pair, "rep": rep, "ms_split": round(s, 2),
                              "ms_lanes": round(l, 2), "same": same}), flush=True)
PY
cat $F/pair_ab.jsonl
