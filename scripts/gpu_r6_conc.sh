#!/bin/bash
# Round 6: sha1_lanes_split alone vs two launches side by side on two streams (the PartHasher's
# compute streams), beside H2D part copies, and after idle gaps; 4 MiB pieces.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_conc}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
timeout -k 10 300 python -u - > $F/concurrent.jsonl 2>> $F/conc.err <<'PY' || { tail -20 $F/conc.err; exit 1; }
import json
from downloader_amd.ops import gpuhash
gv = gpuhash().GpuVerifier(0, 64 << 20, 8)
for lanes in (1, 8, 16, 32, 48, 64, 80):
    for dup in (False, True):
        sp, ln, same = gv.kernel_bench_split(4 << 20, lanes, 3, dup)
        print(json.dumps({"lanes": lanes, "dup": dup, "ms_split": round(sp, 2), "ms_lanes": round(ln, 2),
                          "same": same}), flush=True)
PY
cat $F/concurrent.jsonl
