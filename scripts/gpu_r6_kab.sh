#!/bin/bash
# Round 6: kernel-only A/B of sha1_lanes_split vs sha1_lanes<16> (device-resident lanes), with
# then the split kernel's GPU tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_kab}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
echo "== kernel-ab $(date +%T)"
timeout -k 10 300 python -u - > $F/kernel_ab.jsonl 2>> $F/kernel.err <<'PY' || { tail -20 $F/kernel.err; exit 1; }
import json
from downloader_amd.ops import gpuhash
gv = gpuhash().GpuVerifier(0, 64 << 20, 8)
for plen, lanes in ((65536 + 48, 200), (4 << 20, 64), (4 << 20, 1024)):
    for rep in (0, 1):
        s, l, same = gv.kernel_bench_split(plen, lanes, 2)
        print(json.dumps({"piece_len": plen, "lanes": lanes, "rep": rep, "ms_split": round(s, 2),
                          "ms_lanes": round(l, 2), "speedup": round(l / s, 3), "same": same}), flush=True)
PY
cat $F/kernel_ab.jsonl
echo "== tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_hash.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "split or kernels_match or part_hasher" > $F/pytest_split.txt 2>&1 || { tail -30 $F/pytest_split.txt; exit 1; }
tail -1 $F/pytest_split.txt
