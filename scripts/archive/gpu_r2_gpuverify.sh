#!/bin/bash
# Torrent disk staging (webseed runs written to disk, pieces verified as runs land) with the
# gfx950 kernel vs host multi-buffer SHA-1, plus a kernel trace of the GPU run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_gpuverify}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 400 python -m downloader_amd.bench.configs --config 3 --config 4 --torrent-stream off --verify-backend gpu --reps 2 > $F/disk_gpu.jsonl 2> $F/err.txt && \
timeout -k 10 400 python -m downloader_amd.bench.configs --config 3 --config 4 --torrent-stream off --verify-backend cpu --reps 2 > $F/disk_cpu.jsonl 2>> $F/err.txt && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $F/trace -o trace -- python3 -m downloader_amd.bench.configs --config 3 --scale 0.5 --torrent-stream off --verify-backend gpu > $F/traced.jsonl 2>> $F/err.txt
rc=$?
S=$(find $F/trace -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && cp "$S" $F/kernel_stats.csv && rm -rf $F/trace
python3 - <<PY
import json
for f in ("disk_gpu", "disk_cpu", "traced"):
    try:
        for l in open("$F/" + f + ".jsonl"):
            j = json.loads(l); t = j.get("torrent", {})
            print(f, j["config"], j["MBps"], j.get("MBps_reps"), "cpu", j["worker_cpu_s"], "verify_s", t.get("webseed_verify_s"))
    except FileNotFoundError:
        pass
PY
cat $F/kernel_stats.csv 2>/dev/null | cut -c1-160
exit $rc
