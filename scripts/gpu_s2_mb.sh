#!/bin/bash
# After the AVX-512 multi-buffer SHA-1: torrent configs 3/4 (stream relay and disk staging),
# and full-recheck verification host (16 threads) vs gfx950 kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/s2mb
mkdir -p $F
export LOG_LEVEL=error
grep -m1 -o 'avx512[a-z]*' /proc/cpuinfo | head -3 > $F/cpu.txt
C="timeout -k 10 300 python -m downloader_amd.bench.configs"
for r in 1 2; do
  $C --config 3 --config 4 >> $F/stream.jsonl 2>> $F/err.txt || exit $?
done
$C --config 3 --config 4 --torrent-stream off >> $F/disk.jsonl 2>> $F/err.txt || exit $?
timeout -k 10 400 python -m downloader_amd.bench.verify_bench --gib 4 --piece-mb 1 > $F/verify_1m.jsonl 2>> $F/err.txt || exit $?
timeout -k 10 400 python -m downloader_amd.bench.verify_bench --gib 4 --piece-mb 4 > $F/verify_4m.jsonl 2>> $F/err.txt || exit $?
python3 - <<'PY'
import json
for f in ("stream", "disk"):
    for l in open(f"gpurun_out/s2mb/{f}.jsonl"):
        j = json.loads(l)
        t = j["torrent"]
        print(f, j["config"], j["MBps"], j["job_s"], t.get("staging"), "cpu", j["worker_cpu_s"], j["peer_cpu_s"])
PY
cat $F/verify_1m.jsonl $F/verify_4m.jsonl
