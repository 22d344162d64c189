#!/bin/bash
# Round-2 full re-validation: GPU tier, smoke, headline (+ reference mode in the same call),
# configs 1/3/4/5 tuned and reference (3/4 as 3 reps), peer-wire swarm, TLS (config 2 native
# vs aiohttp, configs 1/3/4 over https), kernel A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_full}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $F/bench_default.json 2> $F/bench.err && \
timeout -k 10 600 python bench.py --compare-reference > $F/bench_vs_reference.json 2>> $F/bench.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 --reps 3 > $F/configs_tuned.jsonl 2> $F/configs.err && \
timeout -k 10 900 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5 --mode reference > $F/configs_ref.jsonl 2>> $F/configs.err && \
timeout -k 10 300 python -m downloader_amd.bench.configs --config 6 > $F/swarm.jsonl 2>> $F/configs.err && \
timeout -k 10 300 python bench.py --tls native > $F/bench_tls_native.json 2>> $F/bench.err && \
timeout -k 10 300 python bench.py --tls aiohttp --steps 2 --warmup 1 --jobs-per-step 32 > $F/bench_tls_aiohttp.json 2>> $F/bench.err && \
timeout -k 10 600 python -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --reps 3 --tls > $F/configs_tls.jsonl 2>> $F/configs.err && \
timeout -k 10 300 python -u -m downloader_amd.bench.verify_bench --kernel-only > $F/kernel.jsonl 2> $F/kernel.err
rc=$?
tail -2 $F/pytest_gpu.txt
cat $F/bench_default.json $F/bench_vs_reference.json $F/bench_tls_native.json $F/bench_tls_aiohttp.json
python3 - <<PY
import json
for f in ("configs_tuned", "configs_ref", "swarm", "configs_tls"):
    try:
        for l in open("$F/" + f + ".jsonl"):
            j = json.loads(l)
            print(f, {k: j.get(k) for k in ("config", "mode", "MBps", "MBps_reps", "p50_latency_s", "p50_s", "jobs_per_s", "worker_cpu_s", "worker_rss_after_MB")})
    except FileNotFoundError:
        pass
PY
exit $rc
