#!/bin/bash
# Config 2 (100 MB HTTP blob -> S3) with origin and S3 over TLS: native OpenSSL transport vs
# aiohttp, plus the plain-http headline in the same call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_tls}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 300 python bench.py > $F/bench_plain.json 2> $F/bench.err && \
timeout -k 10 300 python bench.py --tls native > $F/bench_tls_native.json 2>> $F/bench.err && \
timeout -k 10 300 python bench.py --tls aiohttp --steps 2 --warmup 1 --jobs-per-step 32 > $F/bench_tls_aiohttp.json 2>> $F/bench.err && \
timeout -k 10 120 openssl speed -seconds 2 -bytes 16384 -evp aes-128-gcm > $F/openssl_speed.txt 2>&1
rc=$?
cat $F/bench_plain.json $F/bench_tls_native.json $F/bench_tls_aiohttp.json
tail -1 $F/openssl_speed.txt
exit $rc
