#!/bin/bash
# Round 5: config 6 as the reference's whole magnet job (--swarm-job): a worker takes a
# v1.download whose magnet names the 4 seeders, fetches the metadata from them, downloads
# the swarm on the native wire and stages the file to the S3 sink (eager staging while the
# swarm runs), done marker, v1.convert. 2 GB and 16 GB, host SHA-1 vs `auto` (the gfx950 from
# 8 GiB); 3 jobs per worker, the first its cold one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_swarmjob}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
for sc in 1 8; do
  for i in 1 2; do
    for v in cpu auto; do
      step "$v x$sc $i"
      timeout -k 10 400 python -m downloader_amd.bench.configs --config 6 --swarm-job --reps 3 --scale $sc --swarm-verify $v > $F/job_${v}_x${sc}_$i.json 2>> $F/job.err || { tail -20 $F/job.err; exit 1; }
      python -c "import json;j=json.loads(open('$F/job_${v}_x${sc}_$i.json').read().strip().splitlines()[-1]);print('$v x$sc', j['MBps_reps'], 'MB/s', j['worker_cpu_s_per_GB_reps'], 'CPU-s/GB', j['stage_s'], 'eager', j['eager_upload_s'], 's3', j['s3_bytes_received'])"
    done
  done
done
