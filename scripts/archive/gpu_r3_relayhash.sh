#!/bin/bash
# Streamed-torrent piece hashing: host multi-buffer SHA-1 vs the gfx950 PartHasher.
# GPU tests of the part hasher, then configs 3 (4 GB) and 4 (20 GB, 50 files) x 3 reps each:
# cpu / gpu (64 parts pending) / gpu (160 pending), the job's tail on the host, alternated
# over 2 rounds in one call; then a rocprofv3 kernel trace of a config-4 gpu job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r3_relayhash}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 120 python -c "from downloader_amd.ops import hashing; print('gpu relay hashing:', hashing.gpu_relay_hashing(8))" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_hash.py -x -v --timeout 120 --timeout-method thread \
  -k "part_hasher or gpu_relay" > $F/pytest_parthasher.txt 2>&1 || { tail -30 $F/pytest_parthasher.txt; exit 1; }
tail -1 $F/pytest_parthasher.txt
for round in 1 2; do
  for v in cpu gpu64 gpu160; do
    case $v in
      cpu) args="--stream-verify cpu" ;;
      gpu64) args="--stream-verify gpu --stream-gpu-pending 64" ;;
      gpu160) args="--stream-verify gpu --stream-gpu-pending 160" ;;
    esac
    timeout -k 10 400 python -m downloader_amd.bench.configs --config 3 --config 4 --reps 3 \
      $args > $F/c34_${v}_${round}.jsonl 2>> $F/configs.err || { echo "FAIL $v $round"; tail -20 $F/configs.err; exit 1; }
    python - "$F/c34_${v}_${round}.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    j = json.loads(l)
    g = j.get("gpu_relay", {})
    print(sys.argv[1].split("/")[-1], "config", j["config"], "MBps", j["MBps_reps"], "cpu",
          [r["worker_cpu_s"] for r in j["reps_detail"]], "peer",
          [r["peer_cpu_s"] for r in j["reps_detail"]],
          "gpu_parts", g.get("submitted"), "launches", g.get("device_launches"),
          "max_lanes", g.get("device_max_batch_lanes"))
PY
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$F/rocprof -o c4 -- \
  python -m downloader_amd.bench.configs --config 4 --stream-verify gpu --stream-gpu-pending 160 > $GRAFT_REPO_ROOT/$F/c4_rocprof.jsonl 2>> $GRAFT_REPO_ROOT/$F/configs.err
