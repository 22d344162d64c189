#!/bin/bash
# Round 6: smoke() and a 2-rank bench line (the driver's launch) on the round's last tree.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r6_ntsmoke}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $F/smoke.txt 2>&1 || { tail -20 $F/smoke.txt; exit 1; }
tail -2 $F/smoke.txt
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $F/bench_n2.json 2> $F/bench_n2.err || { tail -20 $F/bench_n2.err; exit 1; }
python3 -c "import json;j=json.loads(open('$F/bench_n2.json').read().strip().splitlines()[-1]);print({k: j.get(k) for k in ('value','n_gpus','vs_baseline','torrent_gpu_MBps','torrent_host_MBps','gpu_part_share')})"
