#!/bin/bash
# Round 5: the driver's multi-rank launch on the 1-GPU box, now that the bench line ends with
# the torrent GPU vs host A/B: 2 ranks (torch.distributed.run, gloo, 8 CPUs each) both with a
# PartHasher on the one device, each rank its own blobd peers; then the driver's exact N=1
# command. A launch-path check, not a scaling number (the ranks share one GPU slot's CPUs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r5_ranks}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
step() { echo "== $1 $(date +%T)"; }
step n2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 > $F/bench_n2.json 2> $F/n2.err || { tail -30 $F/n2.err; exit 1; }
python -c "import json;j=json.loads(open('$F/bench_n2.json').read().strip().splitlines()[-1]);print('n2', j['value'], j['n_gpus'], j['rank_cpus'], 'crc', j.get('crc_relay_MBps'), 'torrent', j.get('torrent_gpu_MBps'), j.get('torrent_host_MBps'), j.get('torrent_ranks'), 'parts', j.get('gpu_parts'), 'fallbacks', j.get('gpu_host_fallbacks'))"
step n1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench_n1.json 2> $F/n1.err || { tail -30 $F/n1.err; exit 1; }
python -c "import json;j=json.loads(open('$F/bench_n1.json').read().strip().splitlines()[-1]);print('n1', j['value'], 'crc', j.get('crc_relay_MBps'), 'torrent', j.get('torrent_gpu_MBps'), j.get('torrent_host_MBps'))"
