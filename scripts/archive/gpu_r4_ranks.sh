#!/bin/bash
# Round 4: the driver's multi-rank launch on the 1-GPU box (2 ranks share its 16 CPUs: a
# check of the launch path - pinning, per-rank peers, relay_plan - not a scaling number),
# then the driver's exact N=1 BENCH command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_ranks}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 > $F/bench_n2.json 2> $F/bench_n2.err || { tail -20 $F/bench_n2.err; exit 1; }
python -c "import json;j=json.loads(open('$F/bench_n2.json').read().strip().splitlines()[-1]);print('n2', j['value'], j['n_gpus'], j['rank_cpus'], j['rank_peers'], j['pipe_kb'], j['concurrency_per_worker'], j['sink_mismatches'])"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench_n1.json 2> $F/bench_n1.err || { tail -20 $F/bench_n1.err; exit 1; }
python -c "import json;j=json.load(open('$F/bench_n1.json'));print('n1', j['value'], j['integrity'], j['crc_relay_MBps'], j['single_put_MBps'])"
