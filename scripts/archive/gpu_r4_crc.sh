#!/bin/bash
# Round 4: where the CRC'd relay's CPU goes. relaybench (csrc/relaybench.cpp) isolates the
# per-byte cost of splice / tee+read / +CRC / peek+CRC / recv+send+CRC on the box's EPYC at
# 1 and 8 relay threads; then the driver's bench line twice (headline, one PUT, CRC'd relay
# with worker and peer CPU per GB) and once with 256 KiB pipes (what 8 ranks of 2 processes
# get from a 64 MiB pipe budget).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_crc}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
lscpu > $F/lscpu.txt 2>&1
for t in 1 8; do
  for m in splice tee teecrc peekcrc copycrc; do
    timeout -k 5 120 taskset -c 0-15 ./downloader_amd/bin/relaybench --mode $m --gb 8 --threads $t >> $F/relaybench.jsonl || exit 1
  done
done
cat $F/relaybench.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench.py > $F/bench_$i.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
  python -c "import json;j=json.load(open('$F/bench_$i.json'));print('bench', j['value'], j['integrity'], j['single_put_MBps'], j['crc_relay_MBps'], 'cpu/GB', j['worker_cpu_s_per_GB'], j['peer_cpu_s_per_GB'], j['crc_relay_worker_cpu_s_per_GB'], j['crc_relay_peer_cpu_s_per_GB'], 'slots', j['gpu_slots'], j['slot_budget_cpus'], j['pipe_budget_bytes'])"
done
timeout -k 10 300 python bench.py --pipe-kb 256 > $F/bench_pipe256.json 2>> $F/bench.err || { tail -20 $F/bench.err; exit 1; }
python -c "import json;j=json.load(open('$F/bench_pipe256.json'));print('pipe256', j['value'], j['crc_relay_MBps'], j['pipes_short'])"
