#!/bin/bash
# Probe: per-user limits and how many processes / threads one bench rank runs at its peak
# (the 8-rank scaling launch runs eight of these side by side).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/probe_tasks}
mkdir -p $F
export LOG_LEVEL=error PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
ulimit -a > $F/ulimit.txt
timeout -k 10 200 python bench.py --no-compare-crc --no-compare-single-put --steps 40 > $F/bench.json 2>> $F/err.txt &
B=$!
max_p=0; max_t=0
for i in $(seq 1 30); do
  sleep 1
  p=$(ps -u $(id -u) -o pid= | wc -l)
  t=$(ps -u $(id -u) -L -o lwp= | wc -l)
  [ $p -gt $max_p ] && max_p=$p
  [ $t -gt $max_t ] && max_t=$t
  kill -0 $B 2>/dev/null || break
done
wait $B
echo "max processes $max_p max threads $max_t" | tee $F/tasks.txt
grep -E "processes|locked|open files" $F/ulimit.txt
