set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
nproc > gpurun_out/env.txt; free -g >> gpurun_out/env.txt; df -h /tmp /dev/shm . >> gpurun_out/env.txt; lscpu | head -20 >> gpurun_out/env.txt
timeout -k 10 300 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --compare-reference > gpurun_out/bench1.log 2>&1
echo "exit $?"
