#!/bin/bash
# PMC counters of the SHA-1 kernels (prefetch / no prefetch, bitop3 / plain) in one pass:
# 5 SQ + 1 GRBM counters, within one pass's limits. Kernel trace and stats in a second run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/r2_pmc}
mkdir -p $F
export TMPDIR=/tmp LOG_LEVEL=error
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $F/pmc -o pmc -- python3 -m downloader_amd.bench.verify_bench --kernel-only --kernel-sizes 1024 --kernel-counts 4096,16384 > $F/pmc.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $F/trace -o trace -- python3 -m downloader_amd.bench.verify_bench --kernel-only > $F/trace.log 2>&1
rc=$?
P=$(find $F/pmc -name '*counter_collection.csv' | head -1)
[ -n "$P" ] && python -m downloader_amd.bench.pmc_summary "$P" 1048576 > $F/pmc_summary.json
S=$(find $F/trace -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && cp "$S" $F/kernel_stats.csv
cat $F/pmc_summary.json 2>/dev/null
exit $rc
