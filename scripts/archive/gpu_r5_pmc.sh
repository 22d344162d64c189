#!/bin/bash
# Round 5: PMC pass (its own run, counters only) over the PartHasher's sha1_lanes on the
# round's last tree - config 4, one job, GPU hashing, 2 GiB budget; 5 SQ + 1 GRBM counters
# fit one pass. Then the summary (VALU instructions per 64-byte block, VALU issue share).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=$R/gpurun_out/${OUT_NAME:-r5_pmc}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=$R
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $F/pmc -o pmc -- python3 -m downloader_amd.bench.configs --config 4 --reps 1 --stream-verify gpu --relay-memory-mb 2048 > $F/pmc_c4.json 2> $F/pmc.err || { tail -20 $F/pmc.err; exit 1; }
P=$(find $F/pmc -name '*counter_collection.csv' | head -1)
[ -n "$P" ] && python3 -m downloader_amd.bench.pmc_summary "$P" 4194304 > $F/pmc_summary.json && cat $F/pmc_summary.json
