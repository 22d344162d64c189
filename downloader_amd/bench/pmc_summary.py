"""Summarise a rocprofv3 ``--pmc`` CSV of the SHA-1 kernels (``scripts/archive/gpu_r2_pmc.sh``).

Groups dispatches by kernel (template arguments kept, so the prefetch / bitop3 variants stay
apart) and grid size, and derives per-wave VALU instruction counts and the fraction of wave
cycles with a VALU instruction issuing - the issue-bound check behind docs/PERFORMANCE.md.

    python -m downloader_amd.bench.pmc_summary <pmc_counter_collection.csv> [piece_len]
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict


def summarise(path: str, piece_len: int = 0):
    acc = defaultdict(lambda: defaultdict(float))
    meta = {}
    dispatches = defaultdict(set)
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if "sha1" not in name:
                continue
            short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            key = (short, int(row["Grid_Size"]))
            acc[key][row["Counter_Name"]] += float(row["Counter_Value"])
            dispatches[key].add(row["Dispatch_Id"])
            meta[key] = int(row["VGPR_Count"])
    out = []
    for key in sorted(acc):
        c = acc[key]
        waves = c.get("SQ_WAVES", 0.0)
        row = {"kernel": key[0], "lanes": key[1], "dispatches": len(dispatches[key]),
               "VGPR_Count": meta[key]}
        if waves:
            row["valu_insts_per_wave"] = round(c.get("SQ_INSTS_VALU", 0.0) / waves, 1)
            if piece_len:
                row["valu_insts_per_64B_block"] = round(row["valu_insts_per_wave"]
                                                        / (piece_len / 64), 1)
                if "split" in key[0]:
                    # three waves (two schedule producers, one rounds consumer) per 64 pieces:
                    # the per-wave figure is their average; per 64 pieces it is their sum
                    row["valu_insts_per_64B_block_per_64_pieces"] = round(
                        3 * row["valu_insts_per_64B_block"], 1)
        if c.get("SQ_WAVE_CYCLES"):
            # SQ_ACTIVE_INST_VALU and SQ_WAVE_CYCLES are both per-wave cycle sums (quad-cycle
            # granularity on CDNA), so their ratio is the fraction of a wave's life spent issuing
            row["valu_active_frac_of_wave_cycles"] = round(
                c.get("SQ_ACTIVE_INST_VALU", 0.0) / c["SQ_WAVE_CYCLES"], 3)
        out.append(row)
    # one row per kernel over every grid size (the relay's launches vary in lanes)
    names = sorted({k[0] for k in acc})
    for n in names:
        keys = [k for k in acc if k[0] == n]
        if len(keys) < 2:
            continue
        tot = defaultdict(float)
        for k in keys:
            for cname, v in acc[k].items():
                tot[cname] += v
        row = {"kernel": n, "lanes": "all", "dispatches": sum(len(dispatches[k]) for k in keys),
               "lanes_mean": round(sum(k[1] * len(dispatches[k]) for k in keys)
                                   / max(1, sum(len(dispatches[k]) for k in keys)), 1)}
        if tot.get("SQ_WAVES"):
            row["valu_insts_per_wave"] = round(tot.get("SQ_INSTS_VALU", 0.0) / tot["SQ_WAVES"], 1)
        if tot.get("SQ_WAVE_CYCLES"):
            row["valu_active_frac_of_wave_cycles"] = round(
                tot.get("SQ_ACTIVE_INST_VALU", 0.0) / tot["SQ_WAVE_CYCLES"], 3)
        out.append(row)
    return out


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        print(__doc__, file=sys.stderr)
        return 2
    json.dump(summarise(argv[0], int(argv[1]) if len(argv) > 1 else 0), sys.stdout, indent=1)
    print()
    return 0


if __name__ == "__main__":
    sys.exit(main())
