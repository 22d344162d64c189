"""Summarise a rocprofv3 ``--kernel-trace`` CSV: per kernel, launches, duration statistics and
the grid size (threads) per launch - for ``sha1_lanes`` one thread is one piece (lane), so
the grid tells how many pieces each launch hashed in parallel - plus the concurrency of the
launches (how many overlap in time).

    python -m downloader_amd.bench.trace_summary <kernel_trace.csv> [--copies
        <memory_copy_trace.csv>] [--json out.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics
import sys
from typing import Dict, List


def summarise(path: str) -> Dict[str, dict]:
    rows: Dict[str, List[dict]] = {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            rows.setdefault(short, []).append(r)
    out: Dict[str, dict] = {}
    for k, rs in rows.items():
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rs]
        grid = [int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) for r in rs]
        spans = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs)
        # max launches running at once
        ev = sorted([(s, 1) for s, _ in spans] + [(e, -1) for _, e in spans])
        cur = peak = 0
        for _, d in ev:
            cur += d
            peak = max(peak, cur)
        busy = 0
        last = 0
        for s, e in spans:              # union of the launches' intervals
            s = max(s, last)
            if e > s:
                busy += e - s
                last = e
        wall = (spans[-1][1] - spans[0][0]) if spans else 0
        # launches that ran alone vs beside another one of the same kernel (any overlap)
        iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs]
        alone = [not any(s1 < e0 and s0 < e1 for m, (s1, e1) in enumerate(iv) if m != j)
                 for j, (s0, e0) in enumerate(iv)]
        solo = [d for d, a in zip(dur, alone) if a]
        both = [d for d, a in zip(dur, alone) if not a]
        extra = {"ms_median": round(statistics.median(dur), 3),
                 "solo_launches": len(solo),
                 "ms_solo_mean": round(statistics.mean(solo), 3) if solo else None,
                 "ms_overlapped_mean": round(statistics.mean(both), 3) if both else None}
        out[k] = {"launches": len(rs), "ms_mean": round(statistics.mean(dur), 3), **extra,
                  "ms_min": round(min(dur), 3), "ms_max": round(max(dur), 3),
                  "ms_total": round(sum(dur), 1),
                  "grid_threads_mean": round(statistics.mean(grid), 1),
                  "grid_threads_min": min(grid), "grid_threads_max": max(grid),
                  "max_concurrent": peak,
                  "device_busy_share": round(busy / wall, 3) if wall else 0.0}
    return out


def summarise_copies(path: str) -> Dict[str, dict]:
    """A rocprofv3 ``--memory-copy-trace`` CSV: per direction, copies, duration statistics,
    bytes and GB/s when the trace has a size column, and the peak of overlapping copies
    (copies on separate SDMA engines run at once)."""
    rows: Dict[str, List[dict]] = {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.setdefault(r.get("Direction", r.get("Operation", "?")), []).append(r)
    out: Dict[str, dict] = {}
    for k, rs in rows.items():
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rs]
        size_key = next((c for c in rs[0] if c.lower() in ("size", "bytes", "copy_bytes")), None)
        d = {"copies": len(rs), "ms_mean": round(statistics.mean(dur), 3),
             "ms_median": round(statistics.median(dur), 3), "ms_max": round(max(dur), 3)}
        if size_key:
            sizes = [int(r[size_key]) for r in rs]
            big = [(b, t) for b, t in zip(sizes, dur) if b >= 1 << 20 and t > 0]
            d["bytes"] = sum(sizes)
            if big:
                d["GBps_median_1MiB_plus"] = round(statistics.median(b / t / 1e6 for b, t in big), 2)
        ev = sorted([(int(r["Start_Timestamp"]), 1) for r in rs] +
                    [(int(r["End_Timestamp"]), -1) for r in rs])
        cur = peak = 0
        for _, x in ev:
            cur += x
            peak = max(peak, cur)
        d["max_concurrent"] = peak
        out[k] = d
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--copies", default="", help="a memory_copy_trace.csv as well")
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    s = summarise(a.trace)
    if a.copies:
        s["memory_copies"] = summarise_copies(a.copies)
    txt = json.dumps(s, indent=1)
    if a.json:
        with open(a.json, "w") as f:
            f.write(txt + "\n")
    print(txt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
