"""Host readiness report (``python -m downloader_amd doctor``).

What a worker's throughput depends on besides its config, checked in one place: the native
extension and which SIMD paths it runs (AVX-512 multi-buffer SHA-1, VPCLMULQDQ CRC32C), the
usable CPUs (affinity and cgroup quota), the open-file limit (one descriptor per torrent file),
the uid's pipe page budget that splice transfers share (fs.pipe-user-pages-soft), the memory
limit and the streamed relay's part-buffer budget derived from it, transparent
huge pages for the relay's part buffers, and the HIP devices for the gfx950 kernels. Each
finding that costs performance comes with a warning saying what to change.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


def report(pipe_sharers: int = 4) -> Dict[str, Any]:
    from . import limits
    from .cpus import effective_cpus
    out: Dict[str, Any] = {"warnings": []}
    warn: List[str] = out["warnings"]

    try:
        from ..ops import native
        n = native()
        out["native"] = {"loaded": True, "sha1_multibuffer": bool(n.sha1_mb_supported()),
                         "crc32c": n.crc32c_impl()}
        if not n.sha1_mb_supported():
            warn.append("no AVX-512 multi-buffer SHA-1: torrent pieces hash ~3-5x slower per "
                        "core (verify_backend auto will use the GPU when one is present)")
        if n.crc32c_impl() != "avx512-vpclmulqdq":
            warn.append("CRC32C without VPCLMULQDQ (~19 GB/s per core instead of 40-50)")
    except Exception as e:               # extension missing / not built
        out["native"] = {"loaded": False, "error": str(e)}
        warn.append("native extension not loaded: run python -m downloader_amd.ops.build")

    out["cpus"] = {"effective": effective_cpus(), "affinity": len(os.sched_getaffinity(0))}

    soft, hard = limits.raise_nofile()
    out["nofile"] = {"soft": soft, "hard": hard}
    if 0 < soft < 4096:
        warn.append(f"open-file limit {soft}: season packs with thousands of files need more "
                    "(raise the hard limit)")

    budget = limits.pipe_budget_bytes()
    size = limits.pipe_size(0, pipe_sharers, budget=budget)
    out["pipes"] = {"euid": os.geteuid(), "budget_bytes": budget or None,
                    "pipe_max_size": int(_read("/proc/sys/fs/pipe-max-size") or 0),
                    "sharers": pipe_sharers, "pipe_bytes": size}
    if budget and size < (256 << 10):
        warn.append(f"splice pipes of {size >> 10} KiB for {pipe_sharers} workers of this uid: "
                    "raise fs.pipe-user-pages-soft or run fewer workers per uid")

    from . import membudget
    from .config import DownloadConfig
    lim = membudget.memory_limit()
    dc = DownloadConfig()
    part = membudget.relay_budget_bytes(dc)
    swarm = membudget.swarm_bytes(dc.swarm_pool_mb) + membudget.swarm_bytes(dc.swarm_backlog_mb)
    # docs/OPERATIONS.md "Memory": fixed part + HIP runtime + part budget + swarm pieces
    worst = part + swarm + int(2.3e9)
    out["memory"] = {"limit_bytes": lim or None,
                     "cgroup_limit_bytes": membudget.cgroup_memory_limit() or None,
                     "workers": membudget.pool_workers(),
                     "part_budget_bytes": part,
                     "swarm_pool_and_backlog_bytes": swarm,
                     "worst_case_worker_bytes": worst}
    if lim and membudget.pool_workers() * worst > lim:
        warn.append(f"{membudget.pool_workers()} workers x ({part >> 20} MiB part budget + "
                    f"{swarm >> 20} MiB swarm pieces + ~2.3 GB) exceed the memory limit of "
                    f"{lim >> 20} MiB: lower download.relay_memory_mb / swarm_pool_mb / "
                    "swarm_backlog_mb or run fewer workers")

    thp = _read("/sys/kernel/mm/transparent_hugepage/enabled")
    out["thp"] = thp
    if thp and "[never]" in thp:
        warn.append("transparent huge pages off: the relay's 64 MiB part buffers fault in "
                    "4 KiB pages (the first streamed torrent after idle runs slower)")

    try:
        from ..ops import gpu_available, gpuhash
        if gpu_available():
            g = gpuhash()
            out["gpu"] = {"devices": g.device_count(), "arch": g.arch()}
        else:
            out["gpu"] = {"devices": 0}
    except Exception as e:
        out["gpu"] = {"devices": 0, "error": str(e)}
    return out
