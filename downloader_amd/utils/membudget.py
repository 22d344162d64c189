"""Process-wide byte budget for the hashed relay's part buffers.

The reference's memory is small and bounded: webtorrent writes pieces to disk through
fs-chunk-store (/root/reference/lib/download.js:64) and minio-js ``fPutObject`` streams one
part at a time (/root/reference/lib/upload.js:45). The streamed-torrent path here instead
relays every S3 part through a pooled buffer as large as the part (its pieces are hashed in
user space, torrent/stream.py), so without a bound a worker's resident memory grew with
relays in flight x part size, plus parts waiting for their DMA to the GPU, plus the idle
buffers kept warm: 9.5 GB peak for two 20 GB jobs in round 3.

One budget now covers all of it. Every relay draws its part's bytes from ``PartBudget``
before it starts (so no source connection is held open while waiting), and gives them back
when its buffer returns to the pool: at once for host-hashed parts, at the DMA's completion
for GPU-hashed ones (the part's bytes then live in HBM, not in host memory). The native pool
(``relay_pool_set_budget``) keeps leased + idle buffers inside the same number by unmapping
idle buffers before it maps a new one, and records its high-water mark (``peak_bytes``).

Default: ``download.relay_memory_fraction`` (0.25) of this worker's share of the memory
limit - the cgroup's ``memory.max`` (else physical memory) divided by the worker processes
that share it (``pool_workers``): ``STAGER_POOL_WORKERS`` when set, else the node's GPU slots
(``utils.cpus.gpu_slots``, as the CPU budget is divided) x the worker processes of one slot
(``STAGER_PROCS_PER_SLOT``, set by the supervisor and the bench, default 1). A worker on a
shared 8-GPU node therefore takes 1/8 of the node's budget even when nothing told it how many
neighbours it has. ``download.relay_memory_mb`` overrides it.
"""
from __future__ import annotations

import asyncio
import collections
import os
import weakref
from typing import Deque, Optional, Tuple

MiB = 1 << 20
BUFFER_ALIGN = 2 * MiB          # the native pool maps part buffers in 2 MiB (huge page) units
MIN_BUDGET = 128 * MiB


def cgroup_memory_limit(root: str = "/sys/fs/cgroup") -> int:
    """The cgroup memory limit in bytes (v2 ``memory.max``, v1 ``memory.limit_in_bytes``);
    0 = none."""
    for path in (os.path.join(root, "memory.max"),
                 os.path.join(root, "memory", "memory.limit_in_bytes")):
        try:
            with open(path) as f:
                v = f.read().strip()
        except OSError:
            continue
        if v and v != "max":
            try:
                n = int(v)
            except ValueError:
                continue
            if 0 < n < (1 << 60):            # v1 reports "unlimited" as ~2^63
                return n
    return 0


def physical_memory() -> int:
    try:
        return os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
    except (ValueError, OSError, AttributeError):
        return 0


def memory_limit() -> int:
    """What this container may use: the cgroup limit, else physical memory (0 = unknown)."""
    lim = cgroup_memory_limit()
    phys = physical_memory()
    if lim and phys:
        return min(lim, phys)
    return lim or phys


def _env_int(name: str) -> int:
    try:
        return max(0, int(os.environ.get(name, "") or 0))
    except ValueError:
        return 0


def procs_per_slot() -> int:
    """Worker processes one GPU slot runs (``STAGER_PROCS_PER_SLOT``; supervisor ``-n``,
    bench ``--procs-per-rank``)."""
    return max(1, _env_int("STAGER_PROCS_PER_SLOT"))


def pool_workers() -> int:
    """Worker processes sharing this memory limit: ``STAGER_POOL_WORKERS`` if set, else
    GPU slots of the node x processes per slot (the per-slot share, like the CPU budget)."""
    n = _env_int("STAGER_POOL_WORKERS")
    if n:
        return n
    from .cpus import gpu_slots
    return max(1, gpu_slots()) * procs_per_slot()


def relay_budget_bytes(download_cfg) -> int:
    """The part-buffer budget of this worker process (see the module docstring)."""
    mb = int(getattr(download_cfg, "relay_memory_mb", 0) or 0)
    if mb > 0:
        return mb * MiB
    frac = float(getattr(download_cfg, "relay_memory_fraction", 0.25) or 0.25)
    lim = memory_limit()
    if lim <= 0:
        return 4096 * MiB
    return max(MIN_BUDGET, int(lim // pool_workers() * frac))


def swarm_bytes(mb: int, fraction: float = 0.125, cap_mb: int = 4096) -> int:
    """Swarm piece memory (download.swarm_pool_mb / swarm_backlog_mb): ``mb`` MiB when set,
    else ``fraction`` of this worker's share of the memory limit, at most ``cap_mb`` and at
    least 256 MiB - 4 GiB each on a GPU box's 150 GiB share, 1 GiB in an 8 GiB container."""
    if mb and mb > 0:
        return int(mb) * MiB
    lim = memory_limit()
    if lim <= 0:
        return cap_mb * MiB
    return max(256 * MiB, min(cap_mb * MiB, int(lim // pool_workers() * fraction)))


def buffer_bytes(n: int) -> int:
    """What a part of ``n`` bytes leases from the native pool."""
    return -(-max(1, n) // BUFFER_ALIGN) * BUFFER_ALIGN


class PartBudget:
    """FIFO byte semaphore. A request larger than the whole budget is granted once nothing
    else is held (so a part always makes progress); the native pool then counts that lease as
    ``over_budget``."""

    def __init__(self, capacity: int):
        self.capacity = max(1, int(capacity))
        self.used = 0
        self.peak = 0
        self.waits = 0
        self._waiters: Deque[Tuple[int, asyncio.Future]] = collections.deque()

    def _fits(self, n: int) -> bool:
        return self.used + n <= self.capacity or self.used == 0

    async def acquire(self, n: int) -> int:
        n = buffer_bytes(n)
        if not self._waiters and self._fits(n):
            self._grant(n)
            return n
        self.waits += 1
        fut = asyncio.get_running_loop().create_future()
        self._waiters.append((n, fut))
        try:
            await fut
        except asyncio.CancelledError:
            if fut.done() and not fut.cancelled():
                self.release(n)              # granted just as we were cancelled
            else:
                try:
                    self._waiters.remove((n, fut))
                except ValueError:
                    pass
                self._wake()
            raise
        return n

    def _grant(self, n: int) -> None:
        self.used += n
        self.peak = max(self.peak, self.used)

    def release(self, n: int) -> None:
        self.used = max(0, self.used - n)
        self._wake()

    def _wake(self) -> None:
        while self._waiters:
            n, fut = self._waiters[0]
            if fut.done():
                self._waiters.popleft()
                continue
            if not self._fits(n):
                break
            self._waiters.popleft()
            self._grant(n)
            fut.set_result(None)

    def resize(self, capacity: int) -> None:
        self.capacity = max(1, int(capacity))
        self._wake()

    def stats(self) -> dict:
        return {"capacity": self.capacity, "used": self.used, "peak": self.peak,
                "waits": self.waits, "queued": len(self._waiters)}


_budgets: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def part_budget(capacity: int) -> PartBudget:
    """The process's budget (one per event loop; tests run several loops in turn). The native
    pool gets the same bound."""
    loop = asyncio.get_running_loop()
    b: Optional[PartBudget] = _budgets.get(loop)
    if b is None:
        b = _budgets[loop] = PartBudget(capacity)
    elif b.capacity != capacity:
        b.resize(capacity)
    try:
        from ..ops import native
        native().relay_pool_set_budget(int(capacity))
    except Exception as e:           # no native module: nothing pools part buffers anyway
        global _native_warned
        if not _native_warned:
            _native_warned = True
            from .log import get_logger
            get_logger("membudget").warn("native part pool budget not set", err=str(e))
    return b


_native_warned = False
