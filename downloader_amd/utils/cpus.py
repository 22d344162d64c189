"""CPU budget of this process: the affinity mask capped by the cgroup v2 CPU quota.

Containers (the build pool's GPU boxes: 256 CPUs in the mask, ``cpu.max`` = 16 CPUs) expose
far more CPUs than they may use; sizing thread pools or worker counts by ``os.cpu_count()``
there oversubscribes the quota. Mirrors ``effective_cpus()`` in ``csrc/hashing.cpp``.
"""
from __future__ import annotations

import math
import os
from functools import lru_cache


def cgroup_cpu_quota(path: str = "/sys/fs/cgroup/cpu.max") -> float:
    """CPUs granted by cgroup v2 ``cpu.max`` (``inf`` when unlimited or unreadable)."""
    try:
        with open(path, "r", encoding="ascii") as f:
            quota, period = f.read().split()[:2]
    except (OSError, ValueError):
        return math.inf
    if quota == "max" or int(period) <= 0:
        return math.inf
    return int(quota) / int(period)


@lru_cache(maxsize=1)
def effective_cpus() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = cgroup_cpu_quota()
    if q != math.inf:
        n = min(n, max(1, math.ceil(q)))
    return max(1, n)


def quota_share(available, n: int, quota: float) -> int:
    """CPUs per process when ``n`` processes share ``available`` CPUs under a cgroup quota:
    available / n capped by ceil(quota / n); 0 = do not pin (no quota, or the share would be
    the whole mask). Contiguous pinning to the quota share measured +40 % on the build box,
    whose mask spans 256 CPUs (2 NUMA nodes) but whose quota is 16."""
    n = max(1, n)
    if quota == math.inf:
        return 0
    per = min(len(available) // n, max(2, math.ceil(quota / n)))
    return per if per < len(available) else 0


def pin_share(index: int, n: int, per: int = 0) -> list:
    """Pin this process to slice ``index`` of ``n`` contiguous slices of its CPU mask
    (``per`` CPUs each; 0 = ``quota_share``). Children inherit the mask. Returns the slice
    ([] = left unpinned)."""
    cpus = sorted(os.sched_getaffinity(0))
    if per == 0:
        per = quota_share(cpus, n, cgroup_cpu_quota())
    if per < 2 or per * max(1, n) > len(cpus):
        return []
    mine = cpus[index * per:(index + 1) * per]
    os.sched_setaffinity(0, mine)
    effective_cpus.cache_clear()
    return mine
