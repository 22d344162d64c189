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
