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


def gpu_slots() -> int:
    """GPUs this process may use = worker slots of the node: ``STAGER_GPU_SLOTS``, else the
    ``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES`` list, else the DRM render nodes the
    container can open (the build pool's 1-GPU boxes show one of the host's eight). Never
    initialises HIP."""
    env = os.environ.get("STAGER_GPU_SLOTS", "")
    if env.strip().isdigit() and int(env) > 0:
        return int(env)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        ids = [x for x in os.environ.get(var, "").split(",") if x.strip()]
        if ids:
            return len(ids)
    try:
        n = sum(1 for d in os.listdir("/dev/dri") if d.startswith("renderD"))
    except OSError:
        n = 0
    return max(1, n)


def _core_of(cpu: int, root: str) -> tuple:
    base = f"{root}/cpu{cpu}/topology"
    try:
        with open(f"{base}/physical_package_id", encoding="ascii") as f:
            pkg = int(f.read())
        with open(f"{base}/core_id", encoding="ascii") as f:
            core = int(f.read())
        return (pkg, core)
    except (OSError, ValueError):
        return (-1, cpu)          # unknown topology: every CPU is its own core


def cores(cpus, root: str = "/sys/devices/system/cpu") -> list:
    """CPUs grouped by physical core (SMT siblings together), cores ordered by (package,
    core id), threads within a core ascending."""
    by = {}
    for c in sorted(cpus):
        by.setdefault(_core_of(c, root), []).append(c)
    return [by[k] for k in sorted(by)]


def slot_cpus(index: int, slots: int, budget: int, cpus, root: str = "/sys/devices/system/cpu") -> list:
    """CPUs of worker slot ``index`` of ``slots``: the slot owns a contiguous run of
    ``len(cores) // slots`` physical cores (so no two slots share SMT siblings or, when the
    run fits, a package) and uses ``budget // slots`` of their threads, first threads of each
    core before second ones (under a quota a thread per core beats two threads on one)."""
    groups = cores(cpus, root)
    per_core = len(groups) // max(1, slots)
    want = budget // max(1, slots)
    if per_core < 1 or want < 1:
        return []
    mine = groups[index * per_core:(index + 1) * per_core]
    depth = max(len(g) for g in mine)
    order = [g[t] for t in range(depth) for g in mine if t < len(g)]
    return sorted(order[:want])


def pin_slot(index: int, slots: int) -> list:
    """Pin this process to GPU slot ``index`` of ``slots``' share of the CPU budget
    (min(mask, cgroup quota) / slots). The share does not depend on how many slots are busy,
    so one worker sees the same CPUs whether it runs alone or next to seven others (weak
    scaling). Returns the slice ([] = unpinned: no quota and one slot = the whole machine)."""
    avail = sorted(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    if quota == math.inf and slots <= 1:
        return []
    budget = len(avail) if quota == math.inf else min(len(avail), max(1, math.ceil(quota)))
    mine = slot_cpus(index, slots, budget, avail)
    if not mine:
        return []
    os.sched_setaffinity(0, mine)
    effective_cpus.cache_clear()
    return mine


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
