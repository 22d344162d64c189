"""Worker pool supervisor - the reference's scaling unit is "one more container" (Dockerfile,
SURVEY §2.6 DP analogue); here one process launches N identical workers that all consume the
same ``v1.download`` queue (prefetch-bounded), restarts crashed workers with backoff (the
reference relies on crash-only restart by its orchestrator, index.js:35) and forwards
SIGINT/SIGTERM for a graceful drain.

Workers can be pinned to CPU sets (``cpus_per_worker``) so the page-cache / socket work of one
worker stays on one CCD of the host EPYC.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence


@dataclass
class Slot:
    index: int
    proc: Optional[subprocess.Popen] = None
    restarts: int = 0
    started: float = 0.0
    backoff: float = 1.0
    restart_at: float = 0.0          # > 0: respawn due at this monotonic time
    done: bool = False               # exited 0, or out of restarts: not respawned
    exit_codes: List[int] = field(default_factory=list)


def auto_cpus_per_worker(n_workers: int, available: Sequence[int], quota: float) -> int:
    """Each worker's share of the CPU quota (``utils.cpus.quota_share``)."""
    from ..utils.cpus import quota_share
    return quota_share(available, n_workers, quota) if n_workers > 0 else 0


def cpu_slices(n_workers: int, cpus_per_worker: int, available: Optional[Sequence[int]] = None
               ) -> List[List[int]]:
    """``cpus_per_worker``: K > 0 pins every worker to K contiguous CPUs, 0 = auto (quota
    share, ``auto_cpus_per_worker``), < 0 = no pinning."""
    cpus = sorted(available if available is not None else os.sched_getaffinity(0))
    if cpus_per_worker == 0:
        from ..utils.cpus import cgroup_cpu_quota
        cpus_per_worker = auto_cpus_per_worker(n_workers, cpus, cgroup_cpu_quota())
    if cpus_per_worker <= 0:
        return [[] for _ in range(n_workers)]
    out = []
    for i in range(n_workers):
        s = cpus[(i * cpus_per_worker) % len(cpus):][:cpus_per_worker]
        out.append(s)
    return out


class Supervisor:
    def __init__(self, n: int, argv: Sequence[str], env: Optional[Dict[str, str]] = None,
                 cpus_per_worker: int = 0, max_restarts: int = 10, base_port: int = 0,
                 backoff: float = 1.0):
        self.n = n
        self.argv = list(argv)
        self.env = dict(env or os.environ)
        self.cpus = cpu_slices(n, cpus_per_worker)
        self.max_restarts = max_restarts
        self.base_port = base_port
        self.initial_backoff = backoff
        self.slots = [Slot(i, backoff=backoff) for i in range(n)]
        self.stopping = False

    def _spawn(self, s: Slot) -> None:
        env = dict(self.env)
        env["STAGER_WORKER_INDEX"] = str(s.index)
        # the workers share the uid's pipe page budget: size their splice pipes for all n
        # (an explicit setting in the environment wins)
        env.setdefault("STAGER_DOWNLOAD__PIPE_SHARERS", str(max(4, self.n)))
        # ... and the slot's memory: each sizes its part-buffer budget to its share, memory
        # limit / (GPU slots x workers per slot) (utils/membudget.pool_workers)
        env.setdefault("STAGER_PROCS_PER_SLOT", str(self.n))
        if self.base_port:
            env["PORT"] = str(self.base_port + s.index)   # distinct /health ports
        cpus = self.cpus[s.index]

        def pre() -> None:
            os.setsid()
            if cpus:
                os.sched_setaffinity(0, cpus)
        s.proc = subprocess.Popen(self.argv, env=env, preexec_fn=pre)
        s.started = time.monotonic()

    def start(self) -> None:
        for s in self.slots:
            self._spawn(s)

    def poll(self) -> None:
        """Reap exited workers once each and respawn crashed ones after an exponential
        backoff (reset after 60 s of healthy uptime). Never sleeps: a crash-looping worker
        does not delay the others' restarts or the reaction to SIGTERM."""
        now = time.monotonic()
        for s in self.slots:
            if self.stopping or s.done:
                continue
            if s.proc is not None:
                if s.proc.poll() is None:
                    continue
                rc = s.proc.returncode
                s.exit_codes.append(rc)
                s.proc = None
                if rc == 0 or s.restarts >= self.max_restarts:
                    s.done = True
                    continue
                if now - s.started > 60:
                    s.backoff = self.initial_backoff
                s.restart_at = now + min(s.backoff, 30.0)
                s.backoff *= 2
            if s.proc is None and s.restart_at and now >= s.restart_at:
                s.restart_at = 0.0
                s.restarts += 1
                self._spawn(s)

    def stop(self, timeout: float = 30.0) -> List[int]:
        self.stopping = True
        for s in self.slots:
            if s.proc is not None and s.proc.poll() is None:
                try:
                    s.proc.send_signal(signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.monotonic() + timeout
        codes = []
        for s in self.slots:
            if s.proc is None:
                continue
            try:
                codes.append(s.proc.wait(max(0.1, deadline - time.monotonic())))
            except subprocess.TimeoutExpired:
                s.proc.kill()
                codes.append(s.proc.wait())
        return codes

    def alive(self) -> int:
        return sum(1 for s in self.slots if s.proc is not None and s.proc.poll() is None)

    def run_forever(self) -> int:
        stop = {"flag": False}

        def handler(sig, frm):
            stop["flag"] = True
        signal.signal(signal.SIGINT, handler)
        signal.signal(signal.SIGTERM, handler)
        self.start()
        while not stop["flag"]:
            self.poll()
            if all(s.done for s in self.slots):
                break
            time.sleep(0.5)
        codes = self.stop()
        return 0 if all(c == 0 for c in codes) else 1


def worker_argv(config_path: str = "", extra: Sequence[str] = ()) -> List[str]:
    argv = [sys.executable, "-m", "downloader_amd", "worker"]
    if config_path:
        argv += ["--config", config_path]
    return argv + list(extra)
