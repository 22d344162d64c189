"""Process resource limits.

Torrent storage keeps one descriptor open per file of the torrent for the whole session (the
reference's fs-chunk-store opens a random-access-file per file the same way), and every
connection holds one more. A season pack or a music / comic torrent with thousands of files
would hit the common soft limit of 1,024 open files with EMFILE halfway through the job, so
the worker raises its soft RLIMIT_NOFILE to the hard limit at start (capped), and the storage
checks the headroom before it opens a torrent's files.
"""
from __future__ import annotations

import os
from typing import Tuple

try:
    import resource
except ImportError:          # non-POSIX
    resource = None

NOFILE_CAP = 1 << 20


def raise_nofile(cap: int = NOFILE_CAP) -> Tuple[int, int]:
    """Raise the soft open-file limit to the hard limit (at most ``cap``); returns the
    (soft, hard) limits now in force. Never lowers the soft limit."""
    if resource is None:
        return (-1, -1)
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = hard if hard != resource.RLIM_INFINITY else cap
    want = min(want, cap)
    if soft != resource.RLIM_INFINITY and soft < want:
        try:
            resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
            soft = want
        except (ValueError, OSError):
            pass
    return soft, hard


def open_fds() -> int:
    """Descriptors this process has open (Linux /proc; 0 when unknown)."""
    try:
        return len(os.listdir("/proc/self/fd"))
    except OSError:
        return 0


def fd_headroom() -> int:
    """Descriptors that can still be opened before EMFILE (a large number when unknown)."""
    if resource is None:
        return 1 << 30
    soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
    if soft == resource.RLIM_INFINITY:
        return 1 << 30
    return max(0, soft - open_fds())


PIPE_MAX = 1 << 20          # fs.pipe-max-size default: the most an unprivileged pipe gets
PIPE_MIN = 64 << 10         # below this a splice transfer copies through user space instead
PIPES_PER_PROC = 16         # transfers in flight per worker process (relays, range GETs)


def pipe_budget_bytes() -> int:
    """Pipe capacity this uid may hold before new pipes shrink to two pages
    (``fs.pipe-user-pages-soft`` x page size); 0 = unbounded (root, or no soft limit).
    ``STAGER_PIPE_BUDGET_BYTES`` overrides it (an operator who knows the uid's budget, or a
    rehearsal of an unprivileged node's sizing as root)."""
    env = os.environ.get("STAGER_PIPE_BUDGET_BYTES", "")
    if env.strip().isdigit():
        return int(env)
    if hasattr(os, "geteuid") and os.geteuid() == 0:
        return 0
    try:
        with open("/proc/sys/fs/pipe-user-pages-soft") as f:
            pages = int(f.read().strip() or 0)
    except (OSError, ValueError):
        return 0
    return pages * os.sysconf("SC_PAGE_SIZE") if pages > 0 else 0


def pipe_size(pipe_kb: int = 0, sharers: int = 4, per_proc: int = PIPES_PER_PROC,
              budget: int = -1) -> int:
    """Splice pipe capacity for this process: ``pipe_kb`` when set, else a power of two in
    [64 KiB, 1 MiB] such that ``sharers`` processes x ``per_proc`` pipes fit in three
    quarters of the uid's pipe budget (the rest is headroom for other pipes of the uid)."""
    if pipe_kb > 0:
        return pipe_kb << 10
    if budget < 0:
        budget = pipe_budget_bytes()
    if budget == 0:
        return PIPE_MAX
    share = budget * 3 // 4 // max(1, sharers) // max(1, per_proc)
    size = PIPE_MIN
    while size * 2 <= min(share, PIPE_MAX):
        size *= 2
    return size


PIPE_GOOD = 512 << 10       # pipes this large relay within ~2 % of 1 MiB ones; 256 KiB cost 13 %


def relay_plan(concurrency: int, parts_per_job: int, sharers: int,
               budget: int = -1) -> tuple:
    """(jobs in flight per process, pipe bytes) for ``sharers`` processes of one uid, each
    running ``concurrency`` jobs of ``parts_per_job`` relays (one pipe each): the largest pipe
    (<= 1 MiB) that fits 7/8 of the uid's pipe budget, lowering the concurrency (to 2 at
    least) while the pipe would be smaller than 512 KiB. MI355X box, one 16-CPU rank
    (profiles/archive/r4/pipes/): 1 MiB 66.7 / 66.1 GB/s, 512 KiB 63.2 / 65.8, 512 KiB at 3 jobs
    67.7 / 62.2, 256 KiB 53.6 / 62.5 - so at 8 ranks x 2 processes (64 MiB budget) 3 jobs on
    512 KiB pipes beat 4 jobs on 256 KiB ones."""
    if budget < 0:
        budget = pipe_budget_bytes()
    if budget == 0:
        return concurrency, PIPE_MAX
    usable = budget * 7 // 8
    conc = max(1, concurrency)

    def size_for(c: int) -> int:
        share = usable // max(1, sharers) // max(1, c * parts_per_job)
        size = PIPE_MIN
        while size * 2 <= min(share, PIPE_MAX):
            size *= 2
        return size
    while conc > 2 and size_for(conc) < PIPE_GOOD:
        conc -= 1
    return conc, size_for(conc)


def apply_pipe_size(pipe_kb: int = 0, sharers: int = 4) -> int:
    """Size the native transport's splice pipes (main and tee() duplicate alike);
    returns the main size, 0 without the native module."""
    try:
        from ..ops import native
        n = native()
    except Exception:
        return 0
    main = pipe_size(pipe_kb, sharers)
    # the tee() duplicate pipe as large as the main one: 38.7 - 38.8 vs 32.1 - 35.6 GB/s for
    # the CRC'd headline at 1 MiB vs 256 KiB (profiles/archive/r3_teepipe/)
    tee_kb = int(os.environ.get("STAGER_TEE_PIPE_KB", "0") or 0)     # A/B knob
    n.set_pipe_sizes(main, tee_kb << 10 if tee_kb > 0 else main)
    return main
