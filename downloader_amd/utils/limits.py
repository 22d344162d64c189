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
