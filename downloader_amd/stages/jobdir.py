"""Per-job download directories with resume and duplicate-delivery safety.

The reference stages every job in ``<download_path>/<media.id>`` (lib/download.js:234-240), so
two concurrent deliveries of the same id share (and delete) each other's files (SURVEY App. A
#18), while a retried job starts from scratch (§5.4: no HTTP resume; torrent data may be
re-verified by webtorrent).

Here the job directory is claimed with an exclusive ``flock`` on ``<root>/.locks/<id>.lock``:
the holder uses ``<root>/<id>`` - so a retry of a failed attempt finds its partial data
(HTTP Range resume, multipart resume, torrent recheck) - and a concurrent duplicate that cannot
take the lock works in a private ``<root>/<id>.<token>`` directory instead.
"""
from __future__ import annotations

import fcntl
import os
import secrets
import shutil
from typing import Optional


class JobDir:
    def __init__(self, root: str, job_id: str):
        self.root = root
        self.job_id = job_id.replace("/", "_") or "_"
        self.path = ""
        self.exclusive = False
        self._fd: Optional[int] = None

    def acquire(self) -> str:
        locks = os.path.join(self.root, ".locks")
        os.makedirs(locks, exist_ok=True)
        fd = os.open(os.path.join(locks, self.job_id + ".lock"),
                     os.O_RDWR | os.O_CREAT | getattr(os, "O_CLOEXEC", 0), 0o644)
        try:
            fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except BlockingIOError:
            os.close(fd)
            self.path = os.path.join(self.root, f"{self.job_id}.{secrets.token_hex(4)}")
            self.exclusive = False
        else:
            self._fd = fd
            self.path = os.path.join(self.root, self.job_id)
            self.exclusive = True
        os.makedirs(self.path, exist_ok=True)
        return self.path

    def release(self) -> None:
        if self._fd is not None:
            try:
                fcntl.flock(self._fd, fcntl.LOCK_UN)
            finally:
                os.close(self._fd)
                self._fd = None

    def remove(self) -> None:
        if self.path:
            shutil.rmtree(self.path, ignore_errors=True)
