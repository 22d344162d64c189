"""Piece storage (replaces ``fs-chunk-store`` + ``torrent-piece`` in webtorrent, yarn.lock:1407,3543).

The torrent's files are treated as one concatenated byte space split into pieces. Writes of
verified pieces go straight to the files with ``pwrite``; webseed bodies are spliced into the
files by the native transport (``segments()`` gives the fd/offset pairs). Piece verification
uses the native SHA-1 (``ops.hashing``); a full recheck can run on the MI355X.
"""
from __future__ import annotations

import errno
import os
import threading
from contextlib import contextmanager
from typing import Iterator, List, Optional, Sequence, Tuple

from ..ops import hashing
from ..utils import limits
from .metainfo import Metainfo


class Bitfield:
    __slots__ = ("n", "bits", "count")

    def __init__(self, n: int, data: Optional[bytes] = None):
        self.n = n
        self.bits = bytearray((n + 7) // 8)
        self.count = 0
        if data is not None:
            self.load(data)

    def load(self, data: bytes) -> None:
        need = (self.n + 7) // 8
        if len(data) < need:
            raise ValueError("bitfield too short")
        self.bits = bytearray(data[:need])
        spare = need * 8 - self.n
        if spare and self.bits:
            self.bits[-1] &= (0xFF << spare) & 0xFF
        self.count = sum(bin(b).count("1") for b in self.bits)

    def __contains__(self, i: int) -> bool:
        return bool(self.bits[i >> 3] & (0x80 >> (i & 7)))

    def set(self, i: int) -> bool:
        m = 0x80 >> (i & 7)
        if self.bits[i >> 3] & m:
            return False
        self.bits[i >> 3] |= m
        self.count += 1
        return True

    def clear(self, i: int) -> None:
        m = 0x80 >> (i & 7)
        if self.bits[i >> 3] & m:
            self.bits[i >> 3] &= ~m & 0xFF
            self.count -= 1

    @property
    def complete(self) -> bool:
        return self.count == self.n

    def to_bytes(self) -> bytes:
        return bytes(self.bits)

    def missing(self) -> List[int]:
        return [i for i in range(self.n) if i not in self]


FD_MARGIN = 64      # connections, logs, pipes of the job besides the storage's own files


class Storage:
    def __init__(self, meta: Metainfo, root: str, preallocate: bool = True):
        self.meta = meta
        self.root = root
        self.paths = meta.local_files(root)
        self.fds: List[int] = []
        # executor threads inside write()/read() hold the fds: close() waits for them (a
        # cancelled piece task does not stop its thread's pwrite, and a closed fd number can
        # be reused by the next open of any job in the process)
        self._cv = threading.Condition()
        self._users = 0
        self._closed = False
        # one descriptor per file for the session, plus the verifier's own opens and the
        # job's connections: fail with a clear error instead of EMFILE halfway through
        need = len(self.paths) * 2 + FD_MARGIN
        if need > limits.fd_headroom():
            raise OSError(errno.EMFILE, f"torrent has {len(self.paths)} files: needs about "
                                        f"{need} more open files than RLIMIT_NOFILE leaves "
                                        f"({limits.fd_headroom()}); raise the limit")
        # Only data that was on disk before we created/preallocated the files can be resumed;
        # a fresh (sparse) layout needs no recheck pass at all.
        self.preexisting = any(os.path.isfile(p) and os.path.getsize(p) > 0 for p, _ in self.paths)
        for p, n in self.paths:
            os.makedirs(os.path.dirname(p), exist_ok=True)
            fd = os.open(p, os.O_RDWR | os.O_CREAT | getattr(os, "O_CLOEXEC", 0), 0o644)
            if preallocate and os.fstat(fd).st_size != n:
                os.ftruncate(fd, n)
            self.fds.append(fd)

    def piece_range(self, i: int) -> Tuple[int, int]:
        return i * self.meta.piece_length, self.meta.piece_size(i)

    def segments(self, offset: int, length: int) -> List[Tuple[int, int, int, int]]:
        """(fd, file_offset, length, file_index) for a storage byte range."""
        return [(self.fds[idx], foff, ln, idx) for idx, foff, ln in self.meta.file_spans(offset, length)]

    @contextmanager
    def _use(self) -> Iterator[None]:
        with self._cv:
            if self._closed:
                raise OSError(errno.EBADF, "torrent storage is closed")
            self._users += 1
        try:
            yield
        finally:
            with self._cv:
                self._users -= 1
                if not self._users:
                    self._cv.notify_all()

    def write(self, offset: int, data: bytes) -> None:
        mv = memoryview(data)
        pos = 0
        with self._use():
            for fd, foff, ln, _ in self.segments(offset, len(data)):
                chunk = mv[pos:pos + ln]
                while chunk:
                    w = os.pwrite(fd, chunk, foff)
                    chunk = chunk[w:]
                    foff += w
                pos += ln

    def read(self, offset: int, length: int) -> bytes:
        out = bytearray()
        with self._use():
            for fd, foff, ln, _ in self.segments(offset, length):
                while ln > 0:
                    b = os.pread(fd, ln, foff)
                    if not b:
                        raise OSError("short read from torrent storage")
                    out += b
                    foff += len(b)
                    ln -= len(b)
        return bytes(out)

    def read_block(self, piece: int, begin: int, length: int) -> bytes:
        return self.read(piece * self.meta.piece_length + begin, length)

    def verify(self, pieces: Sequence[int], threads: int = 0) -> List[bool]:
        ok = hashing.verify_pieces(self.paths, self.meta.piece_length, self.meta.pieces,
                                   which=list(pieces), threads=threads)
        return [bool(b) for b in ok]

    def recheck(self, backend: str = "auto", threads: int = 0) -> Bitfield:
        """Verify every piece already on disk (resume after a crash)."""
        bf = Bitfield(self.meta.num_pieces)
        if not self.preexisting:
            return bf
        ok = hashing.verify_pieces(self.paths, self.meta.piece_length, self.meta.pieces,
                                   threads=threads, backend=backend)
        for i, v in enumerate(ok):
            if v:
                bf.set(i)
        return bf

    def sync(self) -> None:
        for fd in self.fds:
            try:
                os.fsync(fd)
            except OSError:
                pass

    def close(self, timeout: float = 30.0) -> None:
        """Close the files once no thread is inside write()/read() (bounded wait: one
        piece's pwrite); later calls fail with EBADF instead of touching a reused fd."""
        with self._cv:
            self._closed = True
            idle = self._cv.wait_for(lambda: not self._users, timeout)
            fds, self.fds = self.fds, []
        if not idle:
            # a write still stuck in the kernel after `timeout` (hung disk): leave its fds
            # open - a leaked descriptor is harmless, a closed-and-reused one is not
            return
        for fd in fds:
            try:
                os.close(fd)
            except OSError:
                pass
