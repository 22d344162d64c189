"""Eager staging of torrent files while the torrent is still downloading.

The reference runs download -> process -> upload strictly in sequence (lib/main.js:129-140;
SURVEY §2.6 "PP analogue"): nothing is uploaded until the whole torrent is on disk. But the
process stage's answer is already known from the metainfo - ``MediaSelector.find_virtual``
walks the torrent's file list exactly like the on-disk walk - so every selected file can be
staged to its final key ``<id>/original/<b64(name)>`` part by part: a multipart part is sent
(sendfile from the page cache) as soon as all torrent pieces covering its byte range have
been verified. When the download finishes only the last parts are left, so the job takes
~max(download, upload) instead of their sum.

Key ownership follows the reference's serial loop (App. A #10: the last file in walk order
wins a basename collision). The upload stage later skips files listed as ``streamed``.
"""
from __future__ import annotations

import asyncio
import bisect
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set, Tuple

from ..models import keys
from ..net.http import FileRange
from ..stages.base import media_type


@dataclass
class _File:
    path: str
    key: str
    offset: int                 # storage offset of the file's first byte
    size: int
    parts: List[Tuple[int, int, int]]            # (number, file offset, length)
    upload_id: str = ""
    etags: Dict[int, str] = field(default_factory=dict)
    scheduled: Set[int] = field(default_factory=set)
    fd: int = -1
    lock: asyncio.Lock = field(default_factory=asyncio.Lock)
    single: bool = False


class EagerUploader:
    def __init__(self, session, job, cfg, sv, selected: List[str]):
        self.s = session
        self.job = job
        self.cfg = cfg
        self.sv = sv
        self.s3 = sv.s3
        self.bucket = cfg.s3.bucket
        meta = session.meta
        self.plen = meta.piece_length
        local = meta.local_files(session.root)
        index = {os.path.abspath(p): i for i, (p, _) in enumerate(local)}
        owner: Dict[str, str] = {}
        for f in selected:
            owner[keys.object_key(job.id, f)] = f        # later file wins the key
        self.files: List[_File] = []
        for key, f in owner.items():
            fi = index[os.path.abspath(f)]
            size = meta.files[fi].length
            single = size <= self.s3.multipart_threshold
            # piece-aligned parts: a part is ready as soon as ITS pieces are verified
            parts = [(1, 0, size)] if single else \
                self.s3.plan_parts(size, meta.files[fi].offset, self.plen)
            self.files.append(_File(f, key, meta.files[fi].offset, size, parts, single=single))
        # by torrent offset, for on_piece's bisect (files never overlap, so the ends are
        # sorted too): per verified piece only the files it touches are looked at
        self._by_off = sorted(self.files, key=lambda f: (f.offset, f.size))
        self._ends = [f.offset + f.size for f in self._by_off]
        self.sem = asyncio.Semaphore(max(1, cfg.s3.max_inflight_parts * 2))
        self.tasks: List[asyncio.Task] = []
        self.error: Optional[BaseException] = None
        self.uploaded_bytes = 0
        self.upload_s = 0.0          # summed part-upload time (with the semaphore held)

    # ---------------------------------------------------------------- readiness
    def _ready(self, f: _File, off: int, ln: int) -> bool:
        if ln == 0:
            return True   # empty file: nothing to wait for
        a = f.offset + off
        p0, p1 = a // self.plen, (a + ln - 1) // self.plen
        have = self.s.have
        return all(i in have for i in range(p0, p1 + 1))

    def start(self) -> None:
        for f in self.files:
            for num, off, ln in f.parts:
                self._maybe(f, num, off, ln)

    def on_piece(self, idx: int) -> None:
        lo, hi = idx * self.plen, idx * self.plen + self.s.meta.piece_size(idx)
        for k in range(bisect.bisect_right(self._ends, lo), len(self._by_off)):
            f = self._by_off[k]
            if f.offset >= hi:
                break
            if f.offset + f.size <= lo:
                continue
            for num, off, ln in f.parts:
                a = f.offset + off
                if a < hi and a + ln > lo:
                    self._maybe(f, num, off, ln)

    def _maybe(self, f: _File, num: int, off: int, ln: int) -> None:
        if num in f.scheduled or self.error is not None or not self._ready(f, off, ln):
            return
        f.scheduled.add(num)
        t = asyncio.get_running_loop().create_task(self._upload(f, num, off, ln))
        self.tasks.append(t)

    # ---------------------------------------------------------------- transfers
    async def _upload(self, f: _File, num: int, off: int, ln: int) -> None:
        try:
            async with self.sem:
                t0 = time.perf_counter()
                if f.fd < 0:
                    f.fd = os.open(f.path, os.O_RDONLY | getattr(os, "O_CLOEXEC", 0))
                if f.single:
                    body = FileRange(f.fd, 0, f.size) if f.size else b""
                    ct = media_type(self.cfg, f.path)
                    await self.s3._request("PUT", self.bucket, f.key, body=body,
                                           headers={"content-type": ct} if ct else None)
                    f.etags[num] = "single"
                else:
                    async with f.lock:
                        if not f.upload_id:
                            f.upload_id = await self.s3.create_multipart_upload(
                                self.bucket, f.key, media_type(self.cfg, f.path),
                                checksum=self.s3.want_checksum())
                    f.etags[num] = await self.s3.upload_part(self.bucket, f.key, f.upload_id, num,
                                                             FileRange(f.fd, off, ln))
                self.uploaded_bytes += ln
                self.upload_s += time.perf_counter() - t0
        except asyncio.CancelledError:
            raise                     # abort(): the job is being torn down already
        except BaseException as e:
            # Surfaced by finish(), and at once through the session: without that a part
            # that failed early (S3 down, 4xx) would only fail the job after the rest of a
            # possibly multi-GB torrent had been downloaded for nothing.
            if self.error is None:
                self.error = e
                self.s.fail(e)

    async def finish(self) -> List[dict]:
        """After the download completed: send whatever is left, complete every multipart
        upload, return the ``streamed`` entries for the upload stage."""
        self.start()   # anything not triggered yet (e.g. pieces completed before start)
        while True:
            pending = [t for t in self.tasks if not t.done()]
            if not pending:
                break
            await asyncio.gather(*pending, return_exceptions=True)
        if self.error is not None:
            await self.abort()
            raise self.error
        out = []
        for f in self.files:
            missing = [n for n, _, _ in f.parts if n not in f.etags]
            if missing:
                await self.abort()
                raise RuntimeError(f"eager upload of {f.path}: parts {missing[:5]} never ready")
            if not f.single:
                await self.s3.complete_multipart_upload(
                    self.bucket, f.key, f.upload_id, [(n, f.etags[n]) for n, _, _ in f.parts])
            out.append({"file": f.path, "key": f.key, "size": f.size})
        self._close_fds()
        return out

    async def abort(self) -> None:
        for t in self.tasks:
            t.cancel()
        await asyncio.gather(*self.tasks, return_exceptions=True)
        for f in self.files:
            if f.upload_id:
                try:
                    await self.s3.abort_multipart_upload(self.bucket, f.key, f.upload_id)
                except Exception:
                    pass
        self._close_fds()

    def _close_fds(self) -> None:
        for f in self.files:
            if f.fd >= 0:
                os.close(f.fd)
                f.fd = -1
