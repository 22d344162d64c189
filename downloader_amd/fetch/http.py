"""HTTP(S) source (reference ``methods.http``, lib/download.js:134-167).

Reference behaviour kept: output file = ``basename(URL.pathname)`` with the query dropped and no
percent-decoding (lib/download.js:139-141); a pathname whose ``path.parse().ext`` is exactly
``.torrent`` chains to the torrent backend (lib/download.js:143-155).

Fixed: non-2xx responses fail the job, stream errors reject, the byte
count is checked against Content-Length, an empty basename falls back to ``index``.

Added: parallel Range GETs (``http_streams``) when the origin advertises ``Accept-Ranges:
bytes`` and the body is large, a bytes/s stall floor, and zero-copy splice() into the staging
file through the native transport.
"""
from __future__ import annotations

import asyncio
import os
import posixpath
import time
from typing import Optional, Tuple
from urllib.parse import urlsplit

from ..net.http import FileSink, HttpError, Progress, TransportSet
from ..stages.select import node_extname
from ..utils.log import Logger, NullLogger


class HttpDownloadError(Exception):
    pass


def output_name(url: str) -> str:
    name = posixpath.basename(urlsplit(url).path)
    return name or "index"


def is_torrent_url(url: str) -> bool:
    return node_extname(posixpath.basename(urlsplit(url).path)) == ".torrent"


async def _watch(progress: Progress, min_rate: float, window: float, task: asyncio.Task) -> None:
    last_b, last_t = progress.bytes, time.monotonic()
    while not task.done():
        await asyncio.sleep(min(1.0, window / 4))
        now = time.monotonic()
        if now - last_t >= window:
            b = progress.bytes
            if (b - last_b) / (now - last_t) < min_rate:
                progress.cancel()
                task.cancel()
                return
            last_b, last_t = b, now


async def probe(t: TransportSet, url: str) -> Tuple[int, bool]:
    """HEAD -> (content_length or -1, accepts byte ranges)."""
    try:
        r = await t.request("HEAD", url, expect_body=False)
    except Exception:
        return -1, False
    if not r.ok:
        return -1, False
    cl = r.header("content-length")
    return (int(cl) if cl and cl.isdigit() else -1,
            (r.header("accept-ranges") or "").lower() == "bytes")


async def download_to(t: TransportSet, url: str, path: str, streams: int = 1,
                      min_split: int = 32 << 20, progress: Optional[Progress] = None,
                      min_rate: float = 0.0, stall_window: float = 30.0,
                      logger: Optional[Logger] = None) -> int:
    log = logger or NullLogger()
    progress = progress or Progress()
    size, ranges = (-1, False)
    if streams > 1:
        size, ranges = await probe(t, url)
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | getattr(os, "O_CLOEXEC", 0), 0o644)
    try:
        if streams > 1 and ranges and size >= 2 * min_split:
            n = int(min(streams, size // min_split))
            step = (size + n - 1) // n
            os.ftruncate(fd, size)
            log.debug("parallel range download", streams=n, size=size)

            async def part(off: int, ln: int) -> int:
                r = await t.request("GET", url, headers=[("Range", f"bytes={off}-{off + ln - 1}")],
                                    sink=FileSink(fd, off, ln), progress=progress)
                if r.status != 206:
                    raise HttpDownloadError(f"range request got HTTP {r.status}")
                if r.written != ln:
                    raise HttpDownloadError(f"short range body {r.written} != {ln}")
                return r.written

            coro = asyncio.gather(*(part(o, min(step, size - o)) for o in range(0, size, step)))
            task = asyncio.ensure_future(coro)
            written = sum(await _guard(task, progress, min_rate, stall_window))
        else:
            task = asyncio.ensure_future(t.request("GET", url, sink=FileSink(fd, 0),
                                                   progress=progress))
            r = await _guard(task, progress, min_rate, stall_window)
            if not r.ok:
                raise HttpDownloadError(f"GET {url} -> HTTP {r.status} {r.reason}")
            cl = r.header("content-length")
            if cl and cl.isdigit() and int(cl) != r.written:
                raise HttpDownloadError(f"truncated body: {r.written} of {cl} bytes")
            written = r.written
    finally:
        os.close(fd)
    return written


async def _guard(task: asyncio.Future, progress: Progress, min_rate: float, window: float):
    if min_rate <= 0:
        return await task
    w = asyncio.ensure_future(_watch(progress, min_rate, window, task))  # type: ignore[arg-type]
    try:
        return await task
    except asyncio.CancelledError:
        if progress.cancelled:
            raise HttpDownloadError(f"download below {min_rate:.0f} B/s for {window:.0f}s")
        raise
    finally:
        w.cancel()


async def fetch_bytes(t: TransportSet, url: str, limit: int = 64 << 20) -> bytes:
    r = await t.request("GET", url)
    if not r.ok:
        raise HttpError(f"GET {url} -> HTTP {r.status}", r.status, r.body)
    if len(r.body) > limit:
        raise HttpError("body too large", r.status)
    return r.body
