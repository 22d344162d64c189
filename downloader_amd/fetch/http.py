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
import json
import os
import posixpath
import time
from typing import Optional, Tuple
from urllib.parse import urlsplit

from ..net.http import FileSink, HttpError, Progress, SourceChanged, TransportSet, pin_headers
from ..net.proxy import ProxyConfig
from ..stages.select import node_extname
from ..utils.aio import gather_strict
from ..utils.log import Logger, NullLogger, redact_url


class HttpDownloadError(Exception):
    pass


def output_name(url: str) -> str:
    """``basename(new URL(url).pathname)`` (lib/download.js:139-141). The WHATWG parser drops
    ``.`` / ``..`` segments (also as ``%2e``), so Node never yields them as a basename: a path
    that ends in one resolves to a directory, i.e. an empty name -> ``index`` here."""
    name = posixpath.basename(urlsplit(url).path)
    if name.lower().replace("%2e", ".") in (".", ".."):
        name = ""
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


async def probe(t: TransportSet, url: str, proxy: Optional[ProxyConfig] = None
                ) -> Tuple[int, bool, str]:
    """HEAD (redirects followed) -> (content_length or -1, accepts byte ranges, final URL)."""
    size, ranges, final, _ = await probe_validated(t, url, proxy)
    return size, ranges, final


async def probe_validated(t: TransportSet, url: str, proxy: Optional[ProxyConfig] = None
                          ) -> Tuple[int, bool, str, str]:
    """``probe`` plus the response's validator: a strong ``ETag``, else ``Last-Modified``
    ("" when the origin gives neither). Partial data is only resumed under the same one."""
    try:
        r = await t.request("HEAD", url, expect_body=False, proxy=proxy)
    except Exception:
        return -1, False, url, ""
    if not r.ok:
        return -1, False, url, ""
    cl = r.header("content-length")
    etag = (r.header("etag") or "").strip()
    validator = etag if etag and not etag.startswith("W/") else \
        ("lm:" + r.header("last-modified") if r.header("last-modified") else "")
    return (int(cl) if cl and cl.isdigit() else -1,
            (r.header("accept-ranges") or "").lower() == "bytes", r.url or url, validator)


SOURCE_RESTARTS = 2


async def download_to(t: TransportSet, url: str, path: str, streams: int = 1,
                      min_split: int = 32 << 20, progress: Optional[Progress] = None,
                      min_rate: float = 0.0, stall_window: float = 30.0,
                      logger: Optional[Logger] = None,
                      proxy: Optional[ProxyConfig] = None,
                      space_reserve: Optional[int] = None) -> int:
    """Download ``url`` to ``path`` through ``path + '.part'`` (renamed when complete).

    Every GET is pinned to the version the probe saw (``pin_headers``: If-Match /
    If-Unmodified-Since, plus If-Range on Range requests): parallel ranges, a resumed tail
    and the whole-file GET are all of one version. When the origin changes mid-transfer the
    partial data is dropped and the file is fetched again from the new version (at most
    ``SOURCE_RESTARTS`` times), never stitched from two.

    Resume (the reference restarts from byte 0): the journal
    ``path + '.part.ranges'`` records the origin's validator (strong ETag / Last-Modified),
    its size and the completed byte ranges; a later attempt with the same job directory skips
    those ranges, or continues a single-stream transfer from the ``.part`` length - but only
    when the origin still reports the same validator and size (otherwise the partial data
    belongs to another version of the file and is discarded). A complete ``path`` of the
    advertised size is reused as is.

    ``space_reserve`` (not None): fail with ENOSPC before fetching when the filesystem cannot
    hold what is still to be written plus that reserve (``stages/space.py``)."""
    log = logger or NullLogger()
    progress = progress or Progress()
    for attempt in range(SOURCE_RESTARTS + 1):
        try:
            return await _download_once(t, url, path, streams, min_split, progress, min_rate,
                                        stall_window, log, proxy, space_reserve)
        except SourceChanged as e:
            if attempt == SOURCE_RESTARTS:
                raise HttpDownloadError(f"origin kept changing during the download: {e}") from e
            log.warn("origin changed mid-download, restarting from the new version", err=str(e))
            for stale in (path + ".part", path + ".part.ranges"):
                try:
                    os.unlink(stale)
                except FileNotFoundError:
                    pass
    raise AssertionError("unreachable")


async def _download_once(t: TransportSet, url: str, path: str, streams: int, min_split: int,
                         progress: Progress, min_rate: float, stall_window: float, log: Logger,
                         proxy: Optional[ProxyConfig], space_reserve: Optional[int]) -> int:
    size, ranges, url, validator = await probe_validated(t, url, proxy)   # later GETs: final URL
    part_path, state_path = path + ".part", path + ".part.ranges"
    if size >= 0 and os.path.isfile(path) and os.path.getsize(path) == size:
        j = _load_journal(state_path)
        if j and validator and j["validator"] == validator and j["size"] == size:
            log.info("resume: file already complete", path=path)
            return 0
        os.unlink(path)                      # another version of the file: fetch again
    journal = _load_journal(state_path) if os.path.exists(part_path) else None
    resumable = bool(journal and validator and journal["validator"] == validator
                     and journal["size"] == size)
    if journal and not resumable:
        log.info("resume: origin changed or unvalidated, restarting", path=path)
    done = list(journal["ranges"]) if resumable else []
    if space_reserve is not None and size > 0:
        from ..stages.space import allocated, ensure_space
        held = allocated(part_path) if resumable else 0
        ensure_space(os.path.dirname(path) or ".", size - held, space_reserve)
    _save_journal(state_path, validator, size, done)
    fd = os.open(part_path, os.O_WRONLY | os.O_CREAT | getattr(os, "O_CLOEXEC", 0), 0o644)
    written = 0
    try:
        if streams > 1 and ranges and size >= 2 * min_split:
            n = int(min(streams, size // min_split))
            step = (size + n - 1) // n
            os.ftruncate(fd, size)
            plan = [(o, min(step, size - o)) for o in range(0, size, step)]
            todo = [(o, ln) for o, ln in plan if [o, ln] not in done]
            if len(todo) < len(plan):
                log.info("resume: skipping completed ranges", done=len(plan) - len(todo))
            log.debug("parallel range download", streams=n, size=size)

            async def part(off: int, ln: int) -> int:
                hdrs = [("Range", f"bytes={off}-{off + ln - 1}")] + pin_headers(validator, True)
                r = await t.request("GET", url, headers=hdrs, sink=FileSink(fd, off, ln),
                                    progress=progress, proxy=proxy)
                if r.status == 412 or (validator and r.status == 200):
                    raise SourceChanged(f"range {off}+{ln}: HTTP {r.status}", r.status)
                if r.status != 206:
                    raise HttpDownloadError(f"range request got HTTP {r.status}")
                if r.written != ln:
                    raise HttpDownloadError(f"short range body {r.written} != {ln}")
                done.append([off, ln])
                _save_journal(state_path, validator, size, done)
                return r.written

            task = asyncio.ensure_future(gather_strict(*(part(o, ln) for o, ln in todo)))
            written = sum(await _guard(task, progress, min_rate, stall_window))
        else:
            have = os.fstat(fd).st_size if (resumable and ranges and size > 0 and not done) \
                else 0
            if not (0 < have < size):
                have = 0
                os.ftruncate(fd, 0)
            hdrs = [("Range", f"bytes={have}-")] if have else []
            hdrs += pin_headers(validator, bool(have))
            if have:
                log.info("resume: continuing partial download", offset=have, size=size)
            task = asyncio.ensure_future(t.request("GET", url, headers=hdrs, proxy=proxy,
                                                   sink=FileSink(fd, have), progress=progress))
            r = await _guard(task, progress, min_rate, stall_window)
            if r.status == 412 or (have and validator and r.status == 200):
                raise SourceChanged(f"GET from {have}: HTTP {r.status}", r.status)
            if not r.ok or (have and r.status != 206):
                raise HttpDownloadError(f"GET {redact_url(url)} -> HTTP {r.status} {r.reason}")
            cl = r.header("content-length")
            if cl and cl.isdigit() and int(cl) != r.written:
                raise HttpDownloadError(f"truncated body: {r.written} of {cl} bytes")
            written = r.written
            if size >= 0 and have + written != size:
                raise HttpDownloadError(f"size mismatch: {have + written} != {size}")
    finally:
        os.close(fd)
    os.replace(part_path, path)
    # the journal stays (ranges = the whole file): a retry whose upload failed reuses the
    # complete file only if the origin still reports this version
    _save_journal(state_path, validator, size, [[0, size]])
    return written


def _load_journal(p: str) -> Optional[dict]:
    """{"validator", "size", "ranges"} or None (missing, unreadable, or a journal without a
    validator - nothing to check partial data against)."""
    try:
        with open(p, "r", encoding="utf-8") as f:
            v = json.load(f)
    except (OSError, ValueError):
        return None
    if not isinstance(v, dict) or not v.get("validator"):
        return None
    rng = v.get("ranges")
    return {"validator": str(v["validator"]), "size": v.get("size"),
            "ranges": [list(x) for x in rng] if isinstance(rng, list) else []}


def _save_journal(p: str, validator: str, size: int, done: list) -> None:
    tmp = p + ".tmp"
    with open(tmp, "w", encoding="utf-8") as f:
        json.dump({"validator": validator, "size": size, "ranges": done}, f)
    os.replace(tmp, p)


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
        raise HttpError(f"GET {redact_url(url)} -> HTTP {r.status}", r.status, r.body)
    if len(r.body) > limit:
        raise HttpError("body too large", r.status)
    return r.body
