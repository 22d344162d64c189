"""Torrent download backend with the reference's watchdog semantics (lib/download.js:43-123).

* metadata must arrive within ``torrent_metadata_timeout_s`` (240 s) or the job fails with
  ``Metadata fetch stalled`` (lib/download.js:47-50) -> ERRORED + retry;
* every ``progress_interval_s`` (30 s) progress is sampled and, when ``floor(pct/2)`` changed,
  emitted as DOWNLOADING progress (lib/download.js:78-88);
* every ``torrent_stall_timeout_s`` (240 s) a progress that did not move raises
  ``DownloadStalled`` (``ERRDLSTALL``, lib/download.js:90-101) -> the job is acked and dropped;
* on success or failure the session is always removed (App. A #7: the reference leaks the
  stall interval and the torrent on the stall path).

``uri`` may be a magnet link, an http(s) URL of a ``.torrent`` (the reference's
``.torrent``-over-HTTP chain, lib/download.js:143-155) or a local ``.torrent`` path.
"""
from __future__ import annotations

import asyncio
import math
import os
import time
from typing import Optional

from ..fetch.http import fetch_bytes
from ..stages.base import DOWNLOADING, DownloadStalled, Job, Services
from .client import TorrentClient
from .magnet import parse_magnet
from .metainfo import parse_torrent
from .session import TorrentSession


class MetadataStalled(Exception):
    def __init__(self) -> None:
        super().__init__("Metadata fetch stalled")


async def get_client(cfg, sv: Services) -> TorrentClient:
    c = sv.extra.get("torrent_client")
    if c is None:
        lock = sv.extra.setdefault("torrent_client_lock", asyncio.Lock())
        async with lock:
            c = sv.extra.get("torrent_client")
            if c is None:
                kw = sv.extra.get("torrent_client_kwargs", {})
                c = TorrentClient.from_config(cfg, transports=sv.transports, **kw)
                await c.start()
                sv.extra["torrent_client"] = c
    return c


async def open_session(client: TorrentClient, uri: str, path: str, sv: Services) -> TorrentSession:
    if uri.startswith("magnet:"):
        return await client.add_magnet(parse_magnet(uri), path)
    if uri.startswith(("http://", "https://")):
        data = await fetch_bytes(sv.transports, uri)
    elif os.path.isfile(uri):
        with open(uri, "rb") as f:
            data = f.read()
    else:
        raise ValueError(f"unsupported torrent source {uri[:40]!r}")
    return await client.add_torrent(parse_torrent(data), path)


async def _start_eager(session: TorrentSession, job: Job, path: str, cfg, sv: Services):
    """Start staging selected files while downloading (torrent.eager) when the job directory
    holds nothing but this torrent's files, so the virtual walk equals the later disk walk."""
    from ..stages.base import ensure_staging_bucket
    from ..stages.select import select_from_config
    from .eager import EagerUploader
    mine = {os.path.abspath(p) for p, _ in session.meta.local_files(path)}
    for dp, _, fns in os.walk(path):
        for fn in fns:
            if os.path.abspath(os.path.join(dp, fn)) not in mine:
                return None
    rels = [os.path.relpath(p, path) for p, _ in session.meta.local_files(path)]
    selected = select_from_config(cfg).find_virtual(path, rels, job.media.type)
    if not selected:
        return None
    await ensure_staging_bucket(sv)
    eager = EagerUploader(session, job, cfg, sv, selected)
    session.piece_listeners.append(eager.on_piece)
    eager.start()
    return eager


async def download_torrent(uri: str, job: Job, path: str, cfg, sv: Services,
                           client: Optional[TorrentClient] = None) -> int:
    d = cfg.download
    t0 = time.perf_counter()
    client = client or await get_client(cfg, sv)
    session = await open_session(client, uri, path, sv)
    # Seconds since the backend was entered: open (metainfo fetched, storage ready), metadata,
    # payload complete and verified, eager staging drained.
    tl = {"open": time.perf_counter() - t0}
    try:
        # 1) metadata stall timer
        meta_wait = asyncio.ensure_future(session.meta_ready.wait())
        fail_wait = asyncio.ensure_future(session.failed.wait())
        try:
            done, _ = await asyncio.wait({meta_wait, fail_wait},
                                         timeout=d.torrent_metadata_timeout_s,
                                         return_when=asyncio.FIRST_COMPLETED)
        finally:
            meta_wait.cancel()
            fail_wait.cancel()
        if session.error is not None:
            raise session.error
        if not session.meta_ready.is_set():
            job.logger.warn("download failed to progress, killing")
            raise MetadataStalled()
        tl["metadata"] = time.perf_counter() - t0
        job.logger.debug("hash", session.info_hash.hex())
        job.logger.debug("files", len(session.meta.files))
        eager = await _start_eager(session, job, path, cfg, sv) if d.eager_upload else None

        # 2) progress ticker + stall watchdog around the transfer
        state = {"last_int": None, "last_progress": None}

        async def ticker() -> None:
            while True:
                await asyncio.sleep(d.progress_interval_s)
                progress = session.progress * 100
                job.logger.info("download progress", progress)
                pint = math.floor(progress / 2)
                if pint != state["last_int"]:
                    await sv.telemetry.emit_progress(job.id, DOWNLOADING, pint)
                state["last_int"] = pint

        async def watchdog() -> None:
            while True:
                await asyncio.sleep(d.torrent_stall_timeout_s)
                progress = session.progress * 100
                job.logger.info("stall check", progress, state["last_progress"])
                if progress == state["last_progress"]:
                    raise DownloadStalled()
                state["last_progress"] = progress

        tasks = [asyncio.ensure_future(session.wait()), asyncio.ensure_future(ticker()),
                 asyncio.ensure_future(watchdog())]
        try:
            done, _ = await asyncio.wait(tasks, return_when=asyncio.FIRST_COMPLETED)
            for t in done:
                t.result()  # propagate DownloadStalled / session errors
            tl["complete"] = time.perf_counter() - t0
            if eager is not None:
                job.stats.setdefault("streamed", []).extend(await eager.finish())
                job.stats["eager_uploaded_bytes"] = eager.uploaded_bytes
                job.stats["eager_upload_s"] = round(eager.upload_s, 4)
                tl["eager_drained"] = time.perf_counter() - t0
        except BaseException:
            if eager is not None:
                await eager.abort()
            raise
        finally:
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
        job.logger.debug("finished, clearing watchers")
        job.stats["torrent"] = {"webseed_bytes": session.webseed_bytes,
                                "peers": session.stats["peers_connected"],
                                "hash_fails": session.stats["hash_fails"],
                                "webseed_fetch_s": round(session.stats["webseed_fetch_s"], 4),
                                "webseed_verify_s": round(session.stats["webseed_verify_s"], 4),
                                "timeline_s": {k: round(v, 4) for k, v in tl.items()}}
        return session.total_bytes()
    finally:
        await client.remove(session)
