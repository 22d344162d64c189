"""Torrent download backend with the reference's watchdog semantics (lib/download.js:43-123).

* metadata must arrive within ``torrent_metadata_timeout_s`` (240 s) or the job fails with
  ``Metadata fetch stalled`` (lib/download.js:47-50) -> ERRORED + retry;
* every ``progress_interval_s`` (30 s) progress is sampled and, when ``floor(pct/2)`` changed,
  emitted as DOWNLOADING progress (lib/download.js:78-88);
* every ``torrent_stall_timeout_s`` (240 s) a progress that did not move raises
  ``DownloadStalled`` (``ERRDLSTALL``, lib/download.js:90-101) -> the job is acked and dropped;
* on success or failure the session is always removed (App. A #7: the reference leaks the
  stall interval and the torrent on the stall path).

``uri`` may be a magnet link, a bare infohash (40 hex / 32 base32 characters, which
webtorrent's parse-torrent accepts: it becomes a magnet with the DHT and
``download.torrent_default_trackers`` as sources), an http(s) URL of a ``.torrent`` (the
reference's ``.torrent``-over-HTTP chain, lib/download.js:143-155) or a local ``.torrent``
path.

A ``.torrent`` whose only source is webseeds is staged by ``torrent/stream.py`` (webseed ->
S3 relay with in-flight piece verification, no disk) under the same watchdogs; everything
else runs a ``TorrentSession`` into the job directory, with eager staging of selected files.
"""
from __future__ import annotations

import asyncio
import math
import os
import time
from typing import Awaitable, Callable, List, Optional

from ..fetch.http import fetch_bytes
from ..stages.base import DOWNLOADING, DownloadStalled, Job, Services
from .client import TorrentClient
from .magnet import parse_magnet, torrent_id_uri
from .metainfo import Metainfo, parse_torrent
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


async def load_metainfo(uri: str, sv: Services) -> Optional[Metainfo]:
    """The metainfo of a ``.torrent`` source (URL or path); None for a magnet link."""
    if uri.startswith("magnet:"):
        return None
    if uri.startswith(("http://", "https://")):
        data = await fetch_bytes(sv.transports, uri)
    elif os.path.isfile(uri):
        with open(uri, "rb") as f:
            data = f.read()
    else:
        raise ValueError(f"unsupported torrent source {uri[:40]!r}")
    return parse_torrent(data)


async def open_session(client: TorrentClient, uri: str, path: str, sv: Services,
                       meta: Optional[Metainfo] = None) -> TorrentSession:
    if uri.startswith("magnet:"):
        return await client.add_magnet(parse_magnet(uri), path)
    return await client.add_torrent(meta or await load_metainfo(uri, sv), path)


def virtual_selection(meta: Metainfo, job: Job, path: str, cfg) -> Optional[List[str]]:
    """The process stage's answer from the metainfo alone (``find_virtual``), when the job
    directory holds nothing but this torrent's files - so it equals the later disk walk."""
    from ..stages.select import select_from_config
    mine = {os.path.abspath(p) for p, _ in meta.local_files(path)}
    for dp, _, fns in os.walk(path):
        for fn in fns:
            if os.path.abspath(os.path.join(dp, fn)) not in mine:
                return None
    rels = [os.path.relpath(p, path) for p, _ in meta.local_files(path)]
    return select_from_config(cfg).find_virtual(path, rels, job.media.type) or None


def stream_webseeds(meta: Metainfo, job: Job, cfg, sv: Services) -> List[str]:
    """Webseeds to stage from with ``torrent/stream.py``; [] = use a session."""
    d = cfg.download
    if cfg.mode != "tuned" or d.torrent_stream == "off" or not d.eager_upload \
            or not d.torrent_enable_webseeds:
        return []
    if d.torrent_stream == "auto" and ((d.torrent_enable_trackers and meta.trackers())
                                       or job.attempt > 0):
        return []
    seeds = [u for u in meta.url_list if sv.s3.can_relay(u)]
    return seeds if seeds and len(seeds) == len(meta.url_list) else []


async def _start_eager(session: TorrentSession, job: Job, path: str, cfg, sv: Services):
    """Start staging selected files while downloading (torrent.eager)."""
    from ..stages.base import ensure_staging_bucket
    from .eager import EagerUploader
    selected = virtual_selection(session.meta, job, path, cfg)
    if not selected:
        return None
    await ensure_staging_bucket(sv)
    eager = EagerUploader(session, job, cfg, sv, selected)
    session.piece_listeners.append(eager.on_piece)
    eager.start()
    return eager


async def _watched(job: Job, sv: Services, d, progress: Callable[[], float],
                   work: Awaitable) -> None:
    """Run ``work`` under the reference's progress ticker (30 s, floor(pct/2) when changed,
    lib/download.js:78-88) and stall watchdog (240 s without progress -> ERRDLSTALL,
    lib/download.js:90-101)."""
    state = {"last_int": None, "last_progress": None}

    async def ticker() -> None:
        while True:
            await asyncio.sleep(d.progress_interval_s)
            pct = progress() * 100
            job.logger.info("download progress", pct)
            pint = math.floor(pct / 2)
            if pint != state["last_int"]:
                await sv.telemetry.emit_progress(job.id, DOWNLOADING, pint)
            state["last_int"] = pint

    async def watchdog() -> None:
        while True:
            await asyncio.sleep(d.torrent_stall_timeout_s)
            pct = progress() * 100
            job.logger.info("stall check", pct, state["last_progress"])
            if pct == state["last_progress"]:
                raise DownloadStalled()
            state["last_progress"] = pct

    tasks = [asyncio.ensure_future(work), asyncio.ensure_future(ticker()),
             asyncio.ensure_future(watchdog())]
    try:
        done, _ = await asyncio.wait(tasks, return_when=asyncio.FIRST_COMPLETED)
        for t in done:
            t.result()  # propagate DownloadStalled / session errors
    finally:
        for t in tasks:
            t.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)


async def _stream_torrent(meta: Metainfo, seeds: List[str], selected: List[str], job: Job,
                          path: str, cfg, sv: Services, t0: float) -> int:
    from ..stages.base import ensure_staging_bucket
    from .stream import StreamStager
    d = cfg.download
    await ensure_staging_bucket(sv)
    st = StreamStager(meta, job, cfg, sv, selected, path, seeds, d.torrent_stream_parallel)
    job.logger.info("streaming webseed torrent straight to staging", files=len(st.targets),
                    skipped_bytes=st.skipped_bytes())
    out: dict = {}

    async def work() -> None:
        out["streamed"] = await st.run()
    await _watched(job, sv, d, lambda: st.progress, work())
    job.stats.setdefault("streamed", []).extend(out["streamed"])
    job.stats["eager_uploaded_bytes"] = st.total
    job.stats["torrent"] = {"staging": "stream", "webseed_bytes": st.fetched_bytes,
                            "peers": 0, "hash_fails": st.hash_fails,
                            "webseed_fetch_s": round(st.stats["relay_s"], 4),
                            "webseed_verify_s": 0.0, "gap_bytes": st.stats["gap_bytes"],
                            "skipped_bytes": st.skipped_bytes(),
                            "verify": st.stats.get("verify", "host"),
                            **({"verify_fallback": st.stats["verify_fallback"]}
                               if "verify_fallback" in st.stats else {}),
                            "parts": st._n_parts,
                            "gpu_parts": st.stats.get("gpu_parts", 0),
                            "gpu_failures": st.stats.get("gpu_failures", 0),
                            "budget": st.stats.get("budget", {}),
                            "timeline": dict(st.timeline),
                            "timeline_s": {"complete": round(time.perf_counter() - t0, 4)}}
    if sv.metrics is not None:
        sv.metrics.bytes_verified.labels("gpu" if st.stats.get("verify") == "gpu" else "host"
                                         ).inc(st.fetched_bytes)
    return st.fetched_bytes


async def download_torrent(uri: str, job: Job, path: str, cfg, sv: Services,
                           client: Optional[TorrentClient] = None) -> int:
    d = cfg.download
    t0 = time.perf_counter()
    uri = torrent_id_uri(uri, d.torrent_default_trackers)
    meta = await load_metainfo(uri, sv)
    if meta is not None and client is None:
        seeds = stream_webseeds(meta, job, cfg, sv)
        selected = virtual_selection(meta, job, path, cfg) if seeds else None
        if selected:
            return await _stream_torrent(meta, seeds, selected, job, path, cfg, sv, t0)
    from ..stages.space import ensure_space, still_to_write
    if meta is not None:        # .torrent URL: check before any payload is fetched
        ensure_space(path, still_to_write(meta.local_files(path)), d.min_free_bytes)
    client = client or await get_client(cfg, sv)
    session = await open_session(client, uri, path, sv, meta)
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
        if meta is None:        # magnet: metadata came from peers; little payload so far
            ensure_space(path, still_to_write(session.meta.local_files(path)), d.min_free_bytes)
        job.logger.debug("hash", session.info_hash.hex())
        job.logger.debug("files", len(session.meta.files))
        eager = await _start_eager(session, job, path, cfg, sv) if d.eager_upload else None

        # 2) progress ticker + stall watchdog around the transfer
        try:
            await _watched(job, sv, d, lambda: session.progress, session.wait())
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
        job.logger.debug("finished, clearing watchers")
        job.stats["torrent"] = {"staging": "disk", "webseed_bytes": session.webseed_bytes,
                                "peers": session.stats["peers_connected"],
                                "hash_fails": session.stats["hash_fails"],
                                "webseed_fetch_s": round(session.stats["webseed_fetch_s"], 4),
                                "webseed_verify_s": round(session.stats["webseed_verify_s"], 4),
                                "timeline_s": {k: round(v, 4) for k, v in tl.items()}}
        if sv.metrics is not None:
            sv.metrics.bytes_verified.labels("gpu" if session._gpu_verify else "host").inc(
                session.verified_bytes)
        return session.total_bytes()
    finally:
        await client.remove(session)
