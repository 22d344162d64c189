"""Download stage (reference lib/download.js:230-276).

Per job: resolve ``<download_path>/<media.id>`` (relative paths against the project root,
lib/download.js:234-240; plus a per-attempt sub-directory, App. A #18), map the ``SourceType``
enum name to a backend (lib/download.js:243,256), emit progress 0 (:255), run the backend,
emit progress 50 (:272) and return ``{'path': dir}``.
"""
from __future__ import annotations

import asyncio
import hashlib
import os
from typing import Any, Awaitable, Callable, Dict, List

from ..fetch import bucket as bucket_src
from ..fetch import http as http_src
from ..fetch import local as file_src
from ..models import api, keys
from ..net.http import Progress, SourceChanged
from ..net.proxy import ProxyConfig
from ..s3.client import S3Error
from ..utils.aio import gather_strict, run_settled
from ..utils.log import redact_url
from .base import (DOWNLOADING, Job, ProtocolNotSupported, Services, Stage,
                   ensure_staging_bucket, media_type)
from .jobdir import JobDir, dir_name
from .select import select_from_config

# a source that changes version mid-transfer is restarted from its new version this often
# before the job fails (and goes through the broker retry)
SOURCE_RESTARTS = 2

Backend = Callable[[str, Job, str], Awaitable[None]]


def _hostport(endpoint: str) -> str:
    e = endpoint.split("://", 1)[-1].rstrip("/").lower()
    return e if ":" in e.rsplit("]", 1)[-1] else e + ":default"


class DownloadStage(Stage):
    name = "download"

    def __init__(self, cfg, services: Services):
        self.cfg = cfg
        self.sv = services
        self.root = cfg.resolved_download_root()
        self.proxy = ProxyConfig(cfg.download.http_proxy)
        self.methods: Dict[str, Backend] = {
            "torrent": self.torrent,
            "http": self.http,
            "file": self.file,
            "bucket": self.bucket,
        }

    def job_dir(self, job: Job) -> str:
        if not self.cfg.instance.per_attempt_dirs:
            return os.path.join(str(self.root), dir_name(job.id))   # no locking
        if job.jobdir is None:
            job.jobdir = JobDir(str(self.root), job.id)
            job.jobdir.acquire()
        return job.jobdir.path

    def _make_dir(self, job: Job) -> str:
        """Claim and create the job directory (one executor hop per job)."""
        path = self.job_dir(job)
        os.makedirs(path, exist_ok=True)
        return path

    def _count(self, proto: str, n: int) -> None:
        if self.sv.metrics is not None and n:
            self.sv.metrics.bytes_downloaded.labels(proto).inc(n)

    async def run(self, job: Job) -> Any:
        media = job.media
        protocol = api.enum_to_string("SourceType", media.source)
        try:
            path = await asyncio.get_running_loop().run_in_executor(None, self._make_dir, job)
            job.logger.info("created downloadPath", path)
        except OSError as e:
            job.logger.error("Failed to create directory", str(e))
        job.logger.info(f"Trying to download with protocol '{protocol}', the URL "
                        f"'{self._redact(media.sourceURI, protocol)}'")
        await self.sv.telemetry.emit_progress(job.id, DOWNLOADING, 0)
        method = self.methods.get(protocol.lower())
        if method is None:
            raise ProtocolNotSupported()
        try:
            await method(media.sourceURI, job, path)
        except Exception as e:
            job.logger.error("Download error: ", str(e))
            raise
        job.logger.info("finished download")
        await self.sv.telemetry.emit_progress(job.id, DOWNLOADING, 50)
        out: Dict[str, Any] = {"path": path}
        if job.stats.get("streamed"):
            out["streamed"] = job.stats["streamed"]
        return out

    @staticmethod
    def _redact(uri: str, protocol: str) -> str:
        """The source URI as logged: bucket:// secret keys (App. A #19), URL passwords and
        signature/token query values of presigned URLs are masked."""
        if protocol.lower() == "bucket":
            try:
                return bucket_src.parse_bucket_uri(uri).redacted()
            except ValueError:
                return "bucket://<invalid>"
        return redact_url(uri)

    # ------------------------------------------------------------------ backends
    async def http(self, url: str, job: Job, path: str) -> None:
        job.logger.info("http", redact_url(url))
        if http_src.is_torrent_url(url):
            job.logger.info("downloading a .torrent, chaining to torrent downloader")
            await self.torrent(url, job, path)
            return
        d = self.cfg.download
        name = http_src.output_name(url)
        if d.stream_http and await self._stream_http(url, name, job, path):
            return
        out = os.path.join(path, name)
        prog = Progress()
        n = await http_src.download_to(self.sv.transports, url, out, d.http_streams,
                                       d.http_min_split, prog, d.http_min_rate,
                                       min(60.0, d.http_timeout_s), job.logger, self.proxy,
                                       space_reserve=d.min_free_bytes)
        job.stats["downloaded_bytes"] = job.stats.get("downloaded_bytes", 0) + n
        self._count("http", n)

    async def _stream_http(self, url: str, name: str, job: Job, path: str) -> bool:
        """Streaming fast path for a single-file HTTP source: origin -> S3 with no disk hop.

        Applies only when the outcome of the process stage is already known - one top-level
        file whose name the media selector accepts - and the origin reports its size (and
        supports Range for multipart sizes). The object lands under the same key, the
        progress curve and done marker are unchanged; otherwise the disk path runs."""
        s3 = self.sv.s3
        if not s3.can_relay(url, self.proxy) or \
                not select_from_config(self.cfg).accepts_single_file(name):
            return False
        size, ranges, final, validator = await http_src.probe_validated(
            self.sv.transports, url, self.proxy)
        if size <= 0 or (size > s3.multipart_threshold and not ranges) or \
                not s3.can_relay(final, self.proxy):
            return False
        await ensure_staging_bucket(self.sv)
        key = keys.object_key(job.id, name)
        job.logger.info("streaming http source straight to staging", key=key, size=size)
        # big objects: a resume journal, so the job's retry relays only the missing parts
        rmin = int(getattr(self.cfg.s3, "relay_resume_min_bytes", 0) or 0)
        resumable = bool(rmin) and size >= rmin and size > s3.multipart_threshold
        journal = keys.relay_journal_key(job.id, name) if resumable else ""
        keep = resumable and job.attempt < self.cfg.broker.max_retries
        for attempt in range(SOURCE_RESTARTS + 1):
            try:
                # every part GET pinned to the probed version: a mid-job change aborts the
                # upload instead of completing a torn object
                await s3.relay_object(self.cfg.s3.bucket, key, final, size, Progress(),
                                      src_proxy=self.proxy,
                                      content_type=media_type(self.cfg, name), ranges=ranges,
                                      validator=validator, journal=journal,
                                      keep_on_error=keep, stats=job.stats)
                break
            except SourceChanged as e:
                if attempt == SOURCE_RESTARTS:
                    raise
                job.logger.warn("origin changed mid-transfer, restarting from the new version",
                                err=str(e))
                job.stats["source_restarts"] = job.stats.get("source_restarts", 0) + 1
                size, ranges, final, validator = await http_src.probe_validated(
                    self.sv.transports, url, self.proxy)
                if size <= 0 or (size > s3.multipart_threshold and not ranges):
                    raise
        job.stats["downloaded_bytes"] = job.stats.get("downloaded_bytes", 0) + size
        job.stats.setdefault("streamed", []).append(
            {"file": os.path.join(path, name), "key": key, "size": size, "virtual": True})
        self._count("http", size)
        return True

    async def file(self, url: str, job: Job, path: str) -> None:
        if not self.cfg.download.allow_file_urls:
            raise file_src.FileUrlsNotAllowed()
        src = file_src.file_uri_to_path(url)
        out = file_src.target_path(url, path)
        d = self.cfg.download
        if d.stream_file and self.cfg.mode == "tuned" and os.path.isfile(src) and \
                select_from_config(self.cfg).accepts_single_file(os.path.basename(out)):
            # the copy's only reader would be the upload: stage straight from the source file
            # (sendfile), the job directory stays empty (reference: copy, then upload)
            await ensure_staging_bucket(self.sv)
            key = keys.object_key(job.id, out)
            size = os.path.getsize(src)
            job.logger.info("staging local file without a copy", key=key, size=size)
            await self.sv.s3.fput_object(self.cfg.s3.bucket, key, src, progress=Progress(),
                                         content_type=media_type(self.cfg, out))
            job.stats["downloaded_bytes"] = job.stats.get("downloaded_bytes", 0) + size
            job.stats.setdefault("streamed", []).append(
                {"file": out, "key": key, "size": size, "virtual": True})
            self._count("file", size)
            return
        job.logger.debug("file", src, "->", out)
        n = await run_settled(file_src.copy_file, src, out)
        job.stats["downloaded_bytes"] = job.stats.get("downloaded_bytes", 0) + n
        self._count("file", n)

    async def bucket(self, url: str, job: Job, path: str) -> None:
        d = self.cfg.download
        if d.stream_bucket and self.cfg.mode == "tuned" and await self._stream_bucket(url, job,
                                                                                     path):
            return
        prog = Progress()
        files = await bucket_src.fetch_bucket(url, path, secure=d.bucket_secure,
                                              concurrency=d.bucket_concurrency,
                                              logger=job.logger, progress=prog,
                                              native=self.cfg.s3.native_transport,
                                              ssl_verify=self.cfg.tls.verify,
                                              ca_file=self.cfg.tls.ca_file,
                                              native_tls=self.cfg.tls.native)
        n = sum(os.path.getsize(f) for f in files)
        job.stats["downloaded_bytes"] = job.stats.get("downloaded_bytes", 0) + n
        self._count("bucket", n)

    async def _stream_bucket(self, url: str, job: Job, path: str) -> bool:
        """bucket:// fast path: the object listing is the file tree the reference would have
        downloaded (``<dir>/<name minus subFolder>``, lib/download.js:218-226), so the media
        selector runs on it before any byte moves (``find_virtual``); each selected object is
        then relayed source S3 -> staging S3 through a presigned GET (Range parts in
        parallel) with no disk hop, and unselected objects (extras, samples) are never
        fetched. Falls back to the disk path when nothing is selected (the process stage then
        fails as in the reference) or the relay cannot reach both endpoints."""
        from ..s3.client import S3Client
        d = self.cfg.download
        src = bucket_src.parse_bucket_uri(url)
        s3 = self.sv.s3
        client = S3Client(src.endpoint, src.access_key, src.secret_key, secure=d.bucket_secure,
                          transports=self.sv.transports)
        if not s3.can_relay(client.base + "/"):
            return False
        prefix = src.sub_folder.rstrip("/") + "/"
        items = [it for it in await client.list_objects(src.bucket, prefix, recursive=True)
                 if it.name and not it.name.endswith("/")]
        by_path: Dict[str, Any] = {}
        for it in items:
            dst = bucket_src.local_name(path, it.name, src.sub_folder)
            if not bucket_src.inside(path, dst):
                raise ValueError(f"object {it.name!r} escapes the download directory")
            by_path[os.path.abspath(dst)] = it
        rel = [os.path.relpath(p, path) for p in by_path]
        selected = select_from_config(self.cfg).find_virtual(path, rel, job.media.type)
        if not selected:
            return False
        await ensure_staging_bucket(self.sv)
        owner: Dict[str, str] = {}              # key -> winning file (last in walk order)
        for f in selected:
            owner[keys.object_key(job.id, f)] = f
        job.logger.info("streaming bucket source straight to staging", objects=len(items),
                        selected=len(selected), staged=len(owner))
        sem = asyncio.Semaphore(max(1, d.bucket_concurrency))
        prog = Progress()
        # same endpoint and credentials as the staging S3: a server-side copy moves no bytes
        # through this worker at all
        same = (_hostport(src.endpoint) == _hostport(s3.endpoint)
                and src.access_key == s3.access_key and d.bucket_server_copy)
        job.stats["bucket_server_copy"] = same

        # big objects keep a resume journal: the job's retry relays only their missing parts
        rmin = int(getattr(self.cfg.s3, "relay_resume_min_bytes", 0) or 0)
        keep = job.attempt < self.cfg.broker.max_retries
        rstats: Dict[str, int] = {}

        reused: List[str] = []
        halted = []        # set by the first failure: objects not begun yet are not started

        async def one(key: str, f: str) -> None:
            try:
                await stage_one(key, f)
            except Exception:
                halted.append(f)
                raise

        async def stage_one(key: str, f: str) -> None:
            it = by_path[f]
            # the staged object records which source version it holds: a retry of the job
            # skips objects an earlier attempt already staged from the same version
            tag = hashlib.sha1(f"{src.bucket}/{it.name}@{it.etag}".encode()).hexdigest() \
                if it.etag else ""
            async with sem:
                if halted:
                    return
                if tag and job.attempt > 0 and not same:
                    try:
                        info = await s3.head_object(self.cfg.s3.bucket, key)
                        if info.size == it.size and info.meta.get("stager-source") == tag:
                            reused.append(f)
                            return
                    except S3Error:
                        pass
                if same:
                    await s3.copy_object(src.bucket, it.name, self.cfg.s3.bucket, key, it.size,
                                         content_type=media_type(self.cfg, f))
                    return
                resumable = bool(rmin) and it.size >= rmin and it.size > s3.multipart_threshold
                await s3.relay_object(self.cfg.s3.bucket, key,
                                      # every Range part is its own request: the URL must
                                      # outlive the slowest object's last part
                                      client.presign("GET", src.bucket, it.name, 12 * 3600),
                                      it.size, prog,
                                      content_type=media_type(self.cfg, f),
                                      # parts pinned to the listed version (If-Match)
                                      validator=f'"{it.etag}"' if it.etag else "",
                                      journal=keys.relay_journal_key(job.id, f)
                                      if resumable else "",
                                      keep_on_error=resumable and keep, stats=rstats,
                                      meta={"stager-source": tag} if tag else None)
        # one object failing: with a retry still to come, the objects already moving finish
        # (the retry reuses them, and a big one keeps its resumable upload); on the last
        # attempt they are cancelled
        await gather_strict(*(one(k, f) for k, f in owner.items()), cancel=not keep)
        if rstats:
            job.stats["resumed_parts"] = rstats["resumed_parts"]
        if reused:
            job.stats["reused_objects"] = len(reused)
        staged = sum(by_path[f].size for f in owner.values())
        job.stats["downloaded_bytes"] = job.stats.get("downloaded_bytes", 0) + staged
        job.stats.setdefault("streamed", []).extend(
            {"file": f, "key": keys.object_key(job.id, f), "size": by_path[f].size,
             "virtual": True} for f in selected)
        job.stats["bucket_skipped_bytes"] = sum(it.size for it in items) - staged
        self._count("bucket", staged)
        return True

    async def torrent(self, uri: str, job: Job, path: str) -> None:
        from ..torrent.backend import download_torrent
        uri_log = redact_url(uri)
        short = uri_log[:25] + "..." if len(uri_log) > 25 else uri_log
        job.logger.info("url", short)
        n = await download_torrent(uri, job, path, self.cfg, self.sv)
        job.stats["downloaded_bytes"] = job.stats.get("downloaded_bytes", 0) + n
        self._count("torrent", n)

    async def close(self) -> None:
        c = self.sv.extra.pop("torrent_client", None)
        if c is not None:
            await c.close()


async def factory(cfg, services: Services) -> Stage:
    # The torrent backends are imported lazily (a worker that never sees a torrent does not
    # pay for them); import them off the event loop at stage creation instead of inside the
    # first torrent job (~15 ms of module setup on that job's clock).
    await asyncio.get_running_loop().run_in_executor(None, _warm_imports)
    return DownloadStage(cfg, services)


def _warm_imports() -> None:
    import importlib
    for mod in ("..torrent.backend", "..torrent.stream", "..torrent.eager", ".space"):
        importlib.import_module(mod, __package__)
