"""Upload stage (reference lib/upload.js:17-66).

Per job: ensure bucket ``triton-staging`` exists (lib/upload.js:29-31), upload every selected
file to ``<id>/original/<base64(basename)>`` (lib/upload.js:43-45), emit progress
``floor(50 + 50*i/n)`` after each file (lib/upload.js:48-51), write the ``done`` marker with body
``"true"`` (lib/upload.js:55) and remove the job directory (lib/upload.js:60-64).

The reference uploads files strictly one after another; here up to ``s3.concurrent_files``
upload at once (each multipart object additionally runs ``max_inflight_parts`` parts in
parallel). Basename collisions (App. A #10) are resolved exactly like the reference's serial
loop - the LAST file in walk order owns the key - by uploading only that file, and are counted
in ``key_collisions_total``.
"""
from __future__ import annotations

import asyncio
import os
from typing import Any, Dict, List

from ..models import keys
from ..utils.aio import gather_strict
from ..net.http import Progress
from .base import DOWNLOADING, Job, Services, Stage, ensure_staging_bucket, media_type
from .jobdir import get_reaper


class UploadStage(Stage):
    name = "upload"

    def __init__(self, cfg, services: Services):
        self.cfg = cfg
        self.sv = services

    async def ensure_bucket(self) -> None:
        await ensure_staging_bucket(self.sv)

    async def run(self, job: Job) -> Any:
        last = job.last_stage or {}
        files = last.get("files")
        download_path = last.get("downloadPath")
        streamed = {s["file"]: s for s in last.get("streamed", [])}
        if not isinstance(files, list):
            raise TypeError(f"Invalid files data type, expected array, got '{type(files).__name__}'")
        job.logger.info("starting file upload")
        await self.ensure_bucket()
        bucket = self.cfg.s3.bucket
        media_id = job.id
        n = len(files)

        # Resolve key ownership first (last file in walk order wins, like the serial loop).
        owner: Dict[str, int] = {}
        for i, f in enumerate(files):
            k = keys.object_key(media_id, f)
            if k in owner:
                job.logger.warn("staging key collision; later file wins", key=k,
                                dropped=files[owner[k]], kept=f)
                if self.sv.metrics is not None:
                    self.sv.metrics.key_collisions.inc()
            owner[k] = i
        for f in files:
            if f not in streamed and not os.path.exists(f):
                job.logger.error("failed to upload file, not found")
                raise FileNotFoundError(f"{f} not found.")

        done = 0
        sem = asyncio.Semaphore(max(1, self.cfg.s3.concurrent_files))
        uploaded: List[int] = []

        async def one(i: int, f: str) -> None:
            nonlocal done
            k = keys.object_key(media_id, f)
            async with sem:
                if owner[k] == i:
                    job.logger.info("upload", os.path.basename(f))
                    prog = Progress()
                    if f in streamed:   # already staged by the streaming download path
                        size = streamed[f]["size"]
                    else:
                        await self.sv.s3.fput_object(bucket, k, f, progress=prog,
                                                     resume=self.cfg.s3.resume_uploads,
                                                     content_type=media_type(self.cfg, f))
                        size = os.path.getsize(f)
                    uploaded.append(size)
                    if self.sv.metrics is not None:
                        self.sv.metrics.bytes_uploaded.inc(size)
            # progress after each finished file (lib/upload.js:48-51): emitted outside any
            # lock - telemetry only queues the event (service/telemetry.py)
            done += 1
            pct = int(done / n * 50 + 50)
            await self.sv.telemetry.emit_progress(media_id, DOWNLOADING, pct)
            job.emitter.emit("progress", pct)

        await gather_strict(*(one(i, f) for i, f in enumerate(files)))
        job.stats["uploaded_bytes"] = sum(uploaded)

        await self.sv.s3.put_object(bucket, keys.done_key(media_id), keys.DONE_BODY)
        job.logger.info("finished uploading all files")
        if download_path:
            try:
                # background: rename into .trash now (the job id's path is free when the
                # stage returns), unlink later; reference mode: delete inline. Either way
                # the syscalls run off the event loop.
                await asyncio.get_running_loop().run_in_executor(
                    None, get_reaper(self.sv).reap, download_path)
            except (OSError, ValueError) as e:
                job.logger.warn("err", f"failed to clean up directory: {e}")
        return {"files": files, "keys": sorted(owner), "bytes": sum(uploaded)}


async def factory(cfg, services: Services) -> Stage:
    return UploadStage(cfg, services)
