"""Process stage (reference lib/process.js:101-122): select the media files to stage."""
from __future__ import annotations

import asyncio
from typing import Any

from .base import Job, Services, Stage
from .select import MediaSelector, NoMediaFilesError, select_from_config


class ProcessStage(Stage):
    name = "process"

    def __init__(self, cfg, services: Services):
        self.cfg = cfg
        self.sv = services

    async def run(self, job: Job) -> Any:
        last = job.last_stage or {}
        root = last["path"]
        if last.get("streamed") and all(s.get("virtual") for s in last["streamed"]):
            # The download stage streamed a single selector-approved file straight to staging
            # (no disk hop); the walk result is that file.
            files = [s["file"] for s in last["streamed"]]
            job.logger.info("found", len(files), "media files (streamed)")
            return {"files": files, "downloadPath": root, "streamed": last["streamed"]}
        job.logger.info("processing directory", root)
        sel: MediaSelector = select_from_config(self.cfg, job.logger)
        files = await asyncio.get_running_loop().run_in_executor(
            None, sel.find, root, job.media.type)
        if not files:
            raise NoMediaFilesError()
        job.logger.info("found", len(files), "media files")
        job.logger.info({"files": files})
        out = {"files": files, "downloadPath": root}
        if last.get("streamed"):   # eagerly staged torrent files: the upload stage skips them
            keep = set(files)      # once: a 10k-file torrent streams 10k entries
            out["streamed"] = [s for s in last["streamed"] if s["file"] in keep]
        return out


async def factory(cfg, services: Services) -> Stage:
    return ProcessStage(cfg, services)
