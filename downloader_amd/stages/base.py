"""Stage-factory contract and per-job state.

Reference contract: each stage module exports ``async (config, emitter, logger) => async job =>
result`` (lib/download.js:30,230; lib/process.js:101-103; lib/upload.js:14,17), is resolved by
name from the list ``['download','process','upload']`` (lib/main.js:28-32,102), must return a
function (lib/main.js:107-110), and each stage receives the message plus ``lastStage`` = the
previous stage's return value (lib/main.js:131-133).

Here a factory is ``async (config, services) -> Stage`` and is built ONCE per worker (App. A
#4: the reference re-initialises stages per message but shares module globals between jobs).
All per-job state lives on ``Job`` (App. A #3/#18: no module globals, per-attempt dirs).
"""
from __future__ import annotations

import asyncio
from dataclasses import dataclass, field
from typing import Any, Awaitable, Callable, Dict, List

from ..models import api, keys
from ..utils.log import Logger, NullLogger


class StageError(Exception):
    code: str = "ERRSTAGE"


class DownloadStalled(StageError):
    """``err.code === 'ERRDLSTALL'`` (lib/download.js:96): the job is acked and dropped."""
    code = "ERRDLSTALL"

    def __init__(self, msg: str = "Download stalled."):
        super().__init__(msg)


class ProtocolNotSupported(StageError):
    code = "ERRPROTO"

    def __init__(self) -> None:
        super().__init__("Protocol not supported.")


class EventEmitter:
    """Per-job event bus handed to every stage (lib/main.js:81). The reference emits only
    ``progress`` and nothing listens; here listeners may subscribe (metrics, tests)."""

    def __init__(self) -> None:
        self._l: Dict[str, List[Callable[..., None]]] = {}

    def on(self, ev: str, fn: Callable[..., None]) -> None:
        self._l.setdefault(ev, []).append(fn)

    def emit(self, ev: str, *args: Any) -> None:
        for fn in list(self._l.get(ev, ())):
            fn(*args)


@dataclass
class Job:
    msg: Any                      # api.Download
    media: Any                    # api.Media
    logger: Logger = field(default_factory=NullLogger)
    emitter: EventEmitter = field(default_factory=EventEmitter)
    last_stage: Any = None
    attempt: int = 0
    attempt_id: str = ""
    headers: Dict[str, Any] = field(default_factory=dict)
    cancel: asyncio.Event = field(default_factory=asyncio.Event)
    stats: Dict[str, Any] = field(default_factory=dict)
    jobdir: Any = None            # stages.jobdir.JobDir claimed by the download stage

    @property
    def id(self) -> str:
        return self.media.id

    # reference-style camelCase view of the previous result
    @property
    def lastStage(self) -> Any:  # noqa: N802
        return self.last_stage


StageFn = Callable[[Job], Awaitable[Any]]


class Stage:
    name = "stage"

    async def run(self, job: Job) -> Any:
        raise NotImplementedError

    async def __call__(self, job: Job) -> Any:
        return await self.run(job)

    async def close(self) -> None:
        pass


@dataclass
class Services:
    """Shared handles given to stage factories (replaces ``global.telem`` etc.)."""
    config: Any
    telemetry: Any
    s3: Any
    transports: Any
    metrics: Any = None
    tracer: Any = None
    logger: Logger = field(default_factory=NullLogger)
    extra: Dict[str, Any] = field(default_factory=dict)


DOWNLOADING = api.STATUS_DOWNLOADING


async def ensure_staging_bucket(sv: Services) -> None:
    """``bucketExists``/``makeBucket('triton-staging')`` (lib/upload.js:29-31), once per worker."""
    if sv.extra.get("bucket_ready"):
        return
    lock = sv.extra.setdefault("bucket_lock", asyncio.Lock())
    async with lock:
        if not sv.extra.get("bucket_ready"):
            await sv.s3.ensure_bucket(sv.config.s3.bucket)
            sv.extra["bucket_ready"] = True


def media_type(cfg, path: str) -> str:
    """Content-Type for a staged file: by extension like minio-js ``fPutObject``
    (``s3.content_type_by_extension``), else "" (S3 then stores application/octet-stream)."""
    return keys.content_type(path) if cfg.s3.content_type_by_extension else ""
