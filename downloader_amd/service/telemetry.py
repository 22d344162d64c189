"""Job status / progress telemetry (the reference's ``triton-core/telemetry``).

Reference calls: ``telem.emitStatus(jobId, 2)`` on receipt (lib/main.js:68), ``emitStatus(jobId,
6)`` on failure (:149) and ``emitProgress(id, DOWNLOADING, pct)`` with the curve 0 -> torrent
floor(pct/2) every 30 s -> 50 -> floor(50 + 50*i/n) per uploaded file (lib/download.js:255,
78-88,272; lib/upload.js:48-51). The wire format inside triton-core is INFERRED to be protobuf
over the broker; here ``api.TelemetryStatus`` / ``api.TelemetryProgress`` are published on
two queues. ``history`` keeps the most recent emitted events (bounded: a long-running worker
must not grow with every job) for tests, the bench and debugging.
"""
from __future__ import annotations

import time
from collections import deque
from typing import Deque, List, Optional, Tuple

from ..broker.base import Broker
from ..models import api
from ..utils.log import Logger, NullLogger


class Telemetry:
    def __init__(self, broker: Optional[Broker], status_queue: str = "v1.telemetry.status",
                 progress_queue: str = "v1.telemetry.progress", enabled: bool = True,
                 logger: Optional[Logger] = None, keep_history: bool = True,
                 history_max: int = 100_000):
        self.broker = broker
        self.status_queue = status_queue
        self.progress_queue = progress_queue
        self.enabled = enabled and broker is not None
        self.log = logger or NullLogger()
        self.keep_history = keep_history
        self.history: Deque[Tuple[str, str, int, Optional[int], float]] = \
            deque(maxlen=history_max)

    @classmethod
    def from_config(cls, cfg, broker: Optional[Broker], logger: Optional[Logger] = None):
        t = cfg.telemetry
        return cls(broker, t.status_queue, t.progress_queue, t.enabled, logger)

    async def connect(self) -> None:
        if self.enabled:
            await self.broker.declare(self.status_queue)
            await self.broker.declare(self.progress_queue)

    async def emit_status(self, media_id: str, status: int) -> None:
        if self.keep_history:
            self.history.append(("status", media_id, int(status), None, time.time()))
        if not self.enabled:
            return
        msg = api.TelemetryStatus(mediaId=media_id, status=int(status))
        try:
            await self.broker.publish(self.status_queue, api.encode(msg), confirm=False)
        except Exception as e:  # telemetry must never fail a job
            self.log.warn("failed to emit status", err=str(e))

    async def emit_progress(self, media_id: str, status: int, progress: int) -> None:
        if self.keep_history:
            self.history.append(("progress", media_id, int(status), int(progress), time.time()))
        if not self.enabled:
            return
        msg = api.TelemetryProgress(mediaId=media_id, status=int(status), progress=int(progress))
        try:
            await self.broker.publish(self.progress_queue, api.encode(msg), confirm=False)
        except Exception as e:
            self.log.warn("failed to emit progress", err=str(e))

    # reference-style aliases
    emitStatus = emit_status
    emitProgress = emit_progress

    def progress_of(self, media_id: str) -> List[int]:
        return [p for k, m, _, p, _ in self.history if k == "progress" and m == media_id]

    def statuses_of(self, media_id: str) -> List[int]:
        return [s for k, m, s, _, _ in self.history if k == "status" and m == media_id]
