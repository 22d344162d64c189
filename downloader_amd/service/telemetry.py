"""Job status / progress telemetry (the reference's ``triton-core/telemetry``).

Reference calls: ``telem.emitStatus(jobId, 2)`` on receipt (lib/main.js:68), ``emitStatus(jobId,
6)`` on failure (:149) and ``emitProgress(id, DOWNLOADING, pct)`` with the curve 0 -> torrent
floor(pct/2) every 30 s -> 50 -> floor(50 + 50*i/n) per uploaded file (lib/download.js:255,
78-88,272; lib/upload.js:48-51). The wire format inside triton-core is INFERRED to be protobuf
over the broker; here ``api.TelemetryStatus`` / ``api.TelemetryProgress`` are published on
two queues. ``history`` keeps the most recent emitted events (bounded: a long-running worker
must not grow with every job) for tests, the bench and debugging.

Telemetry never sits on the data path. In the reference the torrent ticker is decoupled from
the transfer (lib/download.js:78-88) and a progress emit is fire-and-forget
(lib/upload.js:51). Here ``emit_*`` appends to a bounded outbox and returns at once. One
flusher task publishes the outbox in order, each publish bounded by
``telemetry.publish_timeout_s``. While the broker is away the events wait in the outbox; once
it is back they are flushed in order. When the outbox is full the oldest progress event is
dropped (a later one supersedes it; status events go last).
``downloader_telemetry_events_total{outcome=published|dropped|failed}`` counts each event's
fate, and ``downloader_telemetry_buffered`` shows the outbox depth.
"""
from __future__ import annotations

import asyncio
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
                 history_max: int = 100_000, publish_timeout_s: float = 1.0,
                 buffer_max: int = 10_000, retry_max_s: float = 5.0, metrics=None):
        self.broker = broker
        self.status_queue = status_queue
        self.progress_queue = progress_queue
        self.enabled = enabled and broker is not None
        self.log = logger or NullLogger()
        self.keep_history = keep_history
        self.history: Deque[Tuple[str, str, int, Optional[int], float]] = \
            deque(maxlen=history_max)
        self.publish_timeout_s = max(0.01, float(publish_timeout_s))
        self.retry_max_s = max(0.05, float(retry_max_s))
        self.buffer_max = max(1, int(buffer_max))
        self.metrics = metrics
        self._outbox: Deque[Tuple[str, bytes]] = deque()
        self._wake: Optional[asyncio.Event] = None
        self._flusher: Optional[asyncio.Task] = None
        self._idle: Optional[asyncio.Event] = None
        self.counts = {"published": 0, "dropped": 0, "failed": 0}

    @classmethod
    def from_config(cls, cfg, broker: Optional[Broker], logger: Optional[Logger] = None,
                    metrics=None):
        t = cfg.telemetry
        return cls(broker, t.status_queue, t.progress_queue, t.enabled, logger,
                   publish_timeout_s=t.publish_timeout_s, buffer_max=t.buffer_max,
                   retry_max_s=t.retry_max_s, metrics=metrics)

    async def connect(self) -> None:
        if self.enabled:
            await self.broker.declare(self.status_queue)
            await self.broker.declare(self.progress_queue)

    # ------------------------------------------------------------------ emit (never blocks)
    async def emit_status(self, media_id: str, status: int) -> None:
        if self.keep_history:
            self.history.append(("status", media_id, int(status), None, time.time()))
        if self.enabled:
            msg = api.TelemetryStatus(mediaId=media_id, status=int(status))
            self._enqueue(self.status_queue, api.encode(msg))

    async def emit_progress(self, media_id: str, status: int, progress: int) -> None:
        if self.keep_history:
            self.history.append(("progress", media_id, int(status), int(progress), time.time()))
        if self.enabled:
            msg = api.TelemetryProgress(mediaId=media_id, status=int(status),
                                        progress=int(progress))
            self._enqueue(self.progress_queue, api.encode(msg))

    # reference-style aliases
    emitStatus = emit_status
    emitProgress = emit_progress

    def _count(self, outcome: str, n: int = 1) -> None:
        self.counts[outcome] += n
        if self.metrics is not None:
            self.metrics.telemetry_events.labels(outcome).inc(n)

    def _gauge(self) -> None:
        if self.metrics is not None:
            self.metrics.telemetry_buffered.set(len(self._outbox))

    def _enqueue(self, queue: str, body: bytes) -> None:
        if len(self._outbox) >= self.buffer_max:
            # drop the oldest progress event (a later one supersedes it); statuses (2, 6) go
            # only when nothing but statuses is left. The head is never dropped: the flusher
            # may be publishing it right now.
            drop = next((i for i, (q, _) in enumerate(self._outbox)
                         if i and q == self.progress_queue), None)
            if drop is None:
                drop = 1 if len(self._outbox) > 1 else 0
            del self._outbox[drop]
            self._count("dropped")
        self._outbox.append((queue, body))
        self._gauge()
        if self._flusher is None or self._flusher.done():
            loop = asyncio.get_running_loop()
            self._wake = asyncio.Event()
            self._idle = asyncio.Event()
            self._flusher = loop.create_task(self._flush_loop())
        self._idle.clear()
        self._wake.set()

    async def _flush_loop(self) -> None:
        delay = 0.05
        while True:
            if not self._outbox:
                self._idle.set()
                self._wake.clear()
                await self._wake.wait()
                continue
            queue, body = self._outbox[0]
            try:
                await asyncio.wait_for(self.broker.publish(queue, body, confirm=False),
                                       self.publish_timeout_s)
            except asyncio.CancelledError:
                raise
            except Exception as e:
                # broker away or slow: keep the event, retry after a backoff (new events
                # meanwhile only grow the bounded outbox)
                self._count("failed")
                if delay == 0.05:
                    self.log.warn("telemetry publish failed, buffering", err=str(e) or
                                  type(e).__name__, buffered=len(self._outbox))
                await asyncio.sleep(delay)
                delay = min(self.retry_max_s, delay * 2)
                continue
            delay = 0.05
            if self._outbox and self._outbox[0][1] is body:
                self._outbox.popleft()
            self._count("published")
            self._gauge()

    @property
    def buffered(self) -> int:
        return len(self._outbox)

    async def flush(self, timeout: float) -> bool:
        """Wait (at most ``timeout`` s) until every buffered event is published."""
        if not self._outbox or self._idle is None:
            return not self._outbox
        try:
            await asyncio.wait_for(self._idle.wait(), timeout)
        except asyncio.TimeoutError:
            return False
        return True

    async def close(self, timeout: float = 2.0) -> None:
        """Flush what the broker takes within ``timeout``, then stop the flusher; events still
        buffered are counted as dropped."""
        await self.flush(timeout)
        if self._flusher is not None:
            self._flusher.cancel()
            # wait() neither raises the flusher's CancelledError nor swallows our own
            await asyncio.wait({self._flusher})
            self._flusher = None
        if self._outbox:
            self._count("dropped", len(self._outbox))
            self._outbox.clear()
            self._gauge()

    def progress_of(self, media_id: str) -> List[int]:
        return [p for k, m, _, p, _ in self.history if k == "progress" and m == media_id]

    def statuses_of(self, media_id: str) -> List[int]:
        return [s for k, m, s, _, _ in self.history if k == "status" and m == media_id]
