"""Minimal span tracing with trace-id propagation through broker headers.

The reference initialises a Jaeger tracer (index.js:10,15) and passes it to main, which
ignores it (lib/main.js:40): no spans are ever created. This module gives
per-job and per-stage spans exported as JSON lines, with W3C-style ``traceparent`` carried
in message headers so a convert job can be correlated with the download that produced it.
"""
from __future__ import annotations

import atexit
import contextvars
import json
import os
import secrets
import sys
import threading
import time
from collections import deque
from contextlib import contextmanager
from typing import Any, Deque, Dict, Iterator, List, Optional, TextIO

_current: contextvars.ContextVar[Optional["Span"]] = contextvars.ContextVar("span", default=None)


class Span:
    __slots__ = ("tracer", "name", "trace_id", "span_id", "parent_id", "start", "end", "attrs",
                 "status")

    def __init__(self, tracer: "Tracer", name: str, trace_id: str, parent_id: Optional[str]):
        self.tracer = tracer
        self.name = name
        self.trace_id = trace_id
        self.span_id = secrets.token_hex(8)
        self.parent_id = parent_id
        self.start = time.time()
        self.end: Optional[float] = None
        self.attrs: Dict[str, Any] = {}
        self.status = "ok"

    def set(self, **attrs: Any) -> None:
        self.attrs.update(attrs)

    def traceparent(self) -> str:
        return f"00-{self.trace_id}-{self.span_id}-01"

    def to_dict(self) -> Dict[str, Any]:
        return {"name": self.name, "trace_id": self.trace_id, "span_id": self.span_id,
                "parent_id": self.parent_id, "start": self.start, "end": self.end,
                "duration_ms": None if self.end is None else (self.end - self.start) * 1e3,
                "status": self.status, "attrs": self.attrs, "service": self.tracer.service}


def parse_traceparent(tp: Optional[str]) -> Optional[tuple]:
    if not tp:
        return None
    parts = tp.split("-")
    if len(parts) != 4 or len(parts[1]) != 32 or len(parts[2]) != 16:
        return None
    return parts[1], parts[2]


class SpanExporter:
    """JSON-lines span sink on its own thread. Finished spans are queued by the event loop
    (no serialisation, no file I/O there - round 2 opened and wrote the trace file on the
    loop thread for every span, ~4 per job at ~1k jobs/s) and written in batches through one
    open file. The queue is bounded: past ``max_queue`` spans are dropped and counted.

    The thread wakes every ``interval`` s (or once ``batch`` spans are queued), not per span:
    a wake-up per span hands the GIL back and forth with the event loop ~4 times per job,
    which cost more loop time than the spans themselves (config 9 with tracing on)."""

    def __init__(self, path: str = "", stream: Optional[TextIO] = None, max_queue: int = 100_000,
                 interval: float = 0.2, batch: int = 4096):
        self.path = path
        self.stream = stream
        self.max_queue = max_queue
        self.interval = interval
        self.batch = batch
        self._flushing = 0
        self.dropped = 0
        self.written = 0
        self._q: Deque[Span] = deque()
        self._cv = threading.Condition()
        self._closed = False
        self._busy = False
        self._thread = threading.Thread(target=self._run, name="span-export", daemon=True)
        self._thread.start()
        atexit.register(self.close)

    def submit(self, span: Span) -> None:
        with self._cv:
            if self._closed or len(self._q) >= self.max_queue:
                self.dropped += 1
                return
            self._q.append(span)
            if len(self._q) == self.batch:
                self._cv.notify_all()

    def _run(self) -> None:
        f = open(self.path, "a", encoding="utf-8") if self.path else None
        try:
            while True:
                with self._cv:
                    while not self._closed and not self._flushing and len(self._q) < self.batch:
                        self._cv.wait(self.interval)
                        if self._q:
                            break
                    if not self._q and self._closed:
                        return
                    if not self._q:
                        continue
                    batch = list(self._q)
                    self._q.clear()
                    self._busy = True
                out = f or self.stream or sys.stderr
                out.write("".join(json.dumps(s.to_dict(), default=str) + "\n" for s in batch))
                out.flush()
                with self._cv:
                    self.written += len(batch)
                    self._busy = False
                    self._cv.notify_all()
        finally:
            if f is not None:
                f.close()

    def flush(self, timeout: float = 5.0) -> bool:
        """Wait until every queued span is written."""
        end = time.monotonic() + timeout
        with self._cv:
            self._flushing += 1
            self._cv.notify_all()
            try:
                while self._q or self._busy:
                    left = end - time.monotonic()
                    if left <= 0 or not self._thread.is_alive():
                        return False
                    self._cv.wait(left)
            finally:
                self._flushing -= 1
        return True

    def close(self, timeout: float = 5.0) -> None:
        with self._cv:
            if self._closed:
                return
            self._closed = True
            self._cv.notify_all()
        self._thread.join(timeout)


class Tracer:
    def __init__(self, service: str = "downloader", enabled: bool = True,
                 stream: Optional[TextIO] = None, path: str = ""):
        self.service = service
        self.enabled = enabled
        self._stream = stream
        self._path = path
        self._exporter: Optional[SpanExporter] = None
        self._lock = threading.Lock()
        self.finished: List[Span] = []
        self.keep = False

    def _emit(self, span: Span) -> None:
        if self.keep:
            self.finished.append(span)
        if not self.enabled:
            return
        if self._exporter is None:
            with self._lock:
                if self._exporter is None:
                    self._exporter = SpanExporter(self._path, self._stream)
        self._exporter.submit(span)

    def flush(self, timeout: float = 5.0) -> bool:
        return self._exporter.flush(timeout) if self._exporter is not None else True

    def close(self) -> None:
        if self._exporter is not None:
            self._exporter.close()

    @contextmanager
    def span(self, name: str, traceparent: Optional[str] = None, **attrs: Any) -> Iterator[Span]:
        parent = _current.get()
        if parent is not None:
            trace_id, parent_id = parent.trace_id, parent.span_id
        else:
            tp = parse_traceparent(traceparent)
            trace_id, parent_id = tp if tp else (secrets.token_hex(16), None)
        s = Span(self, name, trace_id, parent_id)
        s.attrs.update(attrs)
        tok = _current.set(s)
        try:
            yield s
        except BaseException as e:
            s.status = "error"
            s.attrs["error"] = f"{type(e).__name__}: {e}"
            raise
        finally:
            s.end = time.time()
            _current.reset(tok)
            self._emit(s)


def current_span() -> Optional[Span]:
    return _current.get()


def init_tracer(service: str, enabled: Optional[bool] = None, path: str = "") -> Tracer:
    """``initTracer('downloader', logger)`` equivalent (index.js:15)."""
    if enabled is None:
        enabled = os.environ.get("STAGER_TRACE", "") in ("1", "true")
    return Tracer(service, enabled=enabled, path=path)
