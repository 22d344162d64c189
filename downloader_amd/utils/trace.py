"""Minimal span tracing with trace-id propagation through broker headers.

The reference initialises a Jaeger tracer (index.js:10,15) and passes it to main, which
ignores it (lib/main.js:40): no spans are ever created. This module gives
per-job and per-stage spans exported as JSON lines, with W3C-style ``traceparent`` carried
in message headers so a convert job can be correlated with the download that produced it.
"""
from __future__ import annotations

import contextvars
import json
import os
import secrets
import sys
import threading
import time
from contextlib import contextmanager
from typing import Any, Dict, Iterator, List, Optional, TextIO

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


class Tracer:
    def __init__(self, service: str = "downloader", enabled: bool = True,
                 stream: Optional[TextIO] = None, path: str = ""):
        self.service = service
        self.enabled = enabled
        self._lock = threading.Lock()
        self._stream = stream
        self._path = path
        self.finished: List[Span] = []
        self.keep = False

    def _emit(self, span: Span) -> None:
        if self.keep:
            self.finished.append(span)
        if not self.enabled:
            return
        line = json.dumps(span.to_dict(), default=str)
        with self._lock:
            if self._path:
                with open(self._path, "a", encoding="utf-8") as f:
                    f.write(line + "\n")
            else:
                (self._stream or sys.stderr).write(line + "\n")

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
