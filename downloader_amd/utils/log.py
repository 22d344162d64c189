"""pino-compatible JSON structured logging.

The reference logs with pino (index.js:12-14, lib/main.js:22-24): one JSON object per line
with numeric ``level``, ``time`` (ms since epoch), ``pid``, ``hostname``, ``name`` and ``msg``,
and per-job child loggers carrying ``{jobId, fileId}`` (lib/main.js:75-79, :103-105).
This module reproduces that line format so existing log tooling keeps working.
"""
from __future__ import annotations

import json
import os
import re
import socket
import sys
import threading
import time
from typing import Any, Callable, Dict, List, Optional, TextIO
from urllib.parse import urlsplit, urlunsplit

LEVELS = {"trace": 10, "debug": 20, "info": 30, "warn": 40, "error": 50, "fatal": 60}
_HOST = socket.gethostname()


class Sink:
    """Thread-safe line writer; tests can swap in a ``ListSink``."""

    def __init__(self, stream: Optional[TextIO] = None):
        self.stream = stream or sys.stderr
        self._lock = threading.Lock()

    def write(self, rec: Dict[str, Any]) -> None:
        line = json.dumps(rec, default=str, separators=(",", ":"))
        with self._lock:
            self.stream.write(line + "\n")


class ListSink(Sink):
    def __init__(self):
        super().__init__(stream=None)
        self.records: List[Dict[str, Any]] = []

    def write(self, rec: Dict[str, Any]) -> None:
        with self._lock:
            self.records.append(rec)


_default_sink: Sink = Sink()


def set_default_sink(sink: Sink) -> None:
    global _default_sink
    _default_sink = sink


def _level_from_env() -> int:
    return LEVELS.get(os.environ.get("LOG_LEVEL", "info").lower(), 30)


class Logger:
    def __init__(self, name: str = "downloader", bindings: Optional[Dict[str, Any]] = None,
                 level: Optional[int] = None, sink: Optional[Sink] = None):
        self.bindings: Dict[str, Any] = {"name": name}
        if bindings:
            self.bindings.update(bindings)
        self.level = _level_from_env() if level is None else level
        self._sink = sink

    @property
    def sink(self) -> Sink:
        return self._sink or _default_sink

    def child(self, **bindings: Any) -> "Logger":
        b = dict(self.bindings)
        b.update(bindings)
        lg = Logger(b.pop("name"), b, self.level, self._sink)
        return lg

    def enabled(self, level: str) -> bool:
        return LEVELS[level] >= self.level

    def _log(self, level: str, msg: Any, *args: Any, **fields: Any) -> None:
        lv = LEVELS[level]
        if lv < self.level:
            return
        rec: Dict[str, Any] = {"level": lv, "time": int(time.time() * 1000), "pid": os.getpid(),
                               "hostname": _HOST}
        rec.update(self.bindings)
        if isinstance(msg, dict):
            rec.update(msg)
            msg = " ".join(str(a) for a in args) if args else None
        elif args:
            msg = " ".join([str(msg)] + [str(a) for a in args])
        if isinstance(msg, BaseException):
            rec["err"] = {"type": type(msg).__name__, "message": redact_text(str(msg))}
            msg = str(msg)
        if msg is not None:
            rec["msg"] = redact_text(msg) if isinstance(msg, str) else msg
        for k, v in fields.items():
            rec[k] = redact_text(v) if isinstance(v, str) else v
        self.sink.write(rec)

    def trace(self, msg: Any, *a: Any, **kw: Any) -> None:
        self._log("trace", msg, *a, **kw)

    def debug(self, msg: Any, *a: Any, **kw: Any) -> None:
        self._log("debug", msg, *a, **kw)

    def info(self, msg: Any, *a: Any, **kw: Any) -> None:
        self._log("info", msg, *a, **kw)

    def warn(self, msg: Any, *a: Any, **kw: Any) -> None:
        self._log("warn", msg, *a, **kw)

    warning = warn

    def error(self, msg: Any, *a: Any, **kw: Any) -> None:
        self._log("error", msg, *a, **kw)

    def fatal(self, msg: Any, *a: Any, **kw: Any) -> None:
        self._log("fatal", msg, *a, **kw)


def get_logger(name: str, **bindings: Any) -> Logger:
    return Logger(name, bindings)


NullFn = Callable[..., None]


class NullLogger(Logger):
    """Mirrors the reference tests' ``mockLogger`` (test/process/filter_dirs.js:10-14)."""

    def __init__(self):
        super().__init__("null", level=100)

    def child(self, **bindings: Any) -> "Logger":
        return self


def make_test_logger(name: str = "test") -> Logger:
    """Logger for tests: silent unless ``USE_REAL_LOGGER`` is set (the reference's test switch,
    test/process/filter_dirs.js:19)."""
    return get_logger(name) if os.environ.get("USE_REAL_LOGGER") else NullLogger()


_SECRET_PARAM = re.compile(r"(sig|signature|token|secret|password|passwd|credential|auth|key)",
                           re.IGNORECASE)


def redact_url(url: str) -> str:
    """``url`` for logs: a userinfo password and the values of query parameters that look
    like secrets (``X-Amz-Signature``, ``X-Amz-Credential``, ``token``, ``sig``, ...) become
    ``***``; magnets and anything unparsable pass through unchanged."""
    try:
        u = urlsplit(url)
    except ValueError:
        return url
    if u.scheme not in ("http", "https"):
        return url
    netloc = u.netloc
    if u.password is not None:
        host = u.hostname or ""
        netloc = f"{u.username}:***@{host}" + (f":{u.port}" if u.port else "")
    query = u.query
    if query:
        parts = []
        for kv in query.split("&"):
            k, eq, v = kv.partition("=")
            parts.append(f"{k}=***" if eq and _SECRET_PARAM.search(k) else kv)
        query = "&".join(parts)
    return urlunsplit((u.scheme, netloc, u.path, query, u.fragment))


_URL_IN_TEXT = re.compile(r"https?://[^\s\"'<>]+")


def redact_text(text: str) -> str:
    """``text`` with every http(s) URL in it passed through ``redact_url``: error messages
    quote request URLs (a presigned bucket:// relay source, an origin with a token in its
    query) and must not carry the signature or credential into logs or message headers."""
    if "://" not in text:
        return text
    return _URL_IN_TEXT.sub(lambda m: redact_url(m.group(0)), text)
