"""HTTP/1.1 transports used by the S3 client and the HTTP fetcher.

Two implementations behind one async interface:

* ``NativeTransport`` - ``http://`` and ``https://`` over the C++ ``HttpConn`` (keep-alive
  pool). Plain bodies are spliced socket->file and sent file->socket with ``sendfile``; TLS
  bodies go through OpenSSL on the same threads (``csrc/tls.cpp``). Each request runs on a
  dedicated thread pool with the GIL released, so many transfers (and their encryption)
  proceed in parallel inside one worker process.
  https through a forward proxy tunnels with CONNECT on the same connection.
* ``AiohttpTransport`` - everything when the native module (or its TLS) is off.

A request body is ``bytes`` or a ``FileRange``; a response body is returned in memory or
written into a ``FileSink``.

Redirects: the reference fetches with ``request`` (npm), which follows up to 10 redirects of a
GET/HEAD (``followRedirect``; other methods are not redirected) and drops ``Authorization``
when the host changes. ``TransportSet.request`` and ``NativeTransport.relay`` do the same;
``Response.url`` is the URL that finally answered. A 3xx body is never written into a sink.
"""
from __future__ import annotations

import asyncio
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Set, Tuple, Union
from urllib.parse import quote, urljoin, urlsplit

from .proxy import Proxy, ProxyConfig
from ..utils.log import get_logger, redact_text, redact_url

log = get_logger("http.py")

Headers = Sequence[Tuple[str, str]]

REDIRECTS = (301, 302, 303, 307, 308)
MAX_REDIRECTS = 10          # request@2 maxRedirects


class HttpError(Exception):
    def __init__(self, msg: str, status: int = 0, body: bytes = b""):
        super().__init__(msg)
        self.status = status
        self.body = body


class TransportError(HttpError):
    """Connection-level failure (reset, timeout, refused) - always retryable."""


@dataclass
class FileRange:
    fd: int
    offset: int
    length: int


@dataclass
class FileSink:
    fd: int
    offset: int = 0
    max_bytes: int = 1 << 50


@dataclass
class Response:
    status: int
    headers: List[Tuple[str, str]]
    body: bytes = b""
    written: int = 0
    reason: str = ""
    url: str = ""                # the URL that produced this response (after redirects)
    sent_crc32c: str = ""        # relayed aws-chunked PUT: the trailing CRC32C we sent

    def header(self, name: str, default: Optional[str] = None) -> Optional[str]:
        name = name.lower()
        for k, v in self.headers:
            if k == name:
                return v
        return default

    @property
    def ok(self) -> bool:
        return 200 <= self.status < 300


@dataclass
class Progress:
    """Byte counter updated while a transfer runs (native: updated from C++ threads)."""
    native: object = None
    _bytes: int = 0
    cancelled: bool = False

    @property
    def bytes(self) -> int:
        return self.native.bytes if self.native is not None else self._bytes

    def add(self, n: int) -> None:
        self._bytes += n

    def cancel(self) -> None:
        self.cancelled = True
        if self.native is not None:
            self.native.cancel()


def redirect_target(url: str, r: "Response") -> Optional[str]:
    """Absolute URL a 3xx response points to (None: not a usable redirect)."""
    if r.status not in REDIRECTS:
        return None
    loc = r.header("location")
    if not loc:
        return None
    # Like the WHATWG URL parser: resolve against the current URL and percent-encode what
    # may not appear raw in a request line (spaces, non-ASCII), keeping existing escapes.
    nxt = quote(urljoin(url, loc.strip()), safe=":/?#[]@!$&'()*+,;=%~")
    return nxt if urlsplit(nxt).scheme in ("http", "https") else None


def redirect_headers(url: str, nxt: str, headers: Headers) -> List[Tuple[str, str]]:
    """Headers for the next hop: ``Authorization`` (and a stale ``Host``) is dropped when the
    host changes, as request@2 does; everything else (``Range``!) is kept."""
    same = urlsplit(url).netloc == urlsplit(nxt).netloc
    return [(k, v) for k, v in headers
            if k.lower() != "host" and (same or k.lower() != "authorization")]


def _via_proxy(proxy: Proxy, url: str, headers: Headers
               ) -> Tuple[str, int, str, List[Tuple[str, str]]]:
    """Connect target, absolute-form request target and headers for a plain-http request
    through a forward proxy (RFC 7230 5.3.2)."""
    target = url.split("#", 1)[0]
    hdrs = list(headers)
    if proxy.auth:
        hdrs.append(("Proxy-Authorization", proxy.auth))
    return proxy.host, proxy.port, target, hdrs


def _bracket(host: str) -> str:
    return f"[{host}]" if ":" in host else host      # IPv6 literal


def _host_hdr(host: str, port: int, tls: bool) -> str:
    host = _bracket(host)
    return host if port == (443 if tls else 80) else f"{host}:{port}"


def split_host(url: str) -> Tuple[str, str, int, str]:
    u = urlsplit(url)
    scheme = u.scheme or "http"
    port = u.port or (443 if scheme == "https" else 80)
    path = u.path or "/"
    if u.query:
        path += "?" + u.query
    return scheme, u.hostname or "", port, path


def _build_head(method: str, host_hdr: str, path: str, headers: Headers,
                body_len: Optional[int]) -> bytes:
    lines = [f"{method} {path} HTTP/1.1", f"Host: {host_hdr}"]
    have_len = False
    for k, v in headers:
        lk = k.lower()
        if lk == "host":
            continue
        if lk == "content-length":
            have_len = True
        lines.append(f"{k}: {v}")
    if body_len is not None and not have_len and (body_len > 0 or method in ("PUT", "POST")):
        lines.append(f"Content-Length: {body_len}")
    lines.append("User-Agent: downloader-amd/0.1")
    return ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")


class SourceChanged(TransportError):
    """The origin answered a pinned request (If-Match / If-Unmodified-Since / If-Range) with
    412, or with a whole 200 body where a 206 range was asked: the object is no longer the
    version the transfer started on, so the bytes already moved belong to another version."""


def pin_headers(validator: str, ranged: bool) -> List[Tuple[str, str]]:
    """Request headers that pin a GET to the version ``validator`` (``probe_validated``: a
    strong ETag, or ``lm:<Last-Modified>``): a changed object answers 412 (``If-Match`` /
    ``If-Unmodified-Since``), and - for servers that only honour ``If-Range`` - a ranged GET
    answers 200 with the whole new body instead of the 206 slice."""
    if not validator:
        return []
    if validator.startswith("lm:"):
        date = validator[3:]
        return [("If-Unmodified-Since", date)] + ([("If-Range", date)] if ranged else [])
    return [("If-Match", validator)] + ([("If-Range", validator)] if ranged else [])


# aws-chunked framing of a relayed PUT that carries a trailing CRC32C (S3 flexible checksums):
# "<hex n>\r\n" <n bytes> "\r\n" "0\r\n" "x-amz-checksum-crc32c:<8 b64>\r\n" "\r\n"
CRC_TRAILER = "x-amz-checksum-crc32c"


def aws_chunked_length(n: int) -> int:
    """Encoded Content-Length of an ``n``-byte payload sent as one aws-chunked data chunk
    plus the zero chunk with the CRC32C trailer (csrc/module.cpp ``relay``)."""
    data = len(f"{n:x}") + 2 + n + 2 if n > 0 else 0
    return data + 3 + len(CRC_TRAILER) + 1 + 8 + 2 + 2


class Transport:
    async def request(self, method: str, url: str, headers: Headers = (),
                      body: Union[None, bytes, FileRange] = None, sink: Optional[FileSink] = None,
                      progress: Optional[Progress] = None, expect_body: bool = True,
                      proxy: Optional[Proxy] = None) -> Response:
        raise NotImplementedError

    async def close(self) -> None:
        pass


async def _drain(fut: "asyncio.Future", timeout: float = 10.0) -> None:
    """After cancelling a native call (progress flag set, sockets shut down), wait for its
    worker thread to return before the caller's cancellation completes. The caller may close
    the sink's fd right after (a torrent session closing its storage): a transfer still
    splicing into that descriptor number would write into whatever file reuses it. Bounded:
    the shut-down socket ends a blocked recv / splice at once. The outcome is discarded."""
    try:
        await asyncio.wait_for(asyncio.shield(fut), timeout)
    except BaseException:
        pass
    if fut.done() and not fut.cancelled():
        fut.exception()        # retrieved: no "Future exception was never retrieved" log


class NativeTransport(Transport):
    def __init__(self, max_workers: int = 32, connect_timeout: float = 10.0,
                 io_timeout: float = 300.0, max_idle_per_host: int = 64,
                 idle_ttl: float = 30.0, max_idle_total: int = 512, tls: bool = True,
                 ssl_verify: bool = True, ca_file: str = ""):
        from ..ops import native
        self._n = native()
        # one SSL_CTX for every https connection of this transport (None: http only)
        self._tls = self._n.TlsContext(ssl_verify, ca_file) if tls else None
        # (host, port, tls, via) -> [(conn, released at)], most recently released last (via:
        # the CONNECT proxy of a tunnelled https connection, else None). Idle sockets
        # expire after idle_ttl (servers drop keep-alive connections anyway) and at most
        # max_idle_total stay open over all hosts: a long-running worker that fetched from
        # many origins must not sit on hosts x 64 idle file descriptors.
        self._pool: Dict[tuple, List[Tuple[object, float]]] = {}
        self.idle_ttl = idle_ttl
        self.max_idle_total = max_idle_total
        self._idle_total = 0
        self._lock = threading.Lock()
        self._exec = ThreadPoolExecutor(max_workers=max_workers, thread_name_prefix="xfer")
        # connections of requests in flight (one list per request), so a cancelled request or
        # close() can abort() the socket a blocked native transfer sits on
        self._inflight: Set[int] = set()
        self._slots: Dict[int, List[object]] = {}
        self._aborted: Set[int] = set()     # slots whose request was cancelled
        self.connect_timeout = connect_timeout
        self.io_timeout = io_timeout
        self.max_idle = max_idle_per_host

    def handles(self, url: str, proxied: bool = False) -> bool:
        """http:// always; https:// when TLS is on (behind a proxy: CONNECT tunnel)."""
        if url.startswith("http://"):
            return True
        return url.startswith("https://") and self._tls is not None

    def _acquire(self, host: str, port: int, tls: bool = False,
                 tunnel: Optional[Proxy] = None) -> Tuple[object, bool]:
        key = (host, port, tls, (tunnel.host, tunnel.port, tunnel.auth) if tunnel else None)
        stale = []
        try:
            with self._lock:
                idle = self._pool.get(key)
                now = time.monotonic()
                while idle:
                    conn, t = idle.pop()
                    self._idle_total -= 1
                    if now - t <= self.idle_ttl:
                        return conn, True
                    stale.append(conn)         # older ones below it are staler: drop all
                    stale.extend(c for c, _ in idle)
                    self._idle_total -= len(idle)
                    idle.clear()
        finally:
            for c in stale:
                c.close()
        if tls and self._tls is None:
            raise ValueError("NativeTransport built without TLS")
        conn = None
        try:
            if tunnel is None:
                conn = self._n.HttpConn(host, port, self.connect_timeout, self.io_timeout,
                                        self._tls if tls else None)
            else:                   # https via a forward proxy: CONNECT, then TLS inside
                conn = self._n.HttpConn(tunnel.host, tunnel.port, self.connect_timeout,
                                        self.io_timeout)
                conn.connect_tunnel(f"{_bracket(host)}:{port}", tunnel.auth)
                conn.start_tls(self._tls, host)
        except RuntimeError as e:
            if conn is not None:
                conn.close()
            raise TransportError(str(e)) from e
        conn.pool_key = key
        return conn, False

    def _release(self, conn) -> None:
        if not conn.reusable:
            conn.close()
            return
        drop = []
        with self._lock:
            idle = self._pool.setdefault(conn.pool_key, [])
            if len(idle) < self.max_idle:
                idle.append((conn, time.monotonic()))
                self._idle_total += 1
                conn = None
                if self._idle_total > self.max_idle_total:
                    drop = self._evict_locked()
        if conn is not None:
            conn.close()
        for c in drop:
            c.close()

    def _evict_locked(self) -> List[object]:
        """Over the global idle cap: drop expired sockets everywhere, then the oldest."""
        now = time.monotonic()
        out = []
        for key in list(self._pool):
            lst = self._pool[key]
            keep = [(c, t) for c, t in lst if now - t <= self.idle_ttl]
            out += [c for c, t in lst if now - t > self.idle_ttl]
            if keep:
                self._pool[key] = keep
            else:
                del self._pool[key]
        self._idle_total = sum(len(v) for v in self._pool.values())
        while self._idle_total > self.max_idle_total:
            key = min(self._pool, key=lambda k: self._pool[k][0][1])
            c, _ = self._pool[key].pop(0)
            out.append(c)
            self._idle_total -= 1
            if not self._pool[key]:
                del self._pool[key]
        return out

    def idle_connections(self) -> int:
        with self._lock:
            return self._idle_total

    def _track(self, slot: int, conn) -> None:
        with self._lock:
            self._slots.setdefault(slot, []).append(conn)
            if slot in self._aborted:      # cancelled while this connection was being set up
                conn.abort()

    def _untrack(self, slot: int, conn) -> None:
        """Before the owner releases or closes ``conn``: afterwards an abort must not reach it
        (pooled for another request, or its fd number reused)."""
        with self._lock:
            lst = self._slots.get(slot)
            if lst is not None and conn in lst:
                lst.remove(conn)

    def _abort_slot(self, slot: int) -> None:
        """Cancel one request: shut its sockets down (a blocked recv / send / splice returns
        at once) and make any connection it sets up later dead on arrival. Only this request
        ends - a Progress shared with sibling requests (a job's parts) is not flagged, so a
        fan-out that cancels its other parts can restart with the same counter."""
        with self._lock:   # under the lock: the owner cannot close the fd meanwhile
            self._aborted.add(slot)
            for c in self._slots.get(slot, []):
                c.abort()

    def _slot_aborted(self, slot: int) -> bool:
        with self._lock:
            return slot in self._aborted

    def _do(self, method: str, host: str, port: int, host_hdr: str, path: str,
            headers: Headers, body, sink: Optional[FileSink], nprog,
            expect_body: bool, slot: int = 0, tls: bool = False,
            tunnel: Optional[Proxy] = None) -> Response:
        blen = body.length if isinstance(body, FileRange) else (len(body) if body else 0)
        head = _build_head(method, host_hdr, path, headers, blen if body is not None else
                           (0 if method in ("PUT", "POST") else None))
        for attempt in (0, 1):
            conn, reused = self._acquire(host, port, tls, tunnel)
            self._track(slot, conn)
            try:
                if isinstance(body, FileRange):
                    d = conn.request_fd(head, body.fd, body.offset, body.length, nprog)
                elif sink is not None:
                    d = conn.get_to_fd(head, sink.fd, sink.offset, sink.max_bytes, nprog)
                else:
                    d = conn.request(head, body, expect_body and method != "HEAD")
            except RuntimeError as e:
                self._untrack(slot, conn)
                conn.close()
                # A pooled keep-alive socket may have been closed by the peer: retry once on
                # a fresh connection (the whole request is re-sent; bodies are re-readable).
                if reused and attempt == 0 and not (nprog is not None and nprog.cancelled) \
                        and not self._slot_aborted(slot):
                    continue
                raise TransportError(f"{method} {host}:{port}{path}: {e}") from e
            self._untrack(slot, conn)
            self._release(conn)
            return Response(d["status"], list(d["headers"]), d.get("body", b""),
                            d.get("written", 0), d.get("reason", ""))
        raise TransportError("unreachable")

    async def request(self, method: str, url: str, headers: Headers = (),
                      body: Union[None, bytes, FileRange] = None, sink: Optional[FileSink] = None,
                      progress: Optional[Progress] = None, expect_body: bool = True,
                      proxy: Optional[Proxy] = None) -> Response:
        scheme, host, port, path = split_host(url)
        if not self.handles(url, proxy is not None):
            raise ValueError(f"NativeTransport cannot send {scheme}://"
                             + (" through a proxy" if proxy is not None else ""))
        tls = scheme == "https"
        host_hdr = _host_hdr(host, port, tls)
        tunnel = proxy if tls else None
        if proxy is not None and not tls:   # absolute-form request target to the proxy
            host, port, path, headers = _via_proxy(proxy, url, headers)
        nprog = None
        if progress is not None:
            if progress.native is None:
                progress.native = self._n.Progress()
            nprog = progress.native
        loop = asyncio.get_running_loop()
        slot = self._new_slot()
        fut = loop.run_in_executor(self._exec, self._do, method, host, port, host_hdr, path,
                                   headers, body, sink, nprog, expect_body, slot, tls, tunnel)
        try:
            return await asyncio.shield(fut)
        except asyncio.CancelledError:
            self._abort_slot(slot)
            await _drain(fut)
            raise
        finally:
            self._end_slot(slot)

    def _new_slot(self) -> int:
        with self._lock:
            self._seq = getattr(self, "_seq", 0) + 1
            self._inflight.add(self._seq)
            return self._seq

    def _end_slot(self, slot: int) -> None:
        with self._lock:
            self._inflight.discard(slot)
            self._slots.pop(slot, None)
            self._aborted.discard(slot)

    def _relay(self, src_url: str, src_headers: Headers, dst_url: str, dst_headers: Headers,
               length: int, nprog, slot: int = 0, split: Optional[Tuple[int, int, int]] = None,
               src_proxy: Optional[Proxy] = None, checksum: bool = False, gpu: bool = False
               ) -> Tuple[Response, Optional[Response], int, Optional[dict]]:
        ss, sh, sp, spath = split_host(src_url)
        ds, dh, dp, dpath = split_host(dst_url)
        if not (self.handles(src_url, src_proxy is not None) and self.handles(dst_url)):
            raise TransportError(f"relay {ss}:// -> {ds}://"
                                 + (" through a proxy" if src_proxy is not None else "")
                                 + ": not supported by the native transport")
        stls, dtls = ss == "https", ds == "https"
        src_host_hdr = _host_hdr(sh, sp, stls)
        tunnel = src_proxy if stls else None
        if src_proxy is not None and not stls:
            sh, sp, spath, src_headers = _via_proxy(src_proxy, src_url, src_headers)
        get_head = _build_head("GET", src_host_hdr, spath, src_headers, None)
        put_head = _build_head("PUT", _host_hdr(dh, dp, dtls), dpath, dst_headers,
                               aws_chunked_length(length) if checksum else length)
        src, _ = self._acquire(sh, sp, stls, tunnel)
        self._track(slot, src)
        try:
            dst, _ = self._acquire(dh, dp, dtls)
        except BaseException:
            self._untrack(slot, src)
            self._release(src)
            raise
        self._track(slot, dst)
        try:
            if split is None:
                d = src.relay_to(get_head, dst, put_head, length, nprog, crc=checksum)
            else:
                d = src.relay_hashed_to(get_head, dst, put_head, length, *split, nprog,
                                        crc=checksum, gpu=gpu)
        except RuntimeError as e:
            self._untrack(slot, src)
            self._untrack(slot, dst)
            src.close()
            dst.close()
            raise TransportError(f"relay {spath} -> {dpath}: {e}") from e
        self._untrack(slot, src)
        self._untrack(slot, dst)
        self._release(src)
        self._release(dst)
        g = d["get"]
        get = Response(g["status"], list(g["headers"]), d["get_body"], 0, g.get("reason", ""))
        put = None
        if d["put"] is not None:
            p = d["put"]
            put = Response(p["status"], list(p["headers"]), d["put_body"], 0, p.get("reason", ""))
            put.sent_crc32c = d.get("crc32c", "")
        hashed = {k: d[k] for k in ("digests", "head", "tail", "gpu_ticket")} \
            if split is not None else None
        return get, put, d["moved"], hashed

    async def relay(self, src_url: str, src_headers: Headers, dst_url: str, dst_headers: Headers,
                    length: int, progress: Optional[Progress] = None,
                    split: Optional[Tuple[int, int, int]] = None,
                    src_proxy: Optional[ProxyConfig] = None, checksum: bool = False,
                    gpu: bool = False
                    ) -> Tuple[Response, Optional[Response], int, Optional[dict]]:
        """GET ``src_url`` and stream exactly ``length`` body bytes as the body of a PUT to
        ``dst_url`` without touching user space (socket -> pipe -> socket splice; through an
        L2-sized buffer when either end is TLS). The PUT is only sent when the GET answers 2xx
        with exactly that Content-Length.

        ``split=(skip, full_len, piece_len)``: relay through L2-sized user-space chunks and
        SHA-1 body bytes [skip, skip+full_len) as consecutive pieces on the way; the 4th
        result is then ``{"digests", "head", "tail"}`` (``HttpConn.relay_hashed_to``).

        ``checksum``: the PUT body is aws-chunked with a trailing ``x-amz-checksum-crc32c``
        computed on the way (bytes through user space); ``dst_headers`` must carry the
        aws-chunked headers (``S3Client._relay_put`` does). ``gpu`` (with ``split``): the
        part's pieces may go to the installed part hasher (``hashed["gpu_ticket"]``)."""
        nprog = None
        if progress is not None:
            if progress.native is None:
                progress.native = self._n.Progress()
            nprog = progress.native
        loop = asyncio.get_running_loop()
        for _ in range(MAX_REDIRECTS + 1):
            slot = self._new_slot()
            px = src_proxy.for_url(src_url) if src_proxy is not None else None
            fut = loop.run_in_executor(self._exec, self._relay, src_url, src_headers, dst_url,
                                       dst_headers, length, nprog, slot, split, px, checksum,
                                       gpu)
            try:
                out = await asyncio.shield(fut)
            except asyncio.CancelledError as ce:
                self._abort_slot(slot)
                await _drain(fut)
                held = await self._forget_ticket(fut)
                if held is not None:
                    # the device did not give the part's buffer back in time: the caller keeps
                    # its budget bytes until it does (getattr(e, "held_until", None))
                    ce.held_until = held
                raise
            finally:
                self._end_slot(slot)
            get, put = out[0], out[1]
            get.url = src_url
            nxt = redirect_target(src_url, get) if put is None else None
            if nxt is None:
                return out
            if not self.handles(nxt, src_proxy is not None and
                                src_proxy.for_url(nxt) is not None):
                raise TransportError(f"relay source {redact_url(src_url)} redirects to "
                                     f"{redact_url(nxt)}: not "
                                     f"supported by the socket relay", get.status)
            src_headers = redirect_headers(src_url, nxt, src_headers)
            src_url = nxt
        raise TransportError(f"relay source: more than {MAX_REDIRECTS} redirects", 310)

    FORGET_WAIT_S = 5.0

    async def _forget_ticket(self, fut: "asyncio.Future") -> Optional["asyncio.Future"]:
        """A cancelled relay that had queued its part to the GPU hasher: nobody will ask for
        the digests; the native side returns the part's buffer to the pool when its DMA is
        over and drops the result. ``gpu_part_forget`` blocks until the DMA is (milliseconds),
        so it runs on a thread of its own - and this waits for it: the caller gives the part's
        bytes back to its PartBudget when the cancellation reaches it, which must not happen
        while the buffer is still leased (the budget's bound was briefly exceeded).
        The wait is bounded (FORGET_WAIT_S, ADVICE r5: a device that stopped answering must not
        hang the cancellation, nor worker shutdown behind it): past it the future that ends
        when the forget does is returned, and the caller holds the part's budget until then."""
        if not fut.done() or fut.cancelled() or fut.exception() is not None:
            return None
        hashed = fut.result()[3]
        gid = hashed.get("gpu_ticket") if hashed else 0
        if not gid:
            return None
        loop = asyncio.get_running_loop()
        over = loop.create_future()

        def settle() -> None:
            if not over.done():
                over.set_result(None)

        def forget() -> None:
            try:
                self._n.gpu_part_forget(gid)
            finally:
                try:
                    loop.call_soon_threadsafe(settle)
                except RuntimeError:          # the loop is gone: nobody waits any more
                    pass
        threading.Thread(target=forget, name="gpu-part-forget", daemon=True).start()
        try:
            await asyncio.wait_for(asyncio.shield(over), self.FORGET_WAIT_S)
        except asyncio.TimeoutError:
            log.warn("gpu part forget still blocked: its budget stays held until it returns",
                        ticket=gid, waited_s=self.FORGET_WAIT_S)
            return over
        except asyncio.CancelledError:
            pass
        return None

    async def close(self) -> None:
        with self._lock:
            conns = [c for v in self._pool.values() for c, _ in v]
            self._pool.clear()
            self._idle_total = 0
            for v in self._slots.values():
                for c in v:
                    c.abort()   # transfers still running on executor threads fail fast
            self._slots.clear()
        for c in conns:
            c.close()
        self._exec.shutdown(wait=False)


class AiohttpTransport(Transport):
    """Requests when the native transport (or its TLS) is off. TLS peers are verified against
    the system trust store,
    plus ``ca_file`` (PEM bundle, e.g. the private CA of an in-cluster MinIO) when given;
    ``ssl_verify=False`` turns verification off (minio-js ``transport`` with
    ``rejectUnauthorized: false``)."""

    def __init__(self, connect_timeout: float = 10.0, io_timeout: float = 300.0,
                 limit: int = 64, ssl_verify: bool = True, ca_file: str = ""):
        self._session = None
        self.connect_timeout = connect_timeout
        self.io_timeout = io_timeout
        self.limit = limit
        self.ssl_verify = ssl_verify
        self.ca_file = ca_file
        self.max_body = 64 << 20

    def ssl_context(self):
        """Value for aiohttp's ``ssl=``: None = default verified context, False = no checks."""
        if not self.ssl_verify:
            return False
        if not self.ca_file:
            return None
        import ssl
        ctx = ssl.create_default_context()
        ctx.load_verify_locations(cafile=self.ca_file)     # in addition to the system store
        return ctx

    async def _sess(self):
        import aiohttp
        if self._session is None or self._session.closed:
            timeout = aiohttp.ClientTimeout(total=None, connect=self.connect_timeout,
                                            sock_read=self.io_timeout)
            conn = aiohttp.TCPConnector(limit=self.limit, ssl=self.ssl_context())
            self._session = aiohttp.ClientSession(timeout=timeout, connector=conn,
                                                  auto_decompress=False)
        return self._session

    async def request(self, method: str, url: str, headers: Headers = (),
                      body: Union[None, bytes, FileRange] = None, sink: Optional[FileSink] = None,
                      progress: Optional[Progress] = None, expect_body: bool = True,
                      proxy: Optional[Proxy] = None) -> Response:
        import aiohttp
        sess = await self._sess()
        hdrs = [(k, v) for k, v in headers if k.lower() != "host"]
        data = body
        if isinstance(body, FileRange):
            data = _file_iter(body, progress)
            hdrs.append(("Content-Length", str(body.length)))
        loop = asyncio.get_running_loop()
        try:
            async with sess.request(method, url, headers=hdrs, data=data,
                                    allow_redirects=False, compress=None,
                                    proxy=proxy.url if proxy is not None else None) as resp:
                rh = [(k.lower(), v) for k, v in resp.headers.items()]
                final = str(resp.url)
                if sink is not None and 200 <= resp.status < 300 and \
                        (resp.content_length or 0) > sink.max_bytes:
                    # more than asked (a 200 for a Range GET): not written, like the native path
                    return Response(resp.status, rh, b"", 0, resp.reason or "", final)
                if sink is not None and 200 <= resp.status < 300:
                    written = 0
                    async for chunk in resp.content.iter_chunked(1 << 20):
                        if progress is not None and progress.cancelled:
                            raise TransportError("cancelled")
                        if written + len(chunk) > sink.max_bytes:
                            raise HttpError("response body exceeds limit", resp.status)
                        # a cancel must not return while the thread still writes: the
                        # caller closes sink.fd next, and that number can be reused
                        wf = loop.run_in_executor(None, _pwrite_all, sink.fd, chunk,
                                                  sink.offset + written)
                        try:
                            await asyncio.shield(wf)
                        except asyncio.CancelledError:
                            await _drain(wf)
                            raise
                        written += len(chunk)
                        if progress is not None:
                            progress.add(len(chunk))
                    return Response(resp.status, rh, b"", written, resp.reason or "", final)
                payload = b""
                if method != "HEAD" and expect_body:
                    buf = bytearray()       # bounded like the native transport (64 MiB)
                    async for chunk in resp.content.iter_chunked(1 << 20):
                        if len(buf) + len(chunk) > self.max_body:
                            raise HttpError("response body exceeds limit", resp.status)
                        buf += chunk
                    payload = bytes(buf)
                return Response(resp.status, rh, payload, 0, resp.reason or "", final)
        except (aiohttp.ClientConnectionError, aiohttp.ClientPayloadError,
                asyncio.TimeoutError) as e:
            raise TransportError(f"{method} {redact_url(url)}: {type(e).__name__}: "
                                 f"{redact_text(str(e))}") from e

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()


def _pwrite_all(fd: int, data: bytes, off: int) -> None:
    mv = memoryview(data)
    while mv:
        n = os.pwrite(fd, mv, off)
        mv = mv[n:]
        off += n


async def _file_iter(fr: FileRange, progress: Optional[Progress]):
    loop = asyncio.get_running_loop()
    off, left = fr.offset, fr.length
    while left > 0:
        n = min(left, 1 << 20)
        chunk = await loop.run_in_executor(None, os.pread, fr.fd, n, off)
        if not chunk:
            raise HttpError("file shorter than declared body length")
        off += len(chunk)
        left -= len(chunk)
        if progress is not None:
            progress.add(len(chunk))
        yield chunk


@dataclass
class TransportSet:
    """Picks the native transport for plain http and aiohttp for https."""
    native: Optional[NativeTransport] = None
    fallback: AiohttpTransport = field(default_factory=AiohttpTransport)

    def for_url(self, url: str, proxied: bool = False) -> Transport:
        if self.native is not None and self.native.handles(url, proxied):
            return self.native
        return self.fallback

    async def request(self, method: str, url: str, follow_redirects: bool = True,
                      proxy: Optional[ProxyConfig] = None, **kw) -> Response:
        """``proxy``: the source-fetch proxy policy (``net/proxy.py``), resolved per hop;
        S3 and torrent traffic pass none."""
        if method not in ("GET", "HEAD") or not follow_redirects:
            r = await self._one(method, url, proxy, kw)
            r.url = r.url or url
            return r
        for _ in range(MAX_REDIRECTS + 1):
            r = await self._one(method, url, proxy, kw)
            r.url = r.url or url
            nxt = redirect_target(r.url, r)
            if nxt is None:
                return r
            kw["headers"] = redirect_headers(r.url, nxt, kw.get("headers") or ())
            url = nxt
        raise TransportError(f"{method} {redact_url(url)}: more than {MAX_REDIRECTS} redirects",
                             310)

    async def _one(self, method: str, url: str, proxy: Optional[ProxyConfig], kw) -> Response:
        px = proxy.for_url(url) if proxy is not None else None
        if px is not None:
            return await self.for_url(url, True).request(method, url, proxy=px, **kw)
        return await self.for_url(url).request(method, url, **kw)

    async def close(self) -> None:
        if self.native is not None:
            await self.native.close()
        await self.fallback.close()


def make_transports(native: bool = True, max_workers: int = 32, connect_timeout: float = 10.0,
                    io_timeout: float = 300.0, ssl_verify: bool = True,
                    ca_file: str = "", native_tls: bool = True) -> TransportSet:
    nt = NativeTransport(max_workers, connect_timeout, io_timeout, tls=native_tls,
                         ssl_verify=ssl_verify, ca_file=ca_file) if native else None
    return TransportSet(nt, AiohttpTransport(connect_timeout, io_timeout, ssl_verify=ssl_verify,
                                             ca_file=ca_file))


Callback = Callable[[int], None]
