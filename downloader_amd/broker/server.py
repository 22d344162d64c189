"""Bundled AMQP 0-9-1 broker (RabbitMQ stand-in; no broker binary ships in the image).

Speaks the subset the staging service and its tests use - connection/channel lifecycle,
``queue.declare/purge/delete`` on the default exchange, ``basic.qos`` (per-consumer prefetch),
``basic.consume/cancel/publish/get/ack/nack/reject``, publisher confirms and heartbeats -
with RabbitMQ's delivery semantics: round-robin dispatch bounded by prefetch, unacked
messages requeued at the head with ``redelivered`` set when their channel or connection goes
away. Queues are in memory.

RabbitMQ behaviours the worker has to survive are reproduced too:
  * ``consumer_timeout`` - a channel holding a delivery unacked for longer is closed with
    406 PRECONDITION_FAILED (its deliveries requeued), as RabbitMQ >= 3.8.15 does;
  * ``queue.delete`` sends ``basic.cancel`` to the queue's consumers (consumer_cancel_notify);
  * ``x-message-ttl`` + ``x-dead-letter-exchange`` / ``x-dead-letter-routing-key`` queue
    arguments (expired messages are dead-lettered with an ``x-death`` header) - the
    delayed-retry holding queues;
  * TLS listeners (``amqps://``) when given an ``ssl.SSLContext``.

Run standalone: ``python -m downloader_amd broker --port 5672``.
"""
from __future__ import annotations

import asyncio
import dataclasses
import itertools
import ssl
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional, Tuple

from . import amqp_codec as C


@dataclass
class _Msg:
    body: bytes
    props: C.Properties
    redelivered: bool = False
    expires: float = 0.0        # monotonic deadline in a TTL queue (0: none)


@dataclass
class _Consumer:
    tag: str
    queue: str
    chan: "_Chan"
    prefetch: int
    unacked: int = 0


@dataclass
class _Queue:
    name: str
    msgs: Deque[_Msg] = field(default_factory=deque)
    consumers: List[_Consumer] = field(default_factory=list)
    rr: int = 0
    published: int = 0
    delivered: int = 0
    args: Dict = field(default_factory=dict)
    expired: int = 0
    timer: Optional[asyncio.TimerHandle] = None


class _Chan:
    def __init__(self, conn: "_Conn", cid: int):
        self.conn = conn
        self.id = cid
        self.prefetch = 0
        self.consumers: Dict[str, _Consumer] = {}
        # delivery tag -> (queue, message, consumer, monotonic time of delivery)
        self.unacked: Dict[int, Tuple[str, _Msg, Optional[_Consumer], float]] = {}
        self.dtags = itertools.count(1)
        self.confirming = False
        self.pub_seq = 0
        self.pending: Optional[Tuple[str, str]] = None   # (exchange, routing key)
        self.pending_props: Optional[C.Properties] = None
        self.pending_size = 0
        self.pending_body: List[bytes] = []


class _Conn:
    def __init__(self, server: "BrokerServer", reader: asyncio.StreamReader,
                 writer: asyncio.StreamWriter):
        self.s = server
        self.reader = reader
        self.writer = writer
        self.chans: Dict[int, _Chan] = {}
        self.frame_max = 131072
        self.heartbeat = 0
        self.closed = False

    def send(self, data: bytes) -> None:
        if not self.closed and not self.writer.is_closing():
            self.writer.write(data)


class BrokerServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, users: Optional[Dict[str, str]] = None,
                 heartbeat: int = 60, frame_max: int = 131072,
                 consumer_timeout: float = 0.0, ssl_context: Optional[ssl.SSLContext] = None):
        self.host = host
        self.port = port
        # seconds a delivery may stay unacked before its channel is closed (0: never;
        # RabbitMQ's default is 30 min)
        self.consumer_timeout = consumer_timeout
        self.ssl_context = ssl_context
        self.timeouts = 0           # channels closed by consumer_timeout
        self._reaper: Optional[asyncio.Task] = None
        self.users = users if users is not None else {"guest": "guest"}
        self.heartbeat = heartbeat
        self.frame_max = frame_max
        self.queues: Dict[str, _Queue] = {}
        self.conns: List[_Conn] = []
        self._server: Optional[asyncio.AbstractServer] = None
        self._ctags = itertools.count(1)

    @property
    def url(self) -> str:
        scheme = "amqps" if self.ssl_context is not None else "amqp"
        return f"{scheme}://guest:guest@{self.host}:{self.port}/"

    async def start(self) -> "BrokerServer":
        self._server = await asyncio.start_server(self._handle, self.host, self.port,
                                                  reuse_address=True, ssl=self.ssl_context)
        self.port = self._server.sockets[0].getsockname()[1]
        if self.consumer_timeout > 0:
            self._reaper = asyncio.get_running_loop().create_task(self._timeout_loop())
        return self

    async def stop(self) -> None:
        if self._reaper is not None:
            self._reaper.cancel()
        for q in self.queues.values():
            if q.timer is not None:
                q.timer.cancel()
        if self._server is not None:
            self._server.close()
        for c in list(self.conns):
            c.closed = True
            c.writer.close()
        if self._server is not None:
            await self._server.wait_closed()

    async def serve_forever(self) -> None:
        await self.start()
        assert self._server is not None
        await self._server.serve_forever()

    def drop_connections(self) -> None:
        """Fault injection: kill every client connection (broker restart without data loss)."""
        for c in list(self.conns):
            c.writer.transport.abort()

    def depth(self, queue: str) -> int:
        q = self.queues.get(queue)
        return len(q.msgs) if q else 0

    def consumers(self, queue: str) -> int:
        q = self.queues.get(queue)
        return len(q.consumers) if q else 0

    def delete_queue(self, queue: str) -> int:
        """Admin-side delete (rabbitmqctl delete_queue): consumers get ``basic.cancel``."""
        q = self.queues.pop(queue, None)
        if q is None:
            return 0
        if q.timer is not None:
            q.timer.cancel()
        for c in q.consumers:
            c.chan.consumers.pop(c.tag, None)
            c.chan.conn.send(C.method_frame(c.chan.id, C.BASIC_CANCEL, c.tag, False))
        return len(q.msgs)

    def close_consumer_channels(self, queue: str, code: int = 320,
                                text: str = "CONNECTION_FORCED - channel closed by operator") -> int:
        """Fault injection: the broker closes every channel consuming ``queue``."""
        q = self.queues.get(queue)
        chans = {id(c.chan): c.chan for c in (q.consumers if q else [])}
        for ch in chans.values():
            self._chan_error(ch, code, text, (0, 0))
        return len(chans)

    async def _timeout_loop(self) -> None:
        """RabbitMQ's consumer_timeout: a channel with a delivery unacked for longer than
        the limit is closed with 406 and its deliveries are requeued."""
        period = max(0.02, min(1.0, self.consumer_timeout / 4))
        while True:
            await asyncio.sleep(period)
            now = time.monotonic()
            for conn in list(self.conns):
                for ch in list(conn.chans.values()):
                    if any(now - ent[3] > self.consumer_timeout
                           for ent in ch.unacked.values() if ent[2] is not None):
                        self.timeouts += 1
                        ms = int(self.consumer_timeout * 1000)
                        self._chan_error(ch, 406, "PRECONDITION_FAILED - delivery acknowledgement "
                                         f"on channel {ch.id} timed out. Timeout value used: "
                                         f"{ms} ms", (0, 0))

    # ---------------------------------------------------------------- connection handling
    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        conn = _Conn(self, reader, writer)
        try:
            hdr = await asyncio.wait_for(reader.readexactly(8), 10)
            if hdr != C.PROTOCOL_HEADER:
                writer.write(C.PROTOCOL_HEADER)
                writer.close()
                return
            conn.send(C.method_frame(0, C.CONNECTION_START, 0, 9,
                                     {"product": "downloader-amd-broker",
                                      "capabilities": {"publisher_confirms": True,
                                                       "basic.nack": True,
                                                       "consumer_cancel_notify": True}},
                                     "PLAIN", "en_US"))
            m, a = await self._expect(conn, C.CONNECTION_START_OK)
            parts = bytes(a[2]).split(b"\x00")
            user = parts[1].decode() if len(parts) > 2 else ""
            pw = parts[2].decode() if len(parts) > 2 else ""
            if self.users and self.users.get(user) != pw:
                conn.send(C.method_frame(0, C.CONNECTION_CLOSE, 403, "ACCESS_REFUSED", 10, 11))
                await writer.drain()
                writer.close()
                return
            conn.send(C.method_frame(0, C.CONNECTION_TUNE, 2047, self.frame_max, self.heartbeat))
            m, a = await self._expect(conn, C.CONNECTION_TUNE_OK)
            conn.frame_max = a[1] or self.frame_max
            conn.heartbeat = a[2]
            await self._expect(conn, C.CONNECTION_OPEN)
            conn.send(C.method_frame(0, C.CONNECTION_OPEN_OK, ""))
            self.conns.append(conn)
            hb = asyncio.get_running_loop().create_task(self._heartbeats(conn)) if conn.heartbeat else None
            try:
                await self._loop(conn)
            finally:
                if hb is not None:
                    hb.cancel()
        except (asyncio.IncompleteReadError, ConnectionError, OSError, asyncio.TimeoutError,
                C.FrameError):
            pass
        finally:
            conn.closed = True
            if conn in self.conns:
                self.conns.remove(conn)
            for ch in list(conn.chans.values()):
                self._close_channel(ch)
            try:
                writer.close()
            except Exception:
                pass

    async def _expect(self, conn: _Conn, want) -> Tuple[Tuple[int, int], list]:
        while True:
            ftype, ch, payload = await asyncio.wait_for(C.read_frame(conn.reader), 30)
            if ftype == C.FRAME_METHOD:
                m, a = C.decode_method(payload)
                if m == want:
                    return m, a
                raise C.FrameError(f"expected {want}, got {m}")

    async def _heartbeats(self, conn: _Conn) -> None:
        while not conn.closed:
            await asyncio.sleep(max(1.0, conn.heartbeat / 2))
            conn.send(C.heartbeat_frame())

    async def _loop(self, conn: _Conn) -> None:
        timeout = conn.heartbeat * 3 if conn.heartbeat else None
        while not conn.closed:
            ftype, cid, payload = await asyncio.wait_for(C.read_frame(conn.reader), timeout)
            if ftype == C.FRAME_HEARTBEAT:
                continue
            if cid == 0:
                if ftype == C.FRAME_METHOD:
                    m, a = C.decode_method(payload)
                    if m == C.CONNECTION_CLOSE:
                        conn.send(C.method_frame(0, C.CONNECTION_CLOSE_OK))
                        await conn.writer.drain()
                        return
                continue
            if ftype == C.FRAME_METHOD:
                m, a = C.decode_method(payload)
                self._method(conn, cid, m, a)
            elif ftype == C.FRAME_HEADER:
                ch = conn.chans.get(cid)
                if ch is not None and ch.pending is not None:
                    ch.pending_size, ch.pending_props = C.decode_header(payload)
                    if ch.pending_size == 0:
                        self._route(ch)
            elif ftype == C.FRAME_BODY:
                ch = conn.chans.get(cid)
                if ch is not None and ch.pending is not None:
                    ch.pending_body.append(payload)
                    if sum(len(b) for b in ch.pending_body) >= ch.pending_size:
                        self._route(ch)
            if conn.writer.transport.get_write_buffer_size() > 4 << 20:
                await conn.writer.drain()

    # ---------------------------------------------------------------- methods
    def _chan_error(self, ch: _Chan, code: int, text: str, m: Tuple[int, int]) -> None:
        ch.conn.send(C.method_frame(ch.id, C.CHANNEL_CLOSE, code, text, m[0], m[1]))
        self._close_channel(ch)

    def _method(self, conn: _Conn, cid: int, m: Tuple[int, int], a: list) -> None:
        if m == C.CHANNEL_OPEN:
            conn.chans[cid] = _Chan(conn, cid)
            conn.send(C.method_frame(cid, C.CHANNEL_OPEN_OK, b""))
            return
        ch = conn.chans.get(cid)
        if ch is None:
            return
        if m == C.CHANNEL_CLOSE:
            self._close_channel(ch)
            conn.send(C.method_frame(cid, C.CHANNEL_CLOSE_OK))
        elif m == C.CHANNEL_CLOSE_OK:
            self._close_channel(ch)
        elif m == C.QUEUE_DECLARE:
            name, passive = a[1], a[2]
            if not name:
                name = f"amq.gen-{next(self._ctags)}"
            q = self.queues.get(name)
            if q is None:
                if passive:
                    self._chan_error(ch, 404, f"NOT_FOUND - no queue '{name}'", m)
                    return
                q = self.queues[name] = _Queue(name, args=dict(a[7] or {}))
            if not a[6]:
                conn.send(C.method_frame(cid, C.QUEUE_DECLARE_OK, name, len(q.msgs), len(q.consumers)))
        elif m == C.QUEUE_PURGE:
            q = self.queues.get(a[1])
            n = len(q.msgs) if q else 0
            if q:
                q.msgs.clear()
            conn.send(C.method_frame(cid, C.QUEUE_PURGE_OK, n))
        elif m == C.QUEUE_DELETE:
            n = self.delete_queue(a[1])
            conn.send(C.method_frame(cid, C.QUEUE_DELETE_OK, n))
        elif m == C.BASIC_QOS:
            ch.prefetch = a[1]
            conn.send(C.method_frame(cid, C.BASIC_QOS_OK))
        elif m == C.BASIC_CONSUME:
            qname, tag = a[1], a[2] or f"amq.ctag-{next(self._ctags)}"
            q = self.queues.get(qname)
            if q is None:
                self._chan_error(ch, 404, f"NOT_FOUND - no queue '{qname}'", m)
                return
            c = _Consumer(tag, qname, ch, ch.prefetch)
            ch.consumers[tag] = c
            q.consumers.append(c)
            if not a[6]:
                conn.send(C.method_frame(cid, C.BASIC_CONSUME_OK, tag))
            self._dispatch(q)
        elif m == C.BASIC_CANCEL:
            c = ch.consumers.pop(a[0], None)
            if c is not None:
                q = self.queues.get(c.queue)
                if q is not None and c in q.consumers:
                    q.consumers.remove(c)
            if not a[1]:
                conn.send(C.method_frame(cid, C.BASIC_CANCEL_OK, a[0]))
        elif m == C.BASIC_PUBLISH:
            ch.pending = (a[1], a[2])
            ch.pending_body = []
            ch.pending_props = None
        elif m == C.BASIC_GET:
            q = self.queues.get(a[1])
            if q is None or not q.msgs:
                conn.send(C.method_frame(cid, C.BASIC_GET_EMPTY, ""))
                return
            msg = q.msgs.popleft()
            tag = next(ch.dtags)
            if not a[2]:
                ch.unacked[tag] = (q.name, msg, None, time.monotonic())
            conn.send(C.content_frames(cid, C.method_frame(cid, C.BASIC_GET_OK, tag, msg.redelivered,
                                                           "", q.name, len(q.msgs)),
                                       msg.body, msg.props, conn.frame_max))
        elif m == C.BASIC_ACK:
            self._settle(ch, a[0], a[1], requeue=None)
        elif m == C.BASIC_NACK:
            self._settle(ch, a[0], a[1], requeue=a[2])
        elif m == C.BASIC_REJECT:
            self._settle(ch, a[0], False, requeue=a[1])
        elif m == C.BASIC_RECOVER:
            self._requeue_all(ch)
            conn.send(C.method_frame(cid, C.BASIC_RECOVER_OK))
        elif m == C.CONFIRM_SELECT:
            ch.confirming = True
            if not a[0]:
                conn.send(C.method_frame(cid, C.CONFIRM_SELECT_OK))
        elif m == C.CHANNEL_FLOW:
            conn.send(C.method_frame(cid, C.CHANNEL_FLOW_OK, a[0]))

    def _route(self, ch: _Chan) -> None:
        exchange, rkey = ch.pending or ("", "")
        body = b"".join(ch.pending_body)
        props = ch.pending_props or C.Properties()
        ch.pending = None
        ch.pending_body = []
        if exchange == "":
            self._enqueue(rkey, _Msg(body, props))
        if ch.confirming:
            ch.pub_seq += 1
            ch.conn.send(C.method_frame(ch.id, C.BASIC_ACK, ch.pub_seq, False))

    def _enqueue(self, qname: str, msg: _Msg) -> None:
        q = self.queues.get(qname)
        if q is None:
            return                              # unroutable on the default exchange: dropped
        ttl = q.args.get("x-message-ttl")
        if isinstance(ttl, int) and ttl >= 0:
            msg.expires = time.monotonic() + ttl / 1000.0
        q.msgs.append(msg)
        q.published += 1
        self._dispatch(q)
        self._arm_expiry(q)

    def _arm_expiry(self, q: _Queue) -> None:
        if q.timer is not None or not q.msgs or not q.msgs[0].expires:
            return
        delay = max(0.0, q.msgs[0].expires - time.monotonic())
        q.timer = asyncio.get_running_loop().call_later(delay, self._expire, q)

    def _expire(self, q: _Queue) -> None:
        """Dead-letter expired messages from the head (RabbitMQ expires at the head only)."""
        q.timer = None
        now = time.monotonic()
        while q.msgs and q.msgs[0].expires and q.msgs[0].expires <= now:
            msg = q.msgs.popleft()
            q.expired += 1
            if "x-dead-letter-exchange" not in q.args:
                continue                        # no DLX: expired messages are dropped
            rkey = q.args.get("x-dead-letter-routing-key") or q.name
            hdrs = dict(msg.props.headers or {})
            deaths = list(hdrs.get("x-death") or [])
            # as RabbitMQ: one entry per (queue, reason), its count bumped and moved first
            prev = next((d for d in deaths if isinstance(d, dict) and d.get("queue") == q.name
                         and d.get("reason") == "expired"), None)
            if prev is not None:
                deaths.remove(prev)
            deaths.insert(0, {"queue": q.name, "reason": "expired",
                              "count": int(prev.get("count", 0)) + 1 if prev else 1,
                              "exchange": "", "routing-keys": [q.name]})
            hdrs["x-death"] = deaths
            props = dataclasses.replace(msg.props, headers=hdrs)
            if q.args.get("x-dead-letter-exchange", "") == "":
                self._enqueue(rkey, _Msg(msg.body, props))
        if q.name in self.queues:
            self._arm_expiry(q)

    def _dispatch(self, q: _Queue) -> None:
        while q.msgs and q.consumers:
            n = len(q.consumers)
            target = None
            for k in range(n):
                c = q.consumers[(q.rr + k) % n]
                if not c.chan.conn.closed and (c.prefetch == 0 or c.unacked < c.prefetch):
                    target = c
                    q.rr = (q.rr + k + 1) % n
                    break
            if target is None:
                return
            msg = q.msgs.popleft()
            ch = target.chan
            tag = next(ch.dtags)
            ch.unacked[tag] = (q.name, msg, target, time.monotonic())
            target.unacked += 1
            q.delivered += 1
            ch.conn.send(C.content_frames(
                ch.id, C.method_frame(ch.id, C.BASIC_DELIVER, target.tag, tag, msg.redelivered, "", q.name),
                msg.body, msg.props, ch.conn.frame_max))

    def _settle(self, ch: _Chan, tag: int, multiple: bool, requeue: Optional[bool]) -> None:
        tags = [t for t in ch.unacked if t <= tag] if multiple else [tag]
        touched = set()
        for t in sorted(tags, reverse=True):
            ent = ch.unacked.pop(t, None)
            if ent is None:
                continue
            qname, msg, cons, _ = ent
            if cons is not None:
                cons.unacked -= 1
            q = self.queues.get(qname)
            if q is None:
                continue
            if requeue:
                msg.redelivered = True
                q.msgs.appendleft(msg)
            touched.add(qname)
        for qn in touched:
            q = self.queues.get(qn)
            if q is not None:
                self._dispatch(q)

    def _requeue_all(self, ch: _Chan) -> None:
        if ch.unacked:
            self._settle(ch, max(ch.unacked), True, requeue=True)

    def _close_channel(self, ch: _Chan) -> None:
        for c in list(ch.consumers.values()):
            q = self.queues.get(c.queue)
            if q is not None and c in q.consumers:
                q.consumers.remove(c)
        ch.consumers.clear()
        self._requeue_all(ch)
        ch.conn.chans.pop(ch.id, None)


async def run_broker(host: str = "0.0.0.0", port: int = 5672, consumer_timeout: float = 0.0,
                     certfile: str = "", keyfile: str = "", client_ca: str = "") -> None:
    ctx = None
    if certfile:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(certfile, keyfile or None)
        if client_ca:      # mutual TLS: clients must present a certificate from this CA
            ctx.load_verify_locations(cafile=client_ca)
            ctx.verify_mode = ssl.CERT_REQUIRED
    srv = BrokerServer(host, port, consumer_timeout=consumer_timeout, ssl_context=ctx)
    await srv.start()
    print(f"broker listening on {host}:{srv.port}", flush=True)
    while True:
        await asyncio.sleep(3600)
