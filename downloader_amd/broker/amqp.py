"""Asyncio AMQP 0-9-1 client and the ``Broker`` implementation on top of it.

Replaces ``triton-core/amqp`` (amqplib + amqp-connection-manager, yarn.lock:189-204; used at
reference lib/main.js:46-47,145,150,164,168,172,200): PLAIN auth, tune/heartbeats, one
channel for consuming (``basic.qos`` prefetch + ``basic.consume``) and one for publishing
with publisher confirms, ``basic.ack``/``basic.nack``, and automatic reconnect that
re-declares queues and re-subscribes consumers (unacked deliveries of a dead connection are
requeued by the broker, so they are redelivered with ``redelivered=True``).
"""
from __future__ import annotations

import asyncio
import itertools
import platform
from typing import Any, Awaitable, Callable, Dict, List, Optional, Tuple
from urllib.parse import unquote, urlsplit

from . import amqp_codec as C
from .base import Broker, Delivery, Handler, Headers


def parse_url(url: str) -> Tuple[str, int, str, str, str]:
    u = urlsplit(url)
    if u.scheme not in ("amqp", ""):
        raise ValueError("only amqp:// URLs are supported (amqps needs TLS termination)")
    vhost = unquote(u.path[1:]) if u.path and u.path != "/" else "/"
    return (u.hostname or "127.0.0.1", u.port or 5672, unquote(u.username or "guest"),
            unquote(u.password or "guest"), vhost)


class Message:
    def __init__(self, channel: "Channel", delivery_tag: int, redelivered: bool, exchange: str,
                 routing_key: str, props: C.Properties, body: bytes, consumer_tag: str = ""):
        self.channel = channel
        self.delivery_tag = delivery_tag
        self.redelivered = redelivered
        self.exchange = exchange
        self.routing_key = routing_key
        self.props = props
        self.body = body
        self.consumer_tag = consumer_tag


class Channel:
    def __init__(self, conn: "Connection", cid: int):
        self.conn = conn
        self.id = cid
        self._rpc_lock = asyncio.Lock()
        self._waiter: Optional[asyncio.Future] = None
        self._expect: Tuple[Tuple[int, int], ...] = ()
        self.consumers: Dict[str, Callable[[Message], Awaitable[None]]] = {}
        self.closed = False
        self.confirming = False
        self._publish_seq = 0
        self._confirms: Dict[int, asyncio.Future] = {}
        # content assembly
        self._pending_method: Optional[Tuple[Tuple[int, int], List[Any]]] = None
        self._pending_props: Optional[C.Properties] = None
        self._pending_size = 0
        self._pending_body: List[bytes] = []
        self._get_waiter: Optional[asyncio.Future] = None

    async def rpc(self, method: Tuple[int, int], args: List[Any],
                  expect: Tuple[Tuple[int, int], ...]) -> Tuple[Tuple[int, int], List[Any]]:
        async with self._rpc_lock:
            if self.closed:
                raise C.AMQPError("channel closed")
            fut = asyncio.get_running_loop().create_future()
            self._waiter, self._expect = fut, expect
            self.conn.send(C.method_frame(self.id, method, *args))
            try:
                return await asyncio.wait_for(fut, self.conn.rpc_timeout)
            finally:
                self._waiter = None

    def _on_method(self, m: Tuple[int, int], args: List[Any]) -> None:
        if m in C.CONTENT_METHODS:
            self._pending_method = (m, args)
            self._pending_body = []
            return
        if m == C.BASIC_ACK and self.confirming:
            self._settle_confirms(args[0], args[1], True)
            return
        if m == C.BASIC_NACK and self.confirming:
            self._settle_confirms(args[0], args[1], False)
            return
        if m == C.CHANNEL_CLOSE:
            self.closed = True
            self.conn.send(C.method_frame(self.id, C.CHANNEL_CLOSE_OK))
            err = C.AMQPError(f"channel closed by broker: {args[0]} {args[1]}", args[0])
            self._fail(err)
            return
        if m == C.BASIC_CANCEL:  # broker-side cancel (queue deleted)
            self.consumers.pop(args[0], None)
            return
        if m == C.BASIC_GET_EMPTY and self._get_waiter is not None:
            if not self._get_waiter.done():
                self._get_waiter.set_result(None)
            return
        if self._waiter is not None and not self._waiter.done() and m in self._expect:
            self._waiter.set_result((m, args))

    def _fail(self, err: BaseException) -> None:
        if self._waiter is not None and not self._waiter.done():
            self._waiter.set_exception(err)
        if self._get_waiter is not None and not self._get_waiter.done():
            self._get_waiter.set_exception(err)
        for f in self._confirms.values():
            if not f.done():
                f.set_exception(err)
        self._confirms.clear()

    def _settle_confirms(self, tag: int, multiple: bool, ok: bool) -> None:
        tags = [t for t in self._confirms if t <= tag] if multiple else [tag]
        for t in tags:
            f = self._confirms.pop(t, None)
            if f is not None and not f.done():
                if ok:
                    f.set_result(True)
                else:
                    f.set_exception(C.AMQPError("message nacked by broker"))

    def _on_header(self, payload: bytes) -> None:
        self._pending_size, self._pending_props = C.decode_header(payload)
        if self._pending_size == 0:
            self._complete_content()

    def _on_body(self, payload: bytes) -> None:
        self._pending_body.append(payload)
        if sum(len(b) for b in self._pending_body) >= self._pending_size:
            self._complete_content()

    def _complete_content(self) -> None:
        if self._pending_method is None:
            return
        (m, args), props = self._pending_method, self._pending_props or C.Properties()
        body = b"".join(self._pending_body)
        self._pending_method = None
        self._pending_body = []
        if m == C.BASIC_DELIVER:
            ctag, dtag, redelivered, exch, rkey = args
            msg = Message(self, dtag, redelivered, exch, rkey, props, body, ctag)
            cb = self.consumers.get(ctag)
            if cb is not None:
                self.conn._spawn(cb(msg))
        elif m == C.BASIC_GET_OK:
            dtag, redelivered, exch, rkey, _count = args
            if self._get_waiter is not None and not self._get_waiter.done():
                self._get_waiter.set_result(Message(self, dtag, redelivered, exch, rkey, props, body))

    # ---------------------------------------------------------------- API
    async def queue_declare(self, queue: str, durable: bool = True, passive: bool = False,
                            arguments: Optional[Dict[str, Any]] = None) -> Tuple[str, int, int]:
        _, a = await self.rpc(C.QUEUE_DECLARE, [0, queue, passive, durable, False, False, False,
                                                arguments or {}], (C.QUEUE_DECLARE_OK,))
        return a[0], a[1], a[2]

    async def queue_purge(self, queue: str) -> int:
        _, a = await self.rpc(C.QUEUE_PURGE, [0, queue, False], (C.QUEUE_PURGE_OK,))
        return a[0]

    async def queue_delete(self, queue: str) -> int:
        _, a = await self.rpc(C.QUEUE_DELETE, [0, queue, False, False, False], (C.QUEUE_DELETE_OK,))
        return a[0]

    async def basic_qos(self, prefetch_count: int) -> None:
        await self.rpc(C.BASIC_QOS, [0, prefetch_count, False], (C.BASIC_QOS_OK,))

    async def basic_consume(self, queue: str, cb: Callable[[Message], Awaitable[None]],
                            consumer_tag: str = "") -> str:
        _, a = await self.rpc(C.BASIC_CONSUME, [0, queue, consumer_tag, False, False, False, False,
                                                {}], (C.BASIC_CONSUME_OK,))
        self.consumers[a[0]] = cb
        return a[0]

    async def basic_cancel(self, consumer_tag: str) -> None:
        await self.rpc(C.BASIC_CANCEL, [consumer_tag, False], (C.BASIC_CANCEL_OK,))
        self.consumers.pop(consumer_tag, None)

    async def confirm_select(self) -> None:
        await self.rpc(C.CONFIRM_SELECT, [False], (C.CONFIRM_SELECT_OK,))
        self.confirming = True

    async def basic_publish(self, exchange: str, routing_key: str, body: bytes,
                            props: Optional[C.Properties] = None, wait_confirm: bool = True) -> None:
        if self.closed:
            raise C.AMQPError("channel closed")
        fut = None
        if self.confirming:
            self._publish_seq += 1            # the broker numbers every publish
            if wait_confirm:                  # fire-and-forget: no future to leave unread
                fut = asyncio.get_running_loop().create_future()
                self._confirms[self._publish_seq] = fut
        data = C.content_frames(self.id, C.method_frame(self.id, C.BASIC_PUBLISH, 0, exchange,
                                                        routing_key, False, False),
                                bytes(body), props or C.Properties(), self.conn.frame_max)
        self.conn.send(data)
        await self.conn.drain()
        if fut is not None and wait_confirm:
            await asyncio.wait_for(fut, self.conn.rpc_timeout)

    async def basic_get(self, queue: str, no_ack: bool = False) -> Optional[Message]:
        async with self._rpc_lock:
            fut = asyncio.get_running_loop().create_future()
            self._get_waiter = fut
            self.conn.send(C.method_frame(self.id, C.BASIC_GET, 0, queue, no_ack))
            try:
                return await asyncio.wait_for(fut, self.conn.rpc_timeout)
            finally:
                self._get_waiter = None

    def basic_ack(self, tag: int, multiple: bool = False) -> bool:
        """False when the channel or its connection is gone: the broker requeues every
        unacked delivery of a dead channel, so there is nothing left to settle."""
        return self._settle(C.method_frame(self.id, C.BASIC_ACK, tag, multiple))

    def basic_nack(self, tag: int, requeue: bool = True, multiple: bool = False) -> bool:
        return self._settle(C.method_frame(self.id, C.BASIC_NACK, tag, multiple, requeue))

    def _settle(self, frame: bytes) -> bool:
        if self.closed:
            return False
        try:
            self.conn.send(frame)
        except ConnectionError:
            return False
        return True

    async def close(self) -> None:
        if self.closed:
            return
        try:
            await self.rpc(C.CHANNEL_CLOSE, [200, "bye", 0, 0], (C.CHANNEL_CLOSE_OK,))
        except Exception:
            pass
        self.closed = True
        self.conn.channels.pop(self.id, None)


class Connection:
    def __init__(self, url: str, heartbeat: int = 30, frame_max: int = 131072,
                 rpc_timeout: float = 30.0, connect_timeout: float = 10.0):
        self.host, self.port, self.user, self.password, self.vhost = parse_url(url)
        self.heartbeat = heartbeat
        self.frame_max = frame_max
        self.rpc_timeout = rpc_timeout
        self.connect_timeout = connect_timeout
        self.channels: Dict[int, Channel] = {}
        self._ids = itertools.count(1)
        self.reader: Optional[asyncio.StreamReader] = None
        self.writer: Optional[asyncio.StreamWriter] = None
        self._reader_task: Optional[asyncio.Task] = None
        self._hb_task: Optional[asyncio.Task] = None
        self._tasks: set = set()
        self.closed = asyncio.Event()
        self.close_reason: Optional[BaseException] = None
        self.server_properties: Dict[str, Any] = {}

    def _spawn(self, coro) -> None:
        t = asyncio.get_running_loop().create_task(coro)
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)

    def send(self, data: bytes) -> None:
        if self.writer is None or self.writer.is_closing():
            raise ConnectionError("AMQP connection is closed")
        self.writer.write(data)

    async def drain(self) -> None:
        if self.writer is not None and self.writer.transport.get_write_buffer_size() > 1 << 20:
            await self.writer.drain()

    async def connect(self) -> "Connection":
        self.reader, self.writer = await asyncio.wait_for(
            asyncio.open_connection(self.host, self.port), self.connect_timeout)
        self.writer.write(C.PROTOCOL_HEADER)
        m, a = await self._expect_method(C.CONNECTION_START)
        self.server_properties = a[2]
        props = {"product": "downloader-amd", "platform": platform.python_version(),
                 "capabilities": {"publisher_confirms": True, "consumer_cancel_notify": True,
                                  "basic.nack": True}}
        resp = b"\x00" + self.user.encode() + b"\x00" + self.password.encode()
        self.writer.write(C.method_frame(0, C.CONNECTION_START_OK, props, "PLAIN", resp, "en_US"))
        m, a = await self._expect_method(C.CONNECTION_TUNE)
        chmax = a[0] or 2047
        fmax = min(a[1] or self.frame_max, self.frame_max)
        hb = min(a[2], self.heartbeat) if a[2] and self.heartbeat else (a[2] or self.heartbeat)
        self.frame_max, self.heartbeat = max(fmax, C.FRAME_MIN), hb
        self.writer.write(C.method_frame(0, C.CONNECTION_TUNE_OK, chmax, self.frame_max, hb))
        self.writer.write(C.method_frame(0, C.CONNECTION_OPEN, self.vhost, "", False))
        m, a = await self._expect_method(C.CONNECTION_OPEN_OK, C.CONNECTION_CLOSE)
        if m == C.CONNECTION_CLOSE:
            raise C.AMQPError(f"connection refused: {a[0]} {a[1]}", a[0])
        self._reader_task = asyncio.get_running_loop().create_task(self._read_loop())
        if self.heartbeat:
            self._hb_task = asyncio.get_running_loop().create_task(self._heartbeats())
        return self

    async def _expect_method(self, *want) -> Tuple[Tuple[int, int], List[Any]]:
        while True:
            ftype, ch, payload = await asyncio.wait_for(C.read_frame(self.reader),
                                                        self.connect_timeout)
            if ftype == C.FRAME_HEARTBEAT:
                continue
            if ftype != C.FRAME_METHOD:
                raise C.FrameError("unexpected frame during handshake")
            m, a = C.decode_method(payload)
            if m in want:
                return m, a
            if m == C.CONNECTION_CLOSE:
                raise C.AMQPError(f"connection closed: {a[0]} {a[1]}", a[0])

    async def _heartbeats(self) -> None:
        while not self.closed.is_set():
            await asyncio.sleep(max(1.0, self.heartbeat / 2))
            try:
                self.send(C.heartbeat_frame())
            except ConnectionError:
                return

    async def _read_loop(self) -> None:
        err: Optional[BaseException] = None
        timeout = self.heartbeat * 3 if self.heartbeat else None
        try:
            while True:
                ftype, ch, payload = await asyncio.wait_for(C.read_frame(self.reader), timeout)
                if ftype == C.FRAME_HEARTBEAT:
                    continue
                if ch == 0:
                    if ftype == C.FRAME_METHOD:
                        m, a = C.decode_method(payload)
                        if m == C.CONNECTION_CLOSE:
                            self.send(C.method_frame(0, C.CONNECTION_CLOSE_OK))
                            err = C.AMQPError(f"connection closed by broker: {a[0]} {a[1]}", a[0])
                            break
                        if m == C.CONNECTION_CLOSE_OK:
                            break
                    continue
                chan = self.channels.get(ch)
                if chan is None:
                    continue
                if ftype == C.FRAME_METHOD:
                    m, a = C.decode_method(payload)
                    chan._on_method(m, a)
                elif ftype == C.FRAME_HEADER:
                    chan._on_header(payload)
                elif ftype == C.FRAME_BODY:
                    chan._on_body(payload)
        except (asyncio.IncompleteReadError, ConnectionError, OSError, asyncio.TimeoutError,
                C.FrameError) as e:
            err = e
        finally:
            self.close_reason = err
            for chan in self.channels.values():
                chan.closed = True
                chan._fail(err or ConnectionError("connection closed"))
            self.closed.set()
            if self.writer is not None:
                self.writer.close()

    async def channel(self) -> Channel:
        cid = next(self._ids)
        ch = Channel(self, cid)
        self.channels[cid] = ch
        await ch.rpc(C.CHANNEL_OPEN, [""], (C.CHANNEL_OPEN_OK,))
        return ch

    async def close(self) -> None:
        if self.closed.is_set():
            return
        try:
            self.send(C.method_frame(0, C.CONNECTION_CLOSE, 200, "bye", 0, 0))
            await asyncio.wait_for(self.closed.wait(), 2.0)
        except Exception:
            pass
        for t in (self._reader_task, self._hb_task):
            if t is not None:
                t.cancel()
        if self.writer is not None:
            self.writer.close()
        self.closed.set()


# ---------------------------------------------------------------- Broker implementation
def _to_headers(h: Optional[Headers]) -> Dict[str, Any]:
    return {k: v for k, v in (h or {}).items() if v is not None}


class _AmqpDelivery(Delivery):
    def __init__(self, msg: Message, queue: str, gen: int, broker: "AmqpBroker"):
        super().__init__(queue, msg.body, msg.props.headers or {}, msg.redelivered, msg.delivery_tag)
        self._msg = msg
        self._gen = gen
        self._b = broker

    async def _ack(self) -> None:
        if self._gen == self._b._gen:   # acks for a dead connection are moot (broker requeued)
            self._msg.channel.basic_ack(self._msg.delivery_tag)

    async def _nack(self, requeue: bool) -> None:
        if self._gen == self._b._gen:
            self._msg.channel.basic_nack(self._msg.delivery_tag, requeue)


class AmqpBroker(Broker):
    def __init__(self, url: str, heartbeat: int = 30, reconnect_delay: float = 1.0,
                 max_reconnect_delay: float = 30.0, metrics=None, connect_retry_s: float = 0.0,
                 publish_retry_s: float = 120.0):
        self.url = url
        self.publish_retry_s = publish_retry_s
        self.connect_retry_s = connect_retry_s
        self.heartbeat = heartbeat
        self.reconnect_delay = reconnect_delay
        self.max_reconnect_delay = max_reconnect_delay
        self.metrics = metrics
        self.conn: Optional[Connection] = None
        self._cons_ch: Optional[Channel] = None
        self._pub_ch: Optional[Channel] = None
        self._declared: set = set()
        self._consumers: Dict[str, Tuple[str, Handler, int]] = {}
        self._ctags: Dict[str, str] = {}    # our tag -> broker tag (current connection)
        self._ids = itertools.count(1)
        self._gen = 0
        self._lock = asyncio.Lock()
        self._closing = False
        self._watch: Optional[asyncio.Task] = None
        self.connected = False
        self.reconnects = 0

    async def connect(self) -> None:
        deadline = asyncio.get_running_loop().time() + self.connect_retry_s
        delay = self.reconnect_delay
        while True:
            try:
                async with self._lock:
                    if self.connected:
                        return
                    await self._open()
                break
            except (OSError, C.AMQPError, asyncio.TimeoutError, ConnectionError):
                # amqp-connection-manager semantics: keep trying while the broker comes up
                if asyncio.get_running_loop().time() + delay > deadline:
                    raise
                await asyncio.sleep(delay)
                delay = min(self.max_reconnect_delay, delay * 2)
        self._watch = asyncio.get_running_loop().create_task(self._watchdog())

    async def _open(self) -> None:
        self.conn = await Connection(self.url, self.heartbeat).connect()
        self._cons_ch = await self.conn.channel()
        self._pub_ch = await self.conn.channel()
        await self._pub_ch.confirm_select()
        self._gen += 1
        for q in list(self._declared):
            await self._cons_ch.queue_declare(q)
        for tag, (q, handler, prefetch) in list(self._consumers.items()):
            await self._subscribe(tag, q, handler, prefetch)
        self.connected = True

    async def _watchdog(self) -> None:
        delay = self.reconnect_delay
        while not self._closing:
            await self.conn.closed.wait()
            self.connected = False
            if self._closing:
                return
            while not self._closing:
                await asyncio.sleep(delay)
                try:
                    async with self._lock:
                        await self._open()
                    self.reconnects += 1
                    delay = self.reconnect_delay
                    break
                except (OSError, C.AMQPError, asyncio.TimeoutError, ConnectionError):
                    delay = min(self.max_reconnect_delay, delay * 2)

    async def _ready(self) -> None:
        for _ in range(int(max(1.0, self.max_reconnect_delay) * 20)):
            if self.connected and self.conn is not None and not self.conn.closed.is_set():
                return
            if self._closing:
                break
            await asyncio.sleep(0.05)
        raise ConnectionError("AMQP broker not connected")

    async def close(self) -> None:
        self._closing = True
        if self._watch is not None:
            self._watch.cancel()
        if self.conn is not None:
            await self.conn.close()
        self.connected = False

    async def declare(self, queue: str) -> None:
        self._declared.add(queue)
        await self._ready()
        await self._cons_ch.queue_declare(queue)

    async def publish(self, queue: str, body: bytes, headers: Optional[Headers] = None,
                      confirm: bool = True) -> None:
        """Publish (with a broker confirm unless ``confirm=False``). A connection lost before
        the confirm arrives is not an error: the message is sent again once the watchdog has
        reconnected, as amqp-connection-manager's ChannelWrapper does - at-least-once, so a
        consumer may see it twice. Channel-level refusals on a live connection still raise,
        and so does a broker that stays away for ``publish_retry_s``."""
        props = C.Properties(content_type="application/octet-stream", delivery_mode=2,
                             headers=_to_headers(headers))
        loop = asyncio.get_running_loop()
        deadline = loop.time() + self.publish_retry_s
        while True:
            await self._ready()
            conn = self.conn
            try:
                await self._pub_ch.basic_publish("", queue, body, props, wait_confirm=confirm)
                break
            except Exception:   # reset, EOF mid-frame, timeout, channel failure...
                lost = conn is None or conn.closed.is_set() or conn is not self.conn
                if not lost or self._closing or loop.time() > deadline:
                    raise
                if self.metrics is not None:
                    self.metrics.messages.labels(queue, "republish").inc()
                await asyncio.sleep(0.02)   # the watchdog is reconnecting; _ready() waits
        if self.metrics is not None:
            self.metrics.messages.labels(queue, "publish").inc()

    async def _subscribe(self, tag: str, queue: str, handler: Handler, prefetch: int) -> None:
        gen = self._gen

        async def on_msg(msg: Message) -> None:
            d = _AmqpDelivery(msg, queue, gen, self)
            try:
                await handler(d)
            except Exception:
                if not d.settled:
                    await d.nack(requeue=True)

        await self._cons_ch.queue_declare(queue)
        await self._cons_ch.basic_qos(prefetch)
        self._ctags[tag] = await self._cons_ch.basic_consume(queue, on_msg)

    async def consume(self, queue: str, handler: Handler, prefetch: int = 1) -> str:
        await self._ready()
        tag = f"amqp-ctag-{next(self._ids)}"
        self._consumers[tag] = (queue, handler, prefetch)
        self._declared.add(queue)
        await self._subscribe(tag, queue, handler, prefetch)
        return tag

    async def cancel(self, consumer_tag: str) -> None:
        self._consumers.pop(consumer_tag, None)
        btag = self._ctags.pop(consumer_tag, None)
        if btag and self.connected:
            try:
                await self._cons_ch.basic_cancel(btag)
            except Exception:
                pass

    async def get(self, queue: str) -> Optional[Delivery]:
        await self._ready()
        msg = await self._cons_ch.basic_get(queue)
        if msg is None:
            return None
        return _AmqpDelivery(msg, queue, self._gen, self)

    async def queue_size(self, queue: str) -> int:
        await self._ready()
        _, n, _ = await self._cons_ch.queue_declare(queue)
        return n
