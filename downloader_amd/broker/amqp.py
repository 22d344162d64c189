"""Asyncio AMQP 0-9-1 client and the ``Broker`` implementation on top of it.

Replaces ``triton-core/amqp`` (amqplib + amqp-connection-manager, yarn.lock:189-204; used at
reference lib/main.js:46-47,145,150,164,168,172,200): PLAIN auth, tune/heartbeats, one
channel for consuming (``basic.qos`` prefetch + ``basic.consume``) and one for publishing
with publisher confirms, ``basic.ack``/``basic.nack``, and automatic reconnect that
re-declares queues and re-subscribes consumers (unacked deliveries of a dead connection are
requeued by the broker, so they are redelivered with ``redelivered=True``).

Liveness below the connection (amqp-connection-manager re-runs its channel setup whenever a
channel dies): a broker ``channel.close`` (RabbitMQ's ``consumer_timeout`` on a long job, a
406 on a bad ack, a 404 on a deleted queue) reopens that channel on the live connection and
re-runs setup; a broker ``basic.cancel`` (queue deleted, node failover) re-declares the queue
and re-consumes with backoff. When the setup itself fails the connection is aborted and the
reconnect watchdog takes over. ``consumer_live()`` is what ``/readyz`` reports.

``amqps://`` (port 5671) runs the same protocol over asyncio TLS (``tls.verify``,
``tls.ca_file``), as amqplib does for ``dyn('rabbitmq')`` URLs (lib/main.js:46).
"""
from __future__ import annotations

import asyncio
import itertools
import platform
import ssl
from typing import Any, Awaitable, Callable, Dict, List, Optional, Tuple
from urllib.parse import unquote, urlsplit

from . import amqp_codec as C
from .base import Broker, Delivery, Handler, Headers


def parse_url(url: str) -> Tuple[str, int, str, str, str]:
    """``(host, port, user, password, vhost)`` of an ``amqp://`` / ``amqps://`` URL."""
    u = urlsplit(url)
    if u.scheme not in ("amqp", "amqps", ""):
        raise ValueError(f"not an AMQP URL (amqp:// or amqps://): {u.scheme}://")
    vhost = unquote(u.path[1:]) if u.path and u.path != "/" else "/"
    port = u.port or (5671 if u.scheme == "amqps" else 5672)
    return (u.hostname or "127.0.0.1", port, unquote(u.username or "guest"),
            unquote(u.password or "guest"), vhost)


def is_tls_url(url: str) -> bool:
    return urlsplit(url).scheme == "amqps"


def client_ssl_context(verify: bool = True, ca_file: str = "", cert_file: str = "",
                       key_file: str = "") -> ssl.SSLContext:
    """TLS for ``amqps://``: the system trust store plus ``ca_file`` (a private CA, the
    usual RabbitMQ setup); ``verify=False`` accepts any certificate. ``cert_file`` (+
    ``key_file``, else the key is in the same PEM): a client certificate for brokers that
    require one (RabbitMQ ``ssl_options.fail_if_no_peer_cert``; amqplib's ``cert`` / ``key``
    socket options)."""
    ctx = ssl.create_default_context()
    if ca_file:
        ctx.load_verify_locations(cafile=ca_file)
    if cert_file:
        ctx.load_cert_chain(cert_file, key_file or None)
    if not verify:
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
    return ctx


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
        # owner hooks: broker-initiated channel.close / basic.cancel (consumer recovery)
        self.on_close: Optional[Callable[["Channel", BaseException], None]] = None
        self.on_cancel: Optional[Callable[["Channel", str], None]] = None

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
            self.conn.channels.pop(self.id, None)
            try:
                self.conn.send(C.method_frame(self.id, C.CHANNEL_CLOSE_OK))
            except ConnectionError:
                pass
            err = C.AMQPError(f"channel closed by broker: {args[0]} {args[1]}", args[0])
            self._fail(err)
            if self.on_close is not None:
                self.on_close(self, err)
            return
        if m == C.BASIC_CANCEL:  # broker-side cancel (queue deleted, HA failover)
            if self.consumers.pop(args[0], None) is not None and self.on_cancel is not None:
                self.on_cancel(self, args[0])
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
                 rpc_timeout: float = 30.0, connect_timeout: float = 10.0,
                 ssl_context: Optional[ssl.SSLContext] = None):
        self.host, self.port, self.user, self.password, self.vhost = parse_url(url)
        self.ssl_context = ssl_context
        if self.ssl_context is None and is_tls_url(url):
            self.ssl_context = client_ssl_context()
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
        tls = {} if self.ssl_context is None else {"ssl": self.ssl_context,
                                                   "server_hostname": self.host}
        self.reader, self.writer = await asyncio.wait_for(
            asyncio.open_connection(self.host, self.port, **tls), self.connect_timeout)
        try:
            return await self._handshake()
        except BaseException as e:
            self.writer.close()          # no half-open socket left behind
            if isinstance(e, asyncio.IncompleteReadError):
                # the broker hung up mid-handshake (starting up, or a TLS peer that refused
                # our certificate after the handshake): retryable like a refused connect
                raise ConnectionError("broker closed the connection during the handshake") \
                    from e
            raise

    async def _handshake(self) -> "Connection":
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
        # lowest free id: a connection that outlives many channel recoveries stays far
        # below channel_max (2047)
        cid = next(i for i in itertools.count(1) if i not in self.channels)
        ch = Channel(self, cid)
        self.channels[cid] = ch
        await ch.rpc(C.CHANNEL_OPEN, [""], (C.CHANNEL_OPEN_OK,))
        return ch

    def abort(self) -> None:
        """Drop the socket: the read loop fails every channel and sets ``closed``."""
        if self.writer is not None:
            self.writer.transport.abort()

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
                 publish_retry_s: float = 120.0, ssl_context: Optional[ssl.SSLContext] = None,
                 recover_delay: Optional[float] = None):
        self.url = url
        self.ssl_context = ssl_context
        self.publish_retry_s = publish_retry_s
        self.connect_retry_s = connect_retry_s
        self.heartbeat = heartbeat
        self.reconnect_delay = reconnect_delay
        self.max_reconnect_delay = max_reconnect_delay
        # first wait before reopening a broker-closed channel / re-consuming a cancelled
        # consumer (doubles on failure, capped at max_reconnect_delay)
        self.recover_delay = reconnect_delay if recover_delay is None else recover_delay
        self.metrics = metrics
        self.conn: Optional[Connection] = None
        self._cons_ch: Optional[Channel] = None
        self._pub_ch: Optional[Channel] = None
        self._declared: Dict[str, Dict[str, Any]] = {}     # queue -> x-arguments
        self._consumers: Dict[str, Tuple[str, Handler, int]] = {}
        self._ctags: Dict[str, str] = {}    # our tag -> broker tag (current consumer channel)
        self._ids = itertools.count(1)
        self._gen = 0
        self._lock = asyncio.Lock()
        self._closing = False
        self._watch: Optional[asyncio.Task] = None
        self._tasks: set = set()
        self._recovering = False
        self.connected = False
        self.reconnects = 0
        self.channel_recoveries = 0
        self.resubscribes = 0

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

    def _spawn(self, coro) -> None:
        t = asyncio.get_running_loop().create_task(coro)
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)

    async def _open(self) -> None:
        self.connected = False
        self.conn = await Connection(self.url, self.heartbeat,
                                     ssl_context=self.ssl_context).connect()
        self._gen += 1
        self._ctags.clear()
        await self._setup_publisher()
        await self._setup_consumer()
        self.connected = True

    async def _setup_publisher(self) -> None:
        ch = await self.conn.channel()
        ch.on_close = self._on_channel_close
        await ch.confirm_select()
        self._pub_ch = ch

    async def _setup_consumer(self) -> None:
        """Open the consumer channel and re-run the topology: every declared queue, then
        every registered consumer (amqp-connection-manager's ``setup`` callback)."""
        self._ctags.clear()
        ch = await self.conn.channel()
        ch.on_close = self._on_channel_close
        ch.on_cancel = self._on_consumer_cancel
        self._cons_ch = ch
        for q, args in list(self._declared.items()):
            await ch.queue_declare(q, arguments=args)
        for tag, (q, handler, prefetch) in list(self._consumers.items()):
            await self._subscribe(tag, q, handler, prefetch)

    # ------------------------------------------------------------ channel-level recovery
    def _on_channel_close(self, ch: Channel, err: BaseException) -> None:
        if self._closing or ch.conn is not self.conn or ch.conn.closed.is_set():
            return                                  # connection loss: the watchdog's job
        if ch is self._cons_ch:
            self._ctags.clear()                     # the broker cancelled them with the channel
        if not self._recovering:
            self._recovering = True
            self._spawn(self._recover_channels())

    async def _recover_channels(self) -> None:
        delay = self.recover_delay
        try:
            while not self._closing:
                await asyncio.sleep(delay)
                conn = self.conn
                if conn is None or conn.closed.is_set():
                    return                          # the watchdog reconnects and re-runs setup
                try:
                    async with self._lock:
                        if conn is not self.conn:
                            return
                        if self._pub_ch is None or self._pub_ch.closed:
                            await self._setup_publisher()
                        if self._cons_ch is None or self._cons_ch.closed:
                            await self._setup_consumer()
                    self.channel_recoveries += 1
                    if self.metrics is not None:
                        self.metrics.messages.labels("*", "channel_recover").inc()
                    return
                except (C.AMQPError, asyncio.TimeoutError) as e:
                    # setup refused on a live connection (e.g. a 406 on re-declare): retry a
                    # few times, then let the watchdog start from a fresh connection
                    if delay >= self.max_reconnect_delay or isinstance(e, asyncio.TimeoutError):
                        conn.abort()
                        return
                    delay = min(self.max_reconnect_delay, delay * 2)
                except (OSError, ConnectionError):
                    return
        finally:
            self._recovering = False

    def _on_consumer_cancel(self, ch: Channel, btag: str) -> None:
        """Broker-side ``basic.cancel``: the queue went away (deleted, failover). Re-declare
        it and consume again, as amqp-connection-manager's setup re-run does."""
        for tag, b in list(self._ctags.items()):
            if b == btag:
                del self._ctags[tag]
                if not self._closing and tag in self._consumers:
                    self._spawn(self._resubscribe(tag, ch))

    async def _resubscribe(self, tag: str, ch: Channel) -> None:
        delay = self.recover_delay
        while not self._closing:
            await asyncio.sleep(delay)
            try:
                async with self._lock:
                    ent = self._consumers.get(tag)
                    if (ent is None or tag in self._ctags or not self.connected
                            or self._cons_ch is not ch or ch.closed):
                        return                  # cancelled, or a channel/connection setup ran
                    await self._subscribe(tag, *ent)
                self.resubscribes += 1
                if self.metrics is not None:
                    self.metrics.messages.labels(ent[0], "resubscribe").inc()
                return
            except (C.AMQPError, asyncio.TimeoutError, OSError, ConnectionError):
                delay = min(self.max_reconnect_delay, delay * 2)

    def consumer_live(self, consumer_tag: Optional[str] = None) -> bool:
        """True while the broker holds a subscription for ``consumer_tag`` (every registered
        consumer when None) on the live consumer channel - what ``/readyz`` reports. A
        connected client whose consumer was cancelled or whose channel was closed by the
        broker receives nothing and must not look ready."""
        if not self.connected or self.conn is None or self.conn.closed.is_set():
            return False
        if self._cons_ch is None or self._cons_ch.closed:
            return False
        tags = [consumer_tag] if consumer_tag is not None else list(self._consumers)
        return all(t in self._ctags and self._ctags[t] in self._cons_ch.consumers for t in tags)

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
                    if self.conn is not None:
                        self.conn.abort()
                    delay = min(self.max_reconnect_delay, delay * 2)

    def _usable(self) -> bool:
        return (self.connected and self.conn is not None and not self.conn.closed.is_set()
                and self._pub_ch is not None and not self._pub_ch.closed)

    async def _ready(self, timeout: Optional[float] = None) -> None:
        loop = asyncio.get_running_loop()
        end = loop.time() + (max(1.0, self.max_reconnect_delay) if timeout is None else timeout)
        while True:
            if self._usable():
                return
            if self._closing or loop.time() >= end:
                break
            await asyncio.sleep(0.05)
        raise ConnectionError("AMQP broker not connected")

    async def close(self) -> None:
        self._closing = True
        if self._watch is not None:
            self._watch.cancel()
        for t in list(self._tasks):
            t.cancel()
        if self.conn is not None:
            await self.conn.close()
        self.connected = False

    async def declare(self, queue: str, arguments: Optional[Dict[str, Any]] = None) -> None:
        self._declared[queue] = dict(arguments or {})
        await self._ready()
        await self._cons_ch.queue_declare(queue, arguments=arguments)

    async def publish(self, queue: str, body: bytes, headers: Optional[Headers] = None,
                      confirm: bool = True) -> None:
        """Publish (with a broker confirm unless ``confirm=False``). A connection lost before
        the confirm arrives is not an error: the message is sent again once the watchdog has
        reconnected, as amqp-connection-manager's ChannelWrapper does - at-least-once, so a
        consumer may see it twice. A publisher channel closed by the broker is reopened and
        the publish retried the same way. Refusals on a live channel (a nack) still raise,
        and so does a broker that stays away for ``publish_retry_s``."""
        props = C.Properties(content_type="application/octet-stream", delivery_mode=2,
                             headers=_to_headers(headers))
        loop = asyncio.get_running_loop()
        deadline = loop.time() + self.publish_retry_s
        while True:
            conn, ch = self.conn, self._pub_ch
            try:
                await self._ready(max(0.05, deadline - loop.time()))
                conn, ch = self.conn, self._pub_ch
                await ch.basic_publish("", queue, body, props, wait_confirm=confirm)
                break
            except Exception:   # reset, EOF mid-frame, timeout, channel failure, not ready...
                lost = (conn is None or conn.closed.is_set() or conn is not self.conn
                        or ch is None or ch.closed)
                if not lost or self._closing or loop.time() > deadline:
                    raise
                if self.metrics is not None:
                    self.metrics.messages.labels(queue, "republish").inc()
                await asyncio.sleep(0.02)   # watchdog / channel recovery in progress
        if self.metrics is not None:
            self.metrics.messages.labels(queue, "publish").inc()

    async def publish_delayed(self, queue: str, body: bytes, headers: Optional[Headers],
                              delay_s: float) -> None:
        """Deliver to ``queue`` after ``delay_s`` without holding anything in this process:
        publish to a per-delay holding queue whose ``x-message-ttl`` dead-letters the
        message back to ``queue`` through the default exchange (RabbitMQ's delayed-retry
        idiom; one queue per distinct delay, so no head-of-line blocking)."""
        ms = max(1, int(delay_s * 1000))
        hold = f"{queue}.delay.{ms}"
        if hold not in self._declared:
            await self.declare(hold, {"x-message-ttl": ms, "x-dead-letter-exchange": "",
                                      "x-dead-letter-routing-key": queue})
        await self.publish(hold, body, headers)

    async def _subscribe(self, tag: str, queue: str, handler: Handler, prefetch: int) -> None:
        gen = self._gen

        async def on_msg(msg: Message) -> None:
            d = _AmqpDelivery(msg, queue, gen, self)
            try:
                await handler(d)
            except Exception:
                if not d.settled:
                    await d.nack(requeue=True)

        ch = self._cons_ch
        await ch.queue_declare(queue, arguments=self._declared.get(queue))
        await ch.basic_qos(prefetch)
        self._ctags[tag] = await ch.basic_consume(queue, on_msg)

    async def consume(self, queue: str, handler: Handler, prefetch: int = 1) -> str:
        await self._ready()
        tag = f"amqp-ctag-{next(self._ids)}"
        self._consumers[tag] = (queue, handler, prefetch)
        self._declared.setdefault(queue, {})
        async with self._lock:
            if tag not in self._ctags:          # a reconnect under the lock may have done it
                await self._subscribe(tag, queue, handler, prefetch)
        return tag

    async def cancel(self, consumer_tag: str) -> None:
        self._consumers.pop(consumer_tag, None)
        btag = self._ctags.pop(consumer_tag, None)
        if btag and self.connected and self._cons_ch is not None and not self._cons_ch.closed:
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
        _, n, _ = await self._cons_ch.queue_declare(queue, arguments=self._declared.get(queue))
        return n
