"""Message-broker interface (the reference's ``triton-core/amqp``).

Reference surface (lib/main.js:46-47,145,150,164,168,172,200): ``new AMQP(url, prefetch=1,
2, prom)``, ``connect()``, ``listen(queue, fn)``, ``publish(queue, Buffer)``, ``close()`` and a
delivered message exposing ``message.content``, ``ack()`` and ``nack()``.

Backends: ``memory`` (in-process, tests) and ``amqp`` (from-scratch AMQP 0-9-1 client that
talks to RabbitMQ or to the bundled ``downloader_amd.broker.server``).
"""
from __future__ import annotations

import abc
from typing import Any, Awaitable, Callable, Dict, Optional

Headers = Dict[str, Any]


class Delivery(abc.ABC):
    """One delivered message. ``ack``/``nack`` are idempotent (second call is a no-op)."""

    def __init__(self, queue: str, body: bytes, headers: Optional[Headers] = None,
                 redelivered: bool = False, delivery_tag: int = 0):
        self.queue = queue
        self.body = body
        self.headers: Headers = dict(headers or {})
        self.redelivered = redelivered
        self.delivery_tag = delivery_tag
        self.settled = False

    # ``rmsg.message.content`` compatibility (lib/main.js:63)
    @property
    def content(self) -> bytes:
        return self.body

    async def ack(self) -> None:
        if self.settled:
            return
        self.settled = True
        await self._ack()

    async def nack(self, requeue: bool = True) -> None:
        if self.settled:
            return
        self.settled = True
        await self._nack(requeue)

    @abc.abstractmethod
    async def _ack(self) -> None: ...

    @abc.abstractmethod
    async def _nack(self, requeue: bool) -> None: ...


Handler = Callable[[Delivery], Awaitable[None]]


class Broker(abc.ABC):
    connected: bool = False

    @abc.abstractmethod
    async def connect(self) -> None: ...

    @abc.abstractmethod
    async def close(self) -> None: ...

    @abc.abstractmethod
    async def declare(self, queue: str, arguments: Optional[Dict[str, Any]] = None) -> None:
        """Declare ``queue`` (idempotent). ``arguments``: RabbitMQ x-arguments, e.g.
        ``x-message-ttl`` / ``x-dead-letter-exchange`` / ``x-dead-letter-routing-key``."""

    @abc.abstractmethod
    async def publish(self, queue: str, body: bytes, headers: Optional[Headers] = None,
                      confirm: bool = True) -> None:
        """Publish to ``queue``. ``confirm=False``: do not wait for the broker's publisher
        confirm (telemetry: a lost progress event must not cost a round trip per event)."""

    @abc.abstractmethod
    async def consume(self, queue: str, handler: Handler, prefetch: int = 1) -> str:
        """Start delivering ``queue`` to ``handler`` with at most ``prefetch`` unacked
        deliveries outstanding. Returns a consumer tag."""

    @abc.abstractmethod
    async def cancel(self, consumer_tag: str) -> None: ...

    @abc.abstractmethod
    async def get(self, queue: str) -> Optional[Delivery]:
        """Poll one message (basic.get) - used by tests and tools."""

    async def queue_size(self, queue: str) -> int:
        raise NotImplementedError

    async def publish_delayed(self, queue: str, body: bytes, headers: Optional[Headers],
                              delay_s: float) -> None:
        """Publish ``body`` so that it reaches ``queue`` after ``delay_s`` seconds, without
        the caller holding a delivery (or a prefetch slot) while it waits."""
        raise NotImplementedError

    def consumer_live(self, consumer_tag: Optional[str] = None) -> bool:
        """True while ``consumer_tag`` (all consumers when None) is subscribed at the broker
        and can receive deliveries. ``/readyz`` reports it."""
        return self.connected

    # Reference-style aliases -----------------------------------------------------------
    async def listen(self, queue: str, fn: Handler, prefetch: int = 1) -> str:
        return await self.consume(queue, fn, prefetch)


def make_broker(cfg, metrics=None) -> Broker:
    from ..utils.dynamics import dyn
    if cfg.broker.backend == "memory":
        from .memory import MemoryBroker
        return MemoryBroker.shared()
    from .amqp import AmqpBroker, client_ssl_context, is_tls_url
    url = cfg.broker.url or dyn("rabbitmq")
    ctx = None
    if is_tls_url(url):     # amqps://: the same trust settings as every other TLS peer
        ctx = client_ssl_context(cfg.tls.verify, cfg.broker.ca_file or cfg.tls.ca_file,
                                 cfg.broker.cert_file, cfg.broker.key_file)
    return AmqpBroker(url, heartbeat=cfg.broker.heartbeat_s,
                      reconnect_delay=cfg.broker.reconnect_delay_s, metrics=metrics,
                      connect_retry_s=cfg.broker.connect_retry_s, ssl_context=ctx,
                      recover_delay=cfg.broker.recover_delay_s,
                      publish_retry_s=cfg.broker.publish_retry_s)
