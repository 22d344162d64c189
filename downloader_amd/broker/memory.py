"""In-process broker with AMQP-like semantics (prefetch window, ack, nack+requeue,
redelivery of unacked messages when a consumer is cancelled). Used by unit tests and the
single-process bench; every consumer must live on the same event loop."""
from __future__ import annotations

import asyncio
import itertools
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional, Tuple

from .base import Broker, Delivery, Handler, Headers


@dataclass
class _Msg:
    body: bytes
    headers: Headers
    redelivered: bool = False


class _MemDelivery(Delivery):
    def __init__(self, broker: "MemoryBroker", consumer: Optional["_Consumer"], queue: str,
                 msg: _Msg, tag: int):
        super().__init__(queue, msg.body, msg.headers, msg.redelivered, tag)
        self._b = broker
        self._c = consumer
        self._msg = msg

    async def _ack(self) -> None:
        self._b._settle(self, requeue=None)

    async def _nack(self, requeue: bool) -> None:
        self._b._settle(self, requeue=requeue)


@dataclass
class _Consumer:
    tag: str
    queue: str
    handler: Handler
    prefetch: int
    unacked: Dict[int, _MemDelivery] = field(default_factory=dict)
    active: bool = True


class MemoryBroker(Broker):
    _shared: Optional["MemoryBroker"] = None

    def __init__(self) -> None:
        self.queues: Dict[str, Deque[_Msg]] = {}
        self.consumers: Dict[str, _Consumer] = {}
        self.published: List[Tuple[str, bytes, Headers]] = []
        self._tags = itertools.count(1)
        self._ctags = itertools.count(1)
        self._rr: Dict[str, int] = {}
        self._tasks: set = set()
        self.connected = False
        self.fail_publish: int = 0  # fault injection: fail the next N publishes
        self.delayed = 0            # publish_delayed messages not yet due
        self._timers: set = set()

    @classmethod
    def shared(cls) -> "MemoryBroker":
        if cls._shared is None:
            cls._shared = cls()
        return cls._shared

    async def connect(self) -> None:
        self.connected = True

    async def close(self) -> None:
        for tag in list(self.consumers):
            await self.cancel(tag)
        for t in list(self._tasks):
            t.cancel()
        for h in list(self._timers):
            h.cancel()
        self._timers.clear()
        self.connected = False

    async def declare(self, queue: str, arguments: Optional[Dict] = None) -> None:
        self.queues.setdefault(queue, deque())

    async def publish_delayed(self, queue: str, body: bytes, headers: Optional[Headers],
                              delay_s: float) -> None:
        """The delay lives in the event loop (what a TTL holding queue does at a broker)."""
        loop = asyncio.get_running_loop()
        self.delayed += 1

        def fire() -> None:
            self.delayed -= 1
            t = loop.create_task(self.publish(queue, body, headers))
            self._tasks.add(t)
            t.add_done_callback(self._tasks.discard)
        self._timers.add(loop.call_later(max(0.0, delay_s), fire))

    def consumer_live(self, consumer_tag: Optional[str] = None) -> bool:
        if not self.connected:
            return False
        return consumer_tag is None or consumer_tag in self.consumers

    async def publish(self, queue: str, body: bytes, headers: Optional[Headers] = None,
                      confirm: bool = True) -> None:
        if self.fail_publish > 0:
            self.fail_publish -= 1
            raise ConnectionError("injected publish failure")
        q = self.queues.setdefault(queue, deque())
        q.append(_Msg(bytes(body), dict(headers or {})))
        self.published.append((queue, bytes(body), dict(headers or {})))
        self._pump(queue)

    async def consume(self, queue: str, handler: Handler, prefetch: int = 1) -> str:
        await self.declare(queue)
        tag = f"mem-ctag-{next(self._ctags)}"
        self.consumers[tag] = _Consumer(tag, queue, handler, max(1, prefetch))
        self._pump(queue)
        return tag

    async def cancel(self, consumer_tag: str) -> None:
        c = self.consumers.pop(consumer_tag, None)
        if c is None:
            return
        c.active = False
        # Unacked deliveries go back to the head of the queue, flagged redelivered.
        q = self.queues.setdefault(c.queue, deque())
        for d in sorted(c.unacked.values(), key=lambda d: -d.delivery_tag):
            if not d.settled:
                d.settled = True
                m = d._msg
                m.redelivered = True
                q.appendleft(m)
        c.unacked.clear()
        self._pump(c.queue)

    async def get(self, queue: str) -> Optional[Delivery]:
        q = self.queues.get(queue)
        if not q:
            return None
        m = q.popleft()
        return _MemDelivery(self, None, queue, m, next(self._tags))

    async def queue_size(self, queue: str) -> int:
        return len(self.queues.get(queue, ()))

    def drain(self, queue: str) -> List[bytes]:
        q = self.queues.get(queue, deque())
        out = [m.body for m in q]
        q.clear()
        return out

    # ------------------------------------------------------------------ internals
    def _settle(self, d: _MemDelivery, requeue: Optional[bool]) -> None:
        c = d._c
        if c is not None:
            c.unacked.pop(d.delivery_tag, None)
        if requeue:
            m = d._msg
            m.redelivered = True
            self.queues.setdefault(d.queue, deque()).appendleft(m)
        self._pump(d.queue)

    def _pump(self, queue: str) -> None:
        q = self.queues.get(queue)
        if not q:
            return
        cons = [c for c in self.consumers.values() if c.queue == queue and c.active]
        if not cons:
            return
        start = self._rr.get(queue, 0)
        progressed = True
        while q and progressed:
            progressed = False
            for i in range(len(cons)):
                c = cons[(start + i) % len(cons)]
                if not q:
                    break
                if len(c.unacked) >= c.prefetch:
                    continue
                m = q.popleft()
                d = _MemDelivery(self, c, queue, m, next(self._tags))
                c.unacked[d.delivery_tag] = d
                t = asyncio.get_event_loop().create_task(self._dispatch(c, d))
                self._tasks.add(t)
                t.add_done_callback(self._tasks.discard)
                progressed = True
            start += 1
        self._rr[queue] = start

    async def _dispatch(self, c: _Consumer, d: _MemDelivery) -> None:
        try:
            await c.handler(d)
        except Exception:
            # A crashing handler is treated like a channel error: requeue.
            if not d.settled:
                await d.nack(requeue=True)
