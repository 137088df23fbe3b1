"""In-process broker with AMQP 0-9-1 consumer semantics.

Used by tests, local development and the handler-level fault-injection suite.
It models what the reference relies on from RabbitMQ (index.js:43,62,127):

* one queue per topic; competing consumers share a queue (round-robin);
* ``basic.qos(prefetch)`` per consumer: at most ``prefetch`` un-acked
  deliveries outstanding per queue subscription (index.js:43 → 100);
* ``ack`` removes, ``nack(requeue=True)`` puts the message back at the head of
  the queue with ``redelivered=True``, ``nack(requeue=False)``/``reject``
  drops it (counted as dead-lettered);
* closing a consumer requeues everything it had un-acked (channel close);
* a delivery that is never settled keeps its prefetch slot (quirk Q1).
"""
from __future__ import annotations

import asyncio
import collections
import itertools
from typing import Deque, Dict, List, Optional, Sequence, Tuple

from ..ops import Delivery, Settler
from ..topics import TOPIC_IDS, topic_id
from .base import Source


class _Queue:
    __slots__ = ("name", "tid", "messages", "consumers", "rr", "published", "dead_lettered")

    def __init__(self, name: str):
        self.name = name
        self.tid = TOPIC_IDS.get(name, 0)
        self.messages: Deque[Tuple[bytes, bool]] = collections.deque()
        self.consumers: List["MemoryConsumer"] = []
        self.rr = 0
        self.published = 0
        self.dead_lettered = 0


class MemoryBroker:
    def __init__(self):
        self._queues: Dict[str, _Queue] = {}
        self._finished = False

    def queue(self, name: str) -> _Queue:
        q = self._queues.get(name)
        if q is None:
            q = self._queues[name] = _Queue(name)
        return q

    def publish(self, topic: str, body: bytes) -> None:
        if not isinstance(body, (bytes, bytearray)):
            raise TypeError("body must be bytes")
        q = self.queue(topic)
        q.messages.append((bytes(body), False))
        q.published += 1
        self._kick(q)

    def publish_many(self, topic: str, bodies) -> None:
        q = self.queue(topic)
        for b in bodies:
            q.messages.append((bytes(b), False))
            q.published += 1
        self._kick(q)

    def finish(self) -> None:
        """No more publishes: consumers end once their queues are empty."""
        self._finished = True
        for q in self._queues.values():
            for c in q.consumers:
                c._wake()

    @property
    def finished(self) -> bool:
        return self._finished

    def depth(self, topic: str) -> int:
        return len(self.queue(topic).messages)

    def stats(self) -> dict:
        return {name: {"depth": len(q.messages), "published": q.published, "dead_lettered": q.dead_lettered,
                       "consumers": len(q.consumers),
                       "unacked": sum(len(c._unacked_by_q.get(name, ())) for c in q.consumers)}
                for name, q in self._queues.items()}

    def consumer(self, prefetch: int = 100, batch: int = 512) -> "MemoryConsumer":
        return MemoryConsumer(self, prefetch, batch)

    def _kick(self, q: _Queue) -> None:
        for c in q.consumers:
            c._wake()

    def _requeue_front(self, q: _Queue, body: bytes) -> None:
        q.messages.appendleft((body, True))
        self._kick(q)


class MemoryConsumer(Source):
    kind = "memory"

    def __init__(self, broker: MemoryBroker, prefetch: int = 100, batch: int = 512):
        self.broker = broker
        self._prefetch = int(prefetch)
        self.batch = batch
        self._queues: List[_Queue] = []
        self._unacked: Dict[int, Tuple[_Queue, bytes]] = {}
        self._unacked_by_q: Dict[str, set] = collections.defaultdict(set)
        self._tags = itertools.count(1)
        self._event: Optional[asyncio.Event] = None
        self._closed = False
        self._stopping = False
        self._settler = Settler(on_settle=self._on_settle)
        self.delivered = 0

    @property
    def prefetch(self) -> int:
        return self._prefetch

    @property
    def settler(self) -> Settler:
        return self._settler

    async def start(self, topics: Sequence[str]) -> None:
        self._event = asyncio.Event()
        for t in topics:
            topic_id(t)  # validate
            q = self.broker.queue(t)
            q.consumers.append(self)
            self._queues.append(q)
        self._wake()

    def _wake(self) -> None:
        if self._event is not None:
            self._event.set()

    def _window(self, q: _Queue) -> int:
        return self._prefetch - len(self._unacked_by_q[q.name])

    def _take(self) -> List:
        out = []
        progressed = True
        while progressed and len(out) < self.batch:
            progressed = False
            for q in self._queues:
                if not q.messages or self._window(q) <= 0:
                    continue
                # competing consumers: only take our round-robin share when others are waiting
                body, redelivered = q.messages.popleft()
                tag = next(self._tags)
                self._unacked[tag] = (q, body)
                self._unacked_by_q[q.name].add(tag)
                out.append(Delivery(body, q.tid, tag, self._settler, None, redelivered))
                self.delivered += 1
                progressed = True
                if len(out) >= self.batch:
                    break
        return out

    async def batches(self):
        while not self._closed and not self._stopping:
            got = self._take()
            if got:
                yield got
                # let other consumers/tasks run between batches
                await asyncio.sleep(0)
                continue
            if self.broker.finished and all(not q.messages for q in self._queues):
                return
            self._event.clear()
            await self._event.wait()

    def _on_settle(self, d, kind: str, requeue: bool) -> None:
        tag = d.tag
        ent = self._unacked.pop(tag, None)
        if ent is None:
            raise RuntimeError(f"PRECONDITION_FAILED - unknown delivery tag {tag}")
        q, body = ent
        self._unacked_by_q[q.name].discard(tag)
        if kind != "ack":
            if requeue:
                self.broker._requeue_front(q, body)
            else:
                q.dead_lettered += 1
        self._wake()

    async def stop_consuming(self) -> None:
        """Take nothing new; un-acked deliveries can still be settled until :meth:`close`."""
        self._stopping = True
        self._wake()

    @property
    def unacked(self) -> int:
        return len(self._unacked)

    async def close(self) -> None:
        """Channel close: everything un-acked goes back to its queue (redelivered)."""
        if self._closed:
            return
        self._closed = True
        for tag, (q, body) in sorted(self._unacked.items(), reverse=True):
            q.messages.appendleft((body, True))
        self._unacked.clear()
        self._unacked_by_q.clear()
        for q in self._queues:
            if self in q.consumers:
                q.consumers.remove(self)
            self.broker._kick(q)
        self._wake()

    def stats(self) -> dict:
        s = self._settler.stats()
        s["unacked_outstanding"] = len(self._unacked)
        s["delivered"] = self.delivered
        return s
