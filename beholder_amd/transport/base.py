"""Ingest transport interface (SURVEY.md §5 "distributed communication backend").

The reference's only transport is AMQP 0-9-1 via ``triton-core/amqp``:
``new AMQP(dyn('rabbitmq'), 100, 2, prom)``, ``connect()``, and
``listen(topic, fn)`` where ``fn`` receives ``rmsg`` with
``rmsg.message.content`` and ``rmsg.ack()`` (index.js:43-44,62,127).

Here a :class:`Source` yields *batches* of native
:class:`~beholder_amd.ops.Delivery` objects; the service routes each by
``topic_id`` to the registered handler. Implementations:

* :class:`~beholder_amd.transport.ingest.FdSource` — framed stdin / file /
  pipe, read by the native reader thread (BASELINE configs);
* :class:`~beholder_amd.transport.memory.MemoryBroker` — in-process broker
  with AMQP semantics (prefetch window, ack/nack/requeue, redelivery);
* :class:`~beholder_amd.transport.amqp.AmqpSource` — RabbitMQ over a
  hand-written asyncio AMQP 0-9-1 client.
"""
from __future__ import annotations

import abc
from typing import AsyncIterator, Dict, List, Optional, Sequence


class Source(abc.ABC):
    """A stream of deliveries for a set of topics."""

    #: human-readable transport kind
    kind = "abstract"

    @abc.abstractmethod
    async def start(self, topics: Sequence[str]) -> None:
        """Connect and subscribe (``amqp.connect()`` + ``listen`` registration)."""

    @abc.abstractmethod
    def batches(self) -> AsyncIterator[List]:
        """Async iterator of delivery batches; ends when the source is exhausted/closed."""

    @abc.abstractmethod
    async def close(self) -> None:
        """Stop delivering; un-acked deliveries follow the transport's redelivery rules."""

    async def stop_consuming(self) -> None:
        """Graceful-shutdown step 1: deliver nothing new, but keep settlement working so
        in-flight handlers can still ack; :meth:`batches` ends once buffered deliveries are
        handed out. Default: same as :meth:`close`."""
        await self.close()

    @property
    def settler(self):
        """The native Settler shared by this source's deliveries (ack accounting/latency)."""
        return None

    def stats(self) -> Dict:
        return {}

    def describe(self) -> str:
        """What the source consumes from, for the startup log line (service.py)."""
        return self.kind

    def ready(self) -> bool:
        return True

    @property
    def prefetch(self) -> Optional[int]:
        """Transport-enforced in-flight limit, if any (AMQP basic.qos)."""
        return None
