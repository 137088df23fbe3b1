"""AMQP consumer source and publisher — ``triton-core/amqp`` parity.

Reference usage (index.js:43-44,62,127)::

    const amqp = new AMQP(dyn('rabbitmq'), 100, 2, prom)
    await amqp.connect()
    amqp.listen('v1.telemetry.status', async rmsg => { ... rmsg.ack() })

:class:`AmqpSource` does the same: one channel with ``basic.qos(prefetch)``
(100), one queue per topic, manual acks. Queue names, exchange and bindings come from
:class:`.topology.Topology` (``service.amqp``); the default is a durable queue per topic,
named after the topic, on the default exchange (publishers use ``routing_key = topic``).

Reliability (amqp-connection-manager parity):

* startup: ``retries + 1`` connection attempts with exponential backoff, then
  the error propagates (fail fast — the Q10 fix);
* after startup: on connection / channel loss, reconnect forever with
  exponential backoff (0.25 s … 30 s), re-declare, re-qos, re-consume;
* deliveries from a dead channel are *stale*: settling them is a no-op
  (the broker already requeued them, ``redelivered`` set on the next delivery).
"""
from __future__ import annotations

import asyncio
import time
from typing import Dict, List, Optional, Sequence

from ...ops import AckBatcher, Delivery, Settler
from ...topics import TOPIC_IDS, topic_id
from ...utils.waits import Signal
from ..base import Source
from .connection import Channel, Connection
from .topology import Topology
from .wire import AmqpError


class AmqpSource(Source):
    kind = "amqp"

    def __init__(self, url: str, prefetch: int = 100, retries: int = 2, *, logger=None,
                 durable: bool = True, heartbeat: Optional[int] = None, backoff_initial: float = 0.25,
                 backoff_max: float = 30.0, connect_timeout: float = 10.0, native: bool = True,
                 coalesce_acks: bool = True, capture_headers: bool = False,
                 topology: Optional[Topology] = None):
        self.url = url
        self.topology = topology if topology is not None else Topology(durable=durable)
        self.capture_headers = capture_headers  # keep message headers on deliveries (trace context)
        self._prefetch = int(prefetch)
        self.retries = int(retries)
        self.log = logger
        self.durable = durable
        self.heartbeat = heartbeat
        self.backoff_initial = backoff_initial
        self.backoff_max = backoff_max
        self.connect_timeout = connect_timeout
        self.native = native  # assemble deliveries in C (ops.AmqpDemux)
        self.coalesce_acks = coalesce_acks
        self._settler = Settler(on_settle=self._on_settle)
        # acks of the current channel's deliveries are coalesced natively (ops/csrc/py_acks.cpp):
        # one basic.ack(multiple) for the settled prefix + singles above a gap, one write per
        # loop iteration; nack/reject and stale settles still go through _on_settle
        self._batcher: Optional[AckBatcher] = AckBatcher(self._schedule_ack_flush) if coalesce_acks else None
        self._settler.ack_batcher = self._batcher
        self._topics: List[str] = []
        self._tag_topic: Dict[str, int] = {}
        self._conn: Optional[Connection] = None
        self._ch: Optional[Channel] = None
        self._pending: List = []
        self._event: Optional[Signal] = None
        self.idle_wakeups = 0  # batches that came after the consumer waited for deliveries
        # set by the consumer while it waits with nothing queued: deliveries are handed to it from
        # the read callback itself (no wake-up of its task, no extra trip through the loop);
        # it returns what it could not take (prefetch window full), which then queues as usual
        self.direct = None
        self.direct_batches = 0
        self._in_task = False  # a batch from batches() is in the consumer's hands
        self._direct_error: Optional[BaseException] = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None  # set at start(): one lookup, not one per flush
        self._closing = False
        self._stopping = False
        self._reconnect_task: Optional[asyncio.Task] = None
        self.reconnects = 0
        self.delivered = 0
        self.stale_settles = 0
        self.last_error: Optional[str] = None
        self.connected_since = 0.0

    # ------------------------------------------------------------ Source ---
    @property
    def prefetch(self) -> int:
        return self._prefetch

    @property
    def settler(self) -> Settler:
        return self._settler

    async def start(self, topics: Sequence[str]) -> None:
        for t in topics:
            topic_id(t)
        self._topics = list(topics)
        self._event = Signal()
        self._loop = asyncio.get_running_loop()
        delay = self.backoff_initial
        for attempt in range(self.retries + 1):
            try:
                await self._connect()
                return
            except (OSError, AmqpError, asyncio.TimeoutError) as e:
                self.last_error = f"{type(e).__name__}: {e}"
                if attempt == self.retries:
                    raise
                self._warn(f"amqp connect failed ({self.last_error}), retrying in {delay:.2f}s")
                await asyncio.sleep(delay)
                delay = min(delay * 2, self.backoff_max)

    async def _connect(self) -> None:
        conn = Connection(self.url, heartbeat=self.heartbeat, connect_timeout=self.connect_timeout,
                          logger=self.log, on_lost=self._on_lost,
                          native_settler=self._settler if self.native else None,
                          on_deliveries=self._on_native_deliveries if self.native else None,
                          capture_headers=self.capture_headers)
        await conn.open()
        try:
            ch = await conn.channel()
            await ch.basic_qos(self._prefetch)
            tags = {}
            topo = self.topology
            await topo.declare(ch, self._topics)
            for t in self._topics:
                tag = await ch.basic_consume(topo.queue(t), self._on_message, native_topic=TOPIC_IDS[t])
                tags[tag] = TOPIC_IDS[t]
        except BaseException:
            await conn.close()
            raise
        ch.on_close = self._on_channel_close
        if self._batcher is not None:
            self._batcher.bind(ch, ch.id)  # fresh channel: delivery tags restart at 1
        self._conn, self._ch, self._tag_topic = conn, ch, tags
        self.connected_since = time.time()

    def _on_message(self, ch: Channel, method, props, body: bytes) -> None:
        tid = self._tag_topic.get(method.consumer_tag, 0)
        d = Delivery(body, tid, method.delivery_tag, self._settler, None, method.redelivered, ch)
        if self.capture_headers:
            d.headers = props.get("headers")
        self._on_native_deliveries([d])

    def _on_native_deliveries(self, ds) -> None:
        self.delivered += len(ds)
        pending = self._pending
        if pending:
            pending.extend(ds)
            return
        direct = self.direct
        # not while the consumer's task works through a queued batch: what arrives meanwhile
        # queues behind it, so handlers start in delivery order
        if direct is not None and not self._in_task and not self._stopping and not self._closing:
            ds = self._hand_over(direct, ds)
            if not ds:
                return
        self._pending = ds
        self._event.set()

    def _hand_over(self, direct, ds):
        """The deliveries to the waiting consumer, inside one NetPoller batch: the queries its
        handlers issue go out together at the end, and so do the acks of handlers that finish
        there. Returns what it did not take. A failure of the consumer's dispatch ends the direct
        hand-over and is raised from :meth:`batches`, as a failure in its own loop would be."""
        self.direct_batches += 1
        poller = getattr(self._loop, "_beholder_netpoller", None)
        if poller is not None:
            poller._enter()
        try:
            return direct(ds)
        except BaseException as e:  # noqa: BLE001 - re-raised in the consumer's task (batches)
            self.direct = None
            self._direct_error = e
            self._event.set()
            return None
        finally:
            if poller is not None:
                poller._exit()

    def _schedule_ack_flush(self) -> None:
        loop = self._loop
        if loop is None:
            loop = self._loop = asyncio.get_running_loop()
        poller = getattr(loop, "_beholder_netpoller", None)
        if poller is not None and poller.defer(self._flush_acks):
            return  # settled inside a NetPoller batch: flushed at its end, with the batch's other acks
        loop.call_soon(self._flush_acks)

    def _flush_acks(self) -> None:
        b = self._batcher
        data = b.flush()
        ch = self._ch
        if data and ch is not None and ch.is_open and b.channel is ch:
            ch.conn._write_now(data)

    def _on_settle(self, d, kind: str, requeue: bool) -> None:
        """Settles the native batcher did not take: nack/reject, stale channels, no batching."""
        ch: Channel = d.extra
        if ch is None or not ch.is_open or ch is not self._ch:
            self.stale_settles += 1  # channel gone: broker already requeued it
            return
        if kind == "ack":
            ch.basic_ack(d.tag)
            return
        if self._batcher is not None:
            self._batcher.settled_elsewhere(d.tag)
        if kind == "nack":
            ch.basic_nack(d.tag, requeue=requeue)
        else:
            ch.basic_reject(d.tag, requeue=requeue)

    async def batches(self):
        while True:
            if self._direct_error is not None:
                e, self._direct_error = self._direct_error, None
                raise e
            if self._pending:
                batch, self._pending = self._pending, []
                self._in_task = True
                try:
                    yield batch
                finally:
                    self._in_task = False
                continue
            if self._closing or self._stopping:
                return
            self._event.clear()
            await self._event.wait()
            self.idle_wakeups += 1  # this batch came after a wait: the consumer yielded to the loop

    async def stop_consuming(self) -> None:
        """``basic.cancel`` every consumer; the channel stays open so acks of in-flight
        handlers still reach the broker (no redelivery of work already done)."""
        if self._stopping or self._closing:
            return
        self._stopping = True
        if self._reconnect_task is not None:
            self._reconnect_task.cancel()
        ch = self._ch
        if ch is not None and ch.is_open:
            for tag in list(self._tag_topic):
                try:
                    await asyncio.wait_for(ch.basic_cancel(tag), 5)
                except (AmqpError, asyncio.TimeoutError, ConnectionError):
                    break
        if self._event is not None:
            self._event.set()

    async def close(self) -> None:
        if self._closing:
            return
        self._closing = True
        if self._reconnect_task is not None:
            self._reconnect_task.cancel()
        ch, conn = self._ch, self._conn
        if self._batcher is not None:
            self._flush_acks()  # acks of the last handlers go out before the channel closes
            self._batcher.unbind()
        self._ch = None
        if ch is not None and ch.is_open:
            if not self._stopping:
                for tag in list(self._tag_topic):
                    try:
                        await asyncio.wait_for(ch.basic_cancel(tag), 5)
                    except (AmqpError, asyncio.TimeoutError, ConnectionError):
                        break
            await ch.close()
        if conn is not None:
            await conn.close()
        if self._event is not None:
            self._event.set()

    def describe(self) -> str:
        from ...sinks.http import redact
        return f"amqp {redact(self.url)} prefetch={self._prefetch} {self.topology.describe(self._topics)}"

    def ready(self) -> bool:
        return self._ch is not None and self._ch.is_open and not self._closing

    def stats(self) -> dict:
        s = self._settler.stats()
        c = self._conn
        s.update({"connected": self.ready(), "reconnects": self.reconnects, "delivered": self.delivered,
                  "stale_settles": self.stale_settles, "last_error": self.last_error,
                  "bytes_in": c.bytes_in if c else 0, "bytes_out": c.bytes_out if c else 0,
                  "reads": c.reads if c else 0, "writes": c.writes if c else 0,
                  "buffered": len(self._pending),
                  "ack_frames": self._batcher.frames if self._batcher is not None else None,
                  "ack_multiples": self._batcher.multiples if self._batcher is not None else None,
                  "ack_stuck_tag": self._batcher.stuck if self._batcher is not None else None})
        return s

    # --------------------------------------------------------- recovery ---
    def _on_channel_close(self, ch: Channel, err) -> None:
        if err is not None and not self._closing:
            self.last_error = str(err)
            self._schedule_reconnect()

    def _on_lost(self, err) -> None:
        if self._closing:
            return
        self.last_error = str(err) if err else "connection lost"
        self._schedule_reconnect()

    def _schedule_reconnect(self) -> None:
        if self._closing or (self._reconnect_task is not None and not self._reconnect_task.done()):
            return
        self._ch = None
        if self._batcher is not None:
            self._batcher.unbind()  # acks of the dead channel's deliveries are stale from now on
        self._reconnect_task = asyncio.get_running_loop().create_task(self._reconnect_loop())

    async def _reconnect_loop(self) -> None:
        old = self._conn
        if old is not None:
            try:
                await old.close()
            except Exception:  # noqa: BLE001
                pass
        delay = self.backoff_initial
        while not self._closing:
            self._warn(f"amqp connection lost ({self.last_error}); reconnecting in {delay:.2f}s")
            await asyncio.sleep(delay)
            try:
                await self._connect()
                self.reconnects += 1
                self._info(f"amqp reconnected (attempt {self.reconnects})")
                return
            except (OSError, AmqpError, asyncio.TimeoutError) as e:
                self.last_error = f"{type(e).__name__}: {e}"
                delay = min(delay * 2, self.backoff_max)

    def _warn(self, msg: str) -> None:
        if self.log is not None:
            self.log.warn(msg)

    def _info(self, msg: str) -> None:
        if self.log is not None:
            self.log.info(msg)


class AmqpPublisher:
    """``amqp.publish(topic, buffer)`` — what the other triton services call. Routes through
    ``topology`` (default: the default exchange, ``routing_key = topic``)."""

    def __init__(self, url: str, confirm: bool = True, durable: bool = True, persistent: bool = True,
                 topology: Optional[Topology] = None):
        self.url = url
        self.topology = topology if topology is not None else Topology(durable=durable)
        self.confirm = confirm
        self.durable = durable
        self.persistent = persistent
        self._conn: Optional[Connection] = None
        self._ch: Optional[Channel] = None
        self._declared: set = set()

    async def connect(self) -> "AmqpPublisher":
        self._conn = await Connection(self.url).open()
        self._ch = await self._conn.channel()
        if self.confirm:
            await self._ch.confirm_select()
        return self

    async def publish(self, topic: str, body: bytes, wait: bool = False):
        if topic not in self._declared:
            await self.topology.declare(self._ch, [topic])  # messages published before a consumer exists are kept
            self._declared.add(topic)
        exchange, key = self.topology.publish_target(topic)
        props = {"delivery_mode": 2} if self.persistent else None
        return await self._ch.basic_publish(body, routing_key=key, exchange=exchange, properties=props,
                                            wait_confirm=wait)

    async def flush(self) -> None:
        if self._ch is not None:
            await self._ch.wait_confirms()

    async def close(self) -> None:
        if self._ch is not None:
            await self.flush()
            await self._ch.close()
        if self._conn is not None:
            await self._conn.close()


async def publish_frames(url: str, data: bytes, topology: Optional[Topology] = None) -> int:
    """Publish every frame of a framed stream to its topic queue (CLI ``publish``)."""
    from ...topics import topic_name
    from ..framing import iter_frames
    pub = await AmqpPublisher(url, topology=topology).connect()
    n = 0
    try:
        for tid, payload in iter_frames(data):
            name = topic_name(tid)
            if name is None:
                raise ValueError(f"frame with unknown topic id {tid}")
            await pub.publish(name, payload)
            n += 1
        await pub.flush()
    finally:
        await pub.close()
    return n
