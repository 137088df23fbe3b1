"""Replay AMQP broker for consumer-throughput benchmarks.

A deliberately minimal AMQP 0-9-1 server that streams *pre-encoded*
``basic.deliver`` + header + body frames to one consumer connection as fast as
the prefetch window allows, so an AMQP benchmark measures the consumer
(beholder) rather than broker-side encoding. It implements just enough of the
protocol for :class:`~beholder_amd.transport.amqp.AmqpSource`: handshake,
channel.open, basic.qos, queue.declare, basic.consume, basic.ack (incl.
``multiple``), basic.cancel, channel/connection close.

Flow control: one delivery-tag sequence per channel interleaving all queues;
at most ``prefetch × consumers`` un-acked deliveries in flight (RabbitMQ's
per-consumer ``basic.qos`` summed over the channel's consumers).

Run as a process: ``python -m beholder_amd.bench.replay_broker --events N --port P``
(prints ``READY <port>`` then serves one consumer connection). ``--rate R``: paced, event i is
sent at ``t0 + i / R`` (not before; later only when the prefetch window is full), for the
production path's latency at BASELINE's rates; the DONE line then has how late the sends were. ``--shared --consumers N``: any
number of connections share the queues (:class:`SharedQueueBroker`, competing consumers).
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import signal
import struct
import sys
import time
from typing import Dict, List, Optional, Tuple

from ..transport.amqp import wire

_ACK = (60, 80)


class ReplayBroker:
    def __init__(self, events: List[Tuple[str, bytes]], port: int = 0, channel: int = 1, rate: float = 0.0):
        self.events = events
        self.rate = rate
        self.late_us: List[float] = []  # paced: per send batch, how late its first event went out
        # content header + body frames pre-encoded at startup (channel 1: the consumer's first channel)
        self.content = [wire.encode_content(channel, 60, body, None, 131072) for _, body in events]
        self.port = port
        self.acked = 0
        self.sent = 0
        self.done = asyncio.Event()
        self.t_first: Optional[float] = None
        self.t_done: Optional[float] = None

    async def start(self) -> "ReplayBroker":
        self._server = await asyncio.start_server(self._serve, "127.0.0.1", self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    async def _serve(self, r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
        await r.readexactly(8)
        w.write(wire.encode_method(0, "connection.start", version_major=0, version_minor=9,
                                   server_properties={"product": "replay"}, mechanisms=b"PLAIN", locales=b"en_US"))
        parser = wire.FrameParser(0)
        prefetch = 0
        consumers: Dict[str, str] = {}  # queue -> consumer tag
        channel = 0
        mhead: Dict[str, bytes] = {}
        mtail: Dict[str, bytes] = {}
        acked_upto = 0
        acked_run = 0
        above: set = set()
        sent = 0
        total = len(self.events)
        pending_window = asyncio.Event()

        async def pump():
            nonlocal sent
            rate = self.rate
            t0 = None
            while sent < total:
                window = prefetch * max(1, len(consumers)) if prefetch else total
                room = window - (sent - acked_upto)
                if room <= 0:
                    pending_window.clear()
                    await pending_window.wait()
                    continue
                if rate:
                    # paced: everything due by now (event i is due at t0 + i / rate); until the next
                    # due time, sleep (the loop's timers are 1 ms coarse) then yield until it comes
                    now = time.perf_counter()
                    if t0 is None:
                        t0 = now
                    due = min(total, int((now - t0) * rate) + 1)
                    if due <= sent:
                        wait = t0 + sent / rate - now
                        await asyncio.sleep(wait - 0.0012 if wait > 0.0015 else 0)
                        continue
                    self.late_us.append((now - (t0 + sent / rate)) * 1e6)
                    n = min(room, due - sent, 512)
                else:
                    n = min(room, total - sent, 512)
                if self.t_first is None:
                    self.t_first = time.perf_counter()
                parts = []
                for i in range(sent, sent + n):
                    q = self.events[i][0]
                    meth = mhead[q] + struct.pack(">Q", i + 1) + mtail[q]
                    parts.append(struct.pack(">BHI", 1, channel, len(meth)) + meth + b"\xce")
                    parts.append(self.content[i])
                w.write(b"".join(parts))
                sent += n
                self.sent = sent
                await w.drain()

        pump_task = None
        try:
            while True:
                data = await r.read(1 << 17)
                if not data:
                    return
                for ftype, ch, payload in parser.feed(data):
                    if ftype != wire.FRAME_METHOD:
                        continue
                    cid, mid = struct.unpack_from(">HH", payload)
                    if (cid, mid) == _ACK:
                        tag, flags = struct.unpack_from(">QB", payload, 4)
                        # every tag <= acked_run is settled, and the tags in `above` (acked one by
                        # one above a gap); a multiple ack may cover tags acked singly before
                        if flags & 1:
                            if tag > acked_run:
                                acked_run = tag
                                above = {t for t in above if t > acked_run}
                        elif tag > acked_run:
                            above.add(tag)
                        while acked_run + 1 in above:
                            acked_run += 1
                            above.discard(acked_run)
                        acked_upto = acked_run + len(above)  # settled deliveries (window = sent - acked_upto)
                        self.acked = acked_upto
                        pending_window.set()
                        if acked_run >= total and not self.done.is_set():
                            self.t_done = time.perf_counter()
                            self.done.set()
                        continue
                    m = wire.decode_method(payload)
                    n = m.name
                    if n == "connection.start_ok":
                        w.write(wire.encode_method(0, "connection.tune", channel_max=2047, frame_max=131072,
                                                   heartbeat=0))
                    elif n == "connection.open":
                        w.write(wire.encode_method(0, "connection.open_ok", known_hosts=""))
                    elif n == "channel.open":
                        channel = ch
                        w.write(wire.encode_method(ch, "channel.open_ok", channel_id=b""))
                    elif n == "basic.qos":
                        prefetch = m.prefetch_count
                        w.write(wire.encode_method(ch, "basic.qos_ok"))
                    elif n == "queue.declare":
                        w.write(wire.encode_method(ch, "queue.declare_ok", queue=m.queue, message_count=0,
                                                   consumer_count=0))
                    elif n == "basic.consume":
                        consumers[m.queue] = m.consumer_tag
                        w.write(wire.encode_method(ch, "basic.consume_ok", consumer_tag=m.consumer_tag))
                        queues = {q for q, _ in self.events}
                        if queues <= set(consumers) and pump_task is None:
                            if channel != 1:
                                self.content = [wire.encode_content(channel, 60, b, None, 131072)
                                                for _, b in self.events]
                            for q, tag in consumers.items():
                                ct = tag.encode()
                                mhead[q] = struct.pack(">HH", 60, 60) + bytes([len(ct)]) + ct
                                qb = q.encode()
                                mtail[q] = b"\x00" + b"\x00" + bytes([len(qb)]) + qb  # redelivered=0, exchange="", rk
                            pump_task = asyncio.ensure_future(pump())
                    elif n == "basic.cancel":
                        w.write(wire.encode_method(ch, "basic.cancel_ok", consumer_tag=m.consumer_tag))
                    elif n == "channel.close":
                        w.write(wire.encode_method(ch, "channel.close_ok"))
                    elif n == "connection.close":
                        w.write(wire.encode_method(0, "connection.close_ok"))
                        await w.drain()
                        return
        except (ConnectionError, asyncio.IncompleteReadError):
            return
        finally:
            if pump_task is not None:
                pump_task.cancel()
            w.close()


class SharedQueueBroker:
    """Competing consumers on one set of queues (the reference's only scaling mode: N replicas,
    each ``prefetch`` 100, on the same RabbitMQ queues; index.js:43,62,127).

    Every connection that consumes all the queues takes deliveries from one shared queue head;
    delivery starts once ``consumers`` connections have subscribed, so every N starts together.
    Each connection gets the next events while its window (prefetch x its consumers) has room,
    which is how RabbitMQ spreads a saturated queue over consumers. Delivery tags are per
    channel; acks (single, or ``multiple`` up to a tag) are mapped back to the events they
    settle, and every event's acks are counted: ``acked`` (events acked at least once),
    ``dup_acks`` (acks of an event already acked), ``unknown_acks`` (tags never delivered or
    already settled on that channel) and, at the end, ``lost`` (events never acked). A
    connection that closes with deliveries unacked has them requeued (``redelivered``), as
    RabbitMQ does. ``cpu_s``: this process's CPU from the first delivery to the last ack.
    """

    def __init__(self, events: List[Tuple[str, bytes]], port: int = 0, consumers: int = 1, progress_every: int = 0):
        self.progress_every = progress_every  # print "PROGRESS acked=N" each time N more events are acked
        self._next_progress = progress_every or 0
        self.events = events
        self.bodies = [body for _, body in events]
        self._content: Dict[int, List[bytes]] = {}  # channel -> pre-encoded header + body frames
        self.port = port
        self.expected = max(1, consumers)
        self.total = len(events)
        self.cursor = 0
        self.requeue: collections.deque = collections.deque()
        self.ack_counts = bytearray(self.total)
        self.acked = 0
        self.dup_acks = 0
        self.unknown_acks = 0
        self.redelivered = 0
        self.sent = 0
        self.per_conn: List[int] = []
        self.subscribed = 0
        self.go = asyncio.Event()
        self.more = asyncio.Event()  # requeued events for a waiting pump
        self.done = asyncio.Event()
        self.t_first: Optional[float] = None
        self.t_done: Optional[float] = None
        self.cpu_first = 0.0
        self.cpu_s = 0.0

    def content(self, channel: int) -> List[bytes]:
        c = self._content.get(channel)
        if c is None:
            c = self._content[channel] = [wire.encode_content(channel, 60, b, None, 131072) for b in self.bodies]
        return c

    async def start(self) -> "SharedQueueBroker":
        self.content(1)  # the consumers' first channel: encoded before READY
        self._server = await asyncio.start_server(self._serve, "127.0.0.1", self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    def _settle(self, idx: int) -> None:
        n = self.ack_counts[idx]
        if n:
            self.dup_acks += 1
        else:
            self._add_acked(1)
        if n < 255:
            self.ack_counts[idx] = n + 1

    def _add_acked(self, k: int) -> None:
        self.acked += k
        if self.progress_every and self.acked >= self._next_progress:
            self._next_progress = (self.acked // self.progress_every + 1) * self.progress_every
            print(f"PROGRESS acked={self.acked} connections={len(self.per_conn)}", flush=True)
        if self.acked == self.total:
            self.t_done = time.perf_counter()
            self.cpu_s = _cpu_now() - self.cpu_first
            self.done.set()

    def _take(self, n: int) -> List[Tuple[int, bool]]:
        """Up to n events off the shared head: requeued ones first (redelivered)."""
        out: List[Tuple[int, bool]] = []
        while self.requeue and len(out) < n:
            out.append((self.requeue.popleft(), True))
        k = min(n - len(out), self.total - self.cursor)
        if k > 0:
            out.extend((i, False) for i in range(self.cursor, self.cursor + k))
            self.cursor += k
        return out

    async def _serve(self, r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
        await r.readexactly(8)
        w.write(wire.encode_method(0, "connection.start", version_major=0, version_minor=9,
                                   server_properties={"product": "replay-shared"}, mechanisms=b"PLAIN",
                                   locales=b"en_US"))
        parser = wire.FrameParser(0)
        conn = len(self.per_conn)
        self.per_conn.append(0)
        prefetch = 0
        consumers: Dict[str, str] = {}
        channel = 0
        mhead: Dict[str, bytes] = {}
        tags: List[int] = []      # tag - 1 -> event index
        settled = bytearray()     # tag - 1 -> settled on this channel
        state = {"low": 0, "open": 0}  # lowest unsettled tag - 1; deliveries not yet settled
        room_ev = asyncio.Event()

        def settle_tag(t: int) -> None:  # t: tag - 1
            if t < 0 or t >= len(tags) or settled[t]:
                self.unknown_acks += 1
                return
            settled[t] = 1
            state["open"] -= 1
            self._settle(tags[t])

        async def pump():
            await self.go.wait()
            content = self.content(channel)
            events = self.events
            # per queue: the frame header + basic.deliver up to the delivery tag, and the rest of
            # it (redelivered flag, exchange "", routing key, frame end) for both flag values:
            # a delivery is then four appends (the tag packed in place)
            pre: Dict[str, bytes] = {}
            post: Dict[Tuple[str, bool], bytes] = {}
            for q in mhead:
                rk = q.encode()
                size = len(mhead[q]) + 8 + 1 + 1 + 1 + len(rk)
                pre[q] = struct.pack(">BHI", 1, channel, size) + mhead[q]
                for rd in (False, True):
                    post[(q, rd)] = (b"\x01" if rd else b"\x00") + b"\x00" + bytes([len(rk)]) + rk + b"\xce"
            pack_tag = struct.Struct(">Q").pack
            while not self.done.is_set():
                window = prefetch * max(1, len(consumers)) if prefetch else 512
                room = window - state["open"]
                if room <= 0:
                    room_ev.clear()
                    await room_ev.wait()
                    continue
                batch = self._take(min(room, 512))
                if not batch:  # the head is empty: wait for requeued events or the end
                    self.more.clear()
                    waiter = asyncio.ensure_future(self.more.wait())
                    await asyncio.wait([waiter, asyncio.ensure_future(self.done.wait())],
                                       return_when=asyncio.FIRST_COMPLETED)
                    waiter.cancel()
                    continue
                if self.t_first is None:
                    self.t_first = time.perf_counter()
                    self.cpu_first = _cpu_now()
                buf = bytearray()
                tag = len(tags)
                nred = 0
                for idx, redelivered in batch:
                    q = events[idx][0]
                    tag += 1
                    tags.append(idx)
                    buf += pre[q]
                    buf += pack_tag(tag)
                    buf += post[(q, redelivered)]
                    buf += content[idx]
                    nred += redelivered
                settled.extend(bytes(len(batch)))
                state["open"] += len(batch)
                self.per_conn[conn] += len(batch)
                self.sent += len(batch)
                self.redelivered += nred
                w.write(buf)
                await w.drain()

        pump_task = None
        try:
            while True:
                data = await r.read(1 << 17)
                if not data:
                    return
                for ftype, ch, payload in parser.feed(data):
                    if ftype != wire.FRAME_METHOD:
                        continue
                    cid, mid = struct.unpack_from(">HH", payload)
                    if (cid, mid) == _ACK:
                        tag, flags = struct.unpack_from(">QB", payload, 4)
                        if flags & 1:  # multiple: every unsettled tag up to `tag`
                            if tag > len(tags):
                                self.unknown_acks += 1
                                tag = len(tags)
                            low = state["low"]
                            counts = self.ack_counts
                            n_new = 0
                            for t in range(low, tag):  # settle_tag, inlined: one loop per ack frame
                                if settled[t]:
                                    continue
                                settled[t] = 1
                                idx = tags[t]
                                c = counts[idx]
                                if c:
                                    self.dup_acks += 1
                                else:
                                    n_new += 1
                                if c < 255:
                                    counts[idx] = c + 1
                                state["open"] -= 1
                            if n_new:
                                self._add_acked(n_new)
                        else:
                            settle_tag(tag - 1)
                        low = state["low"]
                        while low < len(settled) and settled[low]:
                            low += 1
                        state["low"] = low
                        room_ev.set()
                        continue
                    m = wire.decode_method(payload)
                    n = m.name
                    if n == "connection.start_ok":
                        w.write(wire.encode_method(0, "connection.tune", channel_max=2047, frame_max=131072,
                                                   heartbeat=0))
                    elif n == "connection.open":
                        w.write(wire.encode_method(0, "connection.open_ok", known_hosts=""))
                    elif n == "channel.open":
                        channel = ch
                        w.write(wire.encode_method(ch, "channel.open_ok", channel_id=b""))
                    elif n == "basic.qos":
                        prefetch = m.prefetch_count
                        w.write(wire.encode_method(ch, "basic.qos_ok"))
                    elif n == "queue.declare":
                        w.write(wire.encode_method(ch, "queue.declare_ok", queue=m.queue, message_count=0,
                                                   consumer_count=0))
                    elif n == "basic.consume":
                        consumers[m.queue] = m.consumer_tag
                        w.write(wire.encode_method(ch, "basic.consume_ok", consumer_tag=m.consumer_tag))
                        if {q for q, _ in self.events} <= set(consumers) and pump_task is None:
                            for q, tag in consumers.items():
                                ct = tag.encode()
                                mhead[q] = struct.pack(">HH", 60, 60) + bytes([len(ct)]) + ct
                            pump_task = asyncio.ensure_future(pump())
                            self.subscribed += 1
                            if self.subscribed >= self.expected:
                                self.go.set()
                    elif n == "basic.cancel":
                        w.write(wire.encode_method(ch, "basic.cancel_ok", consumer_tag=m.consumer_tag))
                    elif n == "channel.close":
                        w.write(wire.encode_method(ch, "channel.close_ok"))
                    elif n == "connection.close":
                        w.write(wire.encode_method(0, "connection.close_ok"))
                        await w.drain()
                        return
        except (ConnectionError, asyncio.IncompleteReadError):
            return
        finally:
            if pump_task is not None:
                pump_task.cancel()
            # unacked deliveries go back to the queue head, redelivered (RabbitMQ's requeue on close)
            back = [tags[t] for t in range(state["low"], len(tags)) if not settled[t] and not self.ack_counts[tags[t]]]
            if back:
                self.requeue.extend(back)
                self.more.set()
            w.close()

    def done_line(self) -> str:
        lost = sum(1 for c in self.ack_counts if c == 0)
        span = (self.t_done - self.t_first) if self.t_done and self.t_first else 0.0
        return (f"DONE sent={self.sent} acked={self.acked} published={self.total} dup_acks={self.dup_acks} "
                f"unknown_acks={self.unknown_acks} lost={lost} redelivered={self.redelivered} "
                f"connections={len(self.per_conn)} per_conn={','.join(map(str, self.per_conn))} "
                f"broker_s={span:.6f} cpu_s={self.cpu_s:.6f}")


def _cpu_now() -> float:
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    return ru.ru_utime + ru.ru_stime


def _serve_native(events: List[Tuple[str, bytes]], a) -> None:
    """``--shared`` on the native SharedBroker (ops/csrc_bench/shared_broker.cpp): the same protocol
    subset, queue semantics and accounting as :class:`SharedQueueBroker`, on an epoll loop of its
    own, so the shared-queue curve is not capped by this process. Prints the same READY /
    PROGRESS / DONE / FINAL lines."""
    import array
    import threading

    from ..ops.bench_native import SharedBroker
    names = sorted({q for q, _ in events})
    qi = {q: i for i, q in enumerate(names)}
    pieces = [wire.encode_content(1, 60, body, None, 131072) for _, body in events]
    offs = array.array("Q", [0])
    for p in pieces:
        offs.append(offs[-1] + len(p))
    b = SharedBroker(b"".join(pieces), offs.tobytes(), bytes(qi[q] for q, _ in events), tuple(names), a.consumers)
    del pieces
    port = b.listen()
    if a.hold:  # SIGTERM reaches this thread only (sigwait below), never the loop's
        signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGTERM})
    print(f"READY {port}", flush=True)
    t = threading.Thread(target=b.run, args=(-1.0 if a.hold else 0.2,), name="shared-broker", daemon=True)
    t.start()
    every = a.progress_every
    nxt = every
    while t.is_alive():
        t.join(0.005)
        st = b.stats()
        if every and st["acked"] >= nxt:
            nxt = (st["acked"] // every + 1) * every
            print(f"PROGRESS acked={st['acked']} connections={st['connections']}", flush=True)
        if a.hold and st["done"]:
            time.sleep(0.2)  # late duplicate acks, if any, are counted
            break

    def line() -> str:
        st = b.stats()
        return (f"sent={st['sent']} acked={st['acked']} published={st['published']} dup_acks={st['dup_acks']} "
                f"unknown_acks={st['unknown_acks']} lost={st['lost']} redelivered={st['redelivered']} "
                f"connections={st['connections']} per_conn={','.join(map(str, st['per_conn']))} "
                f"broker_s={st['broker_s']:.6f} cpu_s={st['cpu_s']:.6f}")
    done = line()
    print("DONE " + done, flush=True)
    print("FINAL " + done, flush=True)
    if a.hold:  # still serving (a worker restarted after the last ack gets its session) until SIGTERM
        signal.sigwait({signal.SIGTERM})
        b.stop()
        t.join(5)


async def _main(a) -> None:
    from ..topics import TOPIC_NAMES_BY_ID
    from .generator import Workload
    w = Workload(n_media=a.media, seed=a.seed)
    events = [(TOPIC_NAMES_BY_ID[t], p) for t, p in w.events(a.events)]
    if a.shared and not a.python:
        del w
        _serve_native(events, a)
        return
    if a.shared:
        sb = await SharedQueueBroker(events, a.port, consumers=a.consumers, progress_every=a.progress_every).start()
        del w
        print(f"READY {sb.port}", flush=True)
        await sb.done.wait()
        print(sb.done_line(), flush=True)
        await asyncio.sleep(0.2)  # the consumers' last acks of duplicates, if any, are counted
        print(sb.done_line().replace("DONE ", "FINAL ", 1), flush=True)
        if a.hold:  # still serving (a worker restarted after the last ack gets its session) until SIGTERM
            stop = asyncio.get_running_loop().create_future()
            asyncio.get_running_loop().add_signal_handler(signal.SIGTERM, lambda: stop.done() or stop.set_result(None))
            await stop
        return
    b = await ReplayBroker(events, a.port, rate=a.rate).start()
    del w
    from .stallmon import fake_monitor
    mon = fake_monitor()
    print(f"READY {b.port}", flush=True)
    await b.done.wait()
    mon.stop()
    late = ""
    if b.late_us:
        lu = sorted(b.late_us)
        late = " " + " ".join(f"late_{k}_us={int(lu[min(len(lu) - 1, int(q * len(lu)))])}"
                              for k, q in (("p50", 0.5), ("p99", 0.99), ("max", 1.0)))
    print(f"DONE sent={b.sent} acked={b.acked} broker_s={b.t_done - b.t_first:.6f}{late}", flush=True)
    print(mon.dump_line("broker"), flush=True)
    await asyncio.sleep(0.5)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=200000)
    ap.add_argument("--media", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--rate", type=float, default=0.0,
                    help="paced: events per second (0 = as fast as the prefetch window allows)")
    ap.add_argument("--shared", action="store_true",
                    help="competing consumers: any number of connections share the queues (SharedQueueBroker)")
    ap.add_argument("--consumers", type=int, default=1,
                    help="--shared: start delivering once this many connections have subscribed")
    ap.add_argument("--progress-every", type=int, default=0,
                    help="--shared: print a PROGRESS line each time this many more events are acked")
    ap.add_argument("--hold", action="store_true",
                    help="--shared: keep serving after FINAL until SIGTERM (a consumer restarted after the "
                         "last ack still gets its session)")
    ap.add_argument("--python", action="store_true",
                    help="--shared: the asyncio SharedQueueBroker instead of the native SharedBroker")
    asyncio.run(_main(ap.parse_args(argv)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
