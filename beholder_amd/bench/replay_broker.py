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
(prints ``READY <port>`` then serves one consumer connection).
"""
from __future__ import annotations

import argparse
import asyncio
import struct
import sys
import time
from typing import Dict, List, Optional, Tuple

from ..transport.amqp import wire

_ACK = (60, 80)


class ReplayBroker:
    def __init__(self, events: List[Tuple[str, bytes]], port: int = 0, channel: int = 1):
        self.events = events
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
        sent = 0
        total = len(self.events)
        pending_window = asyncio.Event()

        async def pump():
            nonlocal sent
            while sent < total:
                window = prefetch * max(1, len(consumers)) if prefetch else total
                room = window - (sent - acked_upto)
                if room <= 0:
                    pending_window.clear()
                    await pending_window.wait()
                    continue
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
                        # `acked_upto` counts settled deliveries (window = sent - acked_upto)
                        acked_upto = max(acked_upto, tag) if flags & 1 else acked_upto + 1
                        self.acked = acked_upto
                        pending_window.set()
                        if acked_upto >= total and not self.done.is_set():
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


async def _main(a) -> None:
    from ..topics import TOPIC_NAMES_BY_ID
    from .generator import Workload
    w = Workload(n_media=a.media, seed=a.seed)
    events = [(TOPIC_NAMES_BY_ID[t], p) for t, p in w.events(a.events)]
    b = await ReplayBroker(events, a.port).start()
    del w
    from .stallmon import fake_monitor
    mon = fake_monitor()
    print(f"READY {b.port}", flush=True)
    await b.done.wait()
    mon.stop()
    print(f"DONE sent={b.sent} acked={b.acked} broker_s={b.t_done - b.t_first:.6f}", flush=True)
    print(mon.dump_line("broker"), flush=True)
    await asyncio.sleep(0.5)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=200000)
    ap.add_argument("--media", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--port", type=int, default=0)
    asyncio.run(_main(ap.parse_args(argv)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
