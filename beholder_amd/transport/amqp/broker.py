"""Minimal AMQP 0-9-1 broker (asyncio) for integration tests and local development.

Implements the RabbitMQ semantics beholder depends on (index.js:43,62,127):
durable queues, the default exchange plus direct/fanout/topic exchanges,
``basic.qos`` per-consumer prefetch, round-robin competing consumers,
``ack``/``nack``/``reject`` (incl. ``multiple``), requeue of un-acked
messages on channel/connection close (``redelivered`` set), publisher
confirms, heartbeats. Test hooks: :meth:`AmqpBroker.publish`,
:meth:`AmqpBroker.drop_connections` (simulated broker crash) and counters.

Not a production broker: no persistence, no clustering, no TLS.
"""
from __future__ import annotations

import asyncio
import collections
import itertools
import time
from typing import Any, Deque, Dict, List, Optional, Set, Tuple

from . import wire
from .wire import AmqpError, Method

Message = Tuple[bytes, Dict[str, Any], str, str]  # body, props, exchange, routing_key


class _Queue:
    def __init__(self, name: str, durable: bool, exclusive_owner=None, auto_delete: bool = False):
        self.name = name
        self.durable = durable
        self.exclusive_owner = exclusive_owner
        self.auto_delete = auto_delete
        self.messages: Deque[Tuple[Message, bool]] = collections.deque()  # (msg, redelivered)
        self.consumers: List["_Consumer"] = []
        self.rr = 0
        self.published = 0
        self.delivered = 0
        self.acked = 0
        self.requeued = 0
        self.dead_lettered = 0


class _Consumer:
    def __init__(self, ch: "_BChannel", tag: str, queue: _Queue, no_ack: bool):
        self.ch = ch
        self.tag = tag
        self.queue = queue
        self.no_ack = no_ack
        self.unacked = 0

    def can_take(self) -> bool:
        pc = self.ch.prefetch
        return self.ch.open and self.ch.flow and (self.no_ack or pc == 0 or self.unacked < pc)


class _Exchange:
    def __init__(self, name: str, type_: str, durable: bool = True):
        self.name = name
        self.type = type_
        self.durable = durable
        self.bindings: List[Tuple[str, str]] = []  # (queue, routing_key)


def _topic_match(pattern: str, key: str) -> bool:
    p, k = pattern.split("."), key.split(".")

    def m(i, j):
        if i == len(p):
            return j == len(k)
        if p[i] == "#":
            return any(m(i + 1, jj) for jj in range(j, len(k) + 1))
        if j == len(k):
            return False
        return (p[i] == "*" or p[i] == k[j]) and m(i + 1, j + 1)

    return m(0, 0)


class _BChannel:
    def __init__(self, conn: "_BConn", cid: int):
        self.conn = conn
        self.id = cid
        self.open = True
        self.flow = True
        self.prefetch = 0
        self.consumers: Dict[str, _Consumer] = {}
        self.unacked: Dict[int, Tuple[_Queue, Message, Optional[_Consumer]]] = {}
        self.tags = itertools.count(1)
        self.confirm = False
        self.pub_seq = 0
        # content assembly for basic.publish
        self.pub_method: Optional[Method] = None
        self.pub_props: Dict[str, Any] = {}
        self.pub_size = -1
        self.pub_parts: List[bytes] = []
        self.pub_got = 0


class _BConn:
    def __init__(self, broker: "AmqpBroker", reader, writer):
        self.broker = broker
        self.reader = reader
        self.writer = writer
        self.parser = wire.FrameParser(0)
        self.channels: Dict[int, _BChannel] = {}
        self.frame_max = broker.frame_max
        self.heartbeat = 0
        self.state = "start"
        self.closed = False
        self.last_rx = time.monotonic()
        self.hb_task: Optional[asyncio.Task] = None
        self.user = None

    def send(self, data: bytes) -> None:
        if not self.closed:
            try:
                self.writer.write(data)
            except (ConnectionError, RuntimeError):
                self.closed = True


class AmqpBroker:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, users: Optional[Dict[str, str]] = None,
                 vhosts: Tuple[str, ...] = ("/",), frame_max: int = 131072, heartbeat: int = 60,
                 ssl_context=None):
        self.host = host
        self.port = port
        self.users = users  # None = accept any credentials
        self.vhosts = vhosts
        self.frame_max = frame_max
        self.heartbeat = heartbeat
        self.queues: Dict[str, _Queue] = {}
        self.exchanges: Dict[str, _Exchange] = {
            "": _Exchange("", "direct"), "amq.direct": _Exchange("amq.direct", "direct"),
            "amq.fanout": _Exchange("amq.fanout", "fanout"), "amq.topic": _Exchange("amq.topic", "topic")}
        self.conns: Set[_BConn] = set()
        self._server: Optional[asyncio.AbstractServer] = None
        self.mute_heartbeats = False
        self.connections_total = 0
        self.ssl_context = ssl_context

    # -------------------------------------------------------------- admin ---
    @property
    def url(self) -> str:
        scheme = "amqps" if self.ssl_context is not None else "amqp"
        return f"{scheme}://guest:guest@{self.host}:{self.port}/"

    async def start(self) -> "AmqpBroker":
        self._server = await asyncio.start_server(self._serve, self.host, self.port, ssl=self.ssl_context)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    async def stop(self) -> None:
        await self.drop_connections()
        if self._server is not None:
            self._server.close()
            await self._server.wait_closed()
            self._server = None

    async def drop_connections(self) -> None:
        """Abruptly close every client connection (simulated broker crash / network cut)."""
        for c in list(self.conns):
            self._teardown(c)
            try:
                c.writer.transport.abort()
            except Exception:  # noqa: BLE001
                pass
        await asyncio.sleep(0)

    def declare_queue(self, name: str, durable: bool = True) -> _Queue:
        q = self.queues.get(name)
        if q is None:
            q = self.queues[name] = _Queue(name, durable)
        return q

    def publish(self, routing_key: str, body: bytes, exchange: str = "", properties=None) -> int:
        """Route a message as if published by a client; returns the number of queues it reached."""
        return self._route(exchange, routing_key, (bytes(body), dict(properties or {}), exchange, routing_key))

    def depth(self, queue: str) -> int:
        q = self.queues.get(queue)
        return len(q.messages) if q else 0

    def unacked(self, queue: str) -> int:
        n = 0
        for c in self.conns:
            for ch in c.channels.values():
                n += sum(1 for (q, _m, _c) in ch.unacked.values() if q.name == queue)
        return n

    def stats(self, queue: str) -> Dict[str, int]:
        q = self.queues[queue]
        return {"depth": len(q.messages), "unacked": self.unacked(queue), "published": q.published,
                "delivered": q.delivered, "acked": q.acked, "requeued": q.requeued,
                "dead_lettered": q.dead_lettered, "consumers": len(q.consumers)}

    # ------------------------------------------------------------ serving ---
    async def _serve(self, reader, writer) -> None:
        c = _BConn(self, reader, writer)
        self.conns.add(c)
        self.connections_total += 1
        try:
            hdr = await asyncio.wait_for(reader.readexactly(8), 10)
            if hdr != wire.PROTOCOL_HEADER:
                writer.write(wire.PROTOCOL_HEADER)
                return
            c.send(wire.encode_method(0, "connection.start", version_major=0, version_minor=9,
                                      server_properties={"product": "beholder-test-broker",
                                                         "capabilities": {"publisher_confirms": True,
                                                                          "basic.nack": True,
                                                                          "consumer_cancel_notify": True}},
                                      mechanisms=b"PLAIN AMQPLAIN", locales=b"en_US"))
            while not c.closed:
                data = await reader.read(1 << 17)
                if not data:
                    break
                c.last_rx = time.monotonic()
                for ftype, ch, payload in c.parser.feed(data):
                    self._frame(c, ftype, ch, payload)
                    if c.closed:
                        break
        except (asyncio.IncompleteReadError, asyncio.TimeoutError, ConnectionError, OSError):
            pass
        except AmqpError as e:
            self._conn_close(c, e.reply_code or wire.INTERNAL_ERROR, str(e))
        finally:
            self._teardown(c)
            try:
                writer.close()
            except Exception:  # noqa: BLE001
                pass

    def _teardown(self, c: _BConn) -> None:
        if c in self.conns:
            self.conns.discard(c)
        c.closed = True
        if c.hb_task is not None:
            c.hb_task.cancel()
        for ch in list(c.channels.values()):
            self._channel_gone(ch)
        c.channels.clear()

    def _conn_close(self, c: _BConn, code: int, text: str, cid: int = 0, mid: int = 0) -> None:
        c.send(wire.encode_method(0, "connection.close", reply_code=code, reply_text=text[:255], class_id=cid,
                                  method_id=mid))
        c.state = "closing"

    def _ch_close(self, ch: _BChannel, code: int, text: str, cid: int = 0, mid: int = 0) -> None:
        ch.conn.send(wire.encode_method(ch.id, "channel.close", reply_code=code, reply_text=text[:255],
                                        class_id=cid, method_id=mid))
        self._channel_gone(ch)

    def _channel_gone(self, ch: _BChannel) -> None:
        if not ch.open:
            return
        ch.open = False
        touched = set()
        for cons in ch.consumers.values():
            if cons in cons.queue.consumers:
                cons.queue.consumers.remove(cons)
        # requeue un-acked in original order, at the head, redelivered
        for tag in sorted(ch.unacked, reverse=True):
            q, msg, _cons = ch.unacked[tag]
            q.messages.appendleft((msg, True))
            q.requeued += 1
            touched.add(q)
        ch.unacked.clear()
        ch.consumers.clear()
        for q in touched:
            self._pump(q)

    async def _heartbeats(self, c: _BConn) -> None:
        hb = c.heartbeat
        try:
            while not c.closed:
                await asyncio.sleep(hb / 2)
                if not self.mute_heartbeats:
                    c.send(wire.encode_heartbeat())
                if time.monotonic() - c.last_rx > 2 * hb:
                    self._conn_close(c, wire.CONNECTION_FORCED, "missed heartbeats from client")
                    self._teardown(c)
                    c.writer.close()
                    return
        except asyncio.CancelledError:
            pass

    # ------------------------------------------------------------- frames ---
    def _frame(self, c: _BConn, ftype: int, cid: int, payload: bytes) -> None:
        if ftype == wire.FRAME_HEARTBEAT:
            return
        if cid == 0:
            self._conn_method(c, wire.decode_method(payload))
            return
        ch = c.channels.get(cid)
        if ftype == wire.FRAME_METHOD:
            m = wire.decode_method(payload)
            if m.name == "channel.open":
                if ch is not None and ch.open:
                    self._conn_close(c, wire.CHANNEL_ERROR, "channel already open", 20, 10)
                    return
                c.channels[cid] = _BChannel(c, cid)
                c.send(wire.encode_method(cid, "channel.open_ok", channel_id=b""))
                return
            if ch is None:
                if m.name == "channel.close_ok":
                    return
                self._conn_close(c, wire.CHANNEL_ERROR, f"unknown channel {cid}", m.class_id, m.method_id)
                return
            self._ch_method(ch, m)
        elif ftype == wire.FRAME_HEADER:
            if ch is None or ch.pub_method is None:
                self._conn_close(c, wire.UNEXPECTED_FRAME, "unexpected content header")
                return
            _cls, size, props = wire.decode_content_header(payload)
            ch.pub_props = props
            ch.pub_size = size
            if size == 0:
                self._finish_publish(ch, b"")
        elif ftype == wire.FRAME_BODY:
            if ch is None or ch.pub_method is None or ch.pub_size < 0:
                self._conn_close(c, wire.UNEXPECTED_FRAME, "unexpected content body")
                return
            ch.pub_parts.append(payload)
            ch.pub_got += len(payload)
            if ch.pub_got >= ch.pub_size:
                self._finish_publish(ch, b"".join(ch.pub_parts))

    def _conn_method(self, c: _BConn, m: Method) -> None:
        n = m.name
        if n == "connection.start_ok":
            if m.mechanism != "PLAIN":
                self._conn_close(c, wire.ACCESS_REFUSED, "only PLAIN supported")
                return
            parts = bytes(m.response).split(b"\x00")
            user, pw = (parts[1].decode(), parts[2].decode()) if len(parts) >= 3 else ("", "")
            if self.users is not None and self.users.get(user) != pw:
                self._conn_close(c, wire.ACCESS_REFUSED, f"ACCESS_REFUSED - Login was refused using PLAIN "
                                                         f"for user '{user}'")
                return
            c.user = user
            c.send(wire.encode_method(0, "connection.tune", channel_max=2047, frame_max=self.frame_max,
                                      heartbeat=self.heartbeat))
        elif n == "connection.tune_ok":
            c.frame_max = m.frame_max or self.frame_max
            c.parser.frame_max = c.frame_max
            c.heartbeat = m.heartbeat
            if c.heartbeat:
                c.hb_task = asyncio.get_running_loop().create_task(self._heartbeats(c))
        elif n == "connection.open":
            if m.virtual_host not in self.vhosts:
                self._conn_close(c, wire.INVALID_PATH, f"NOT_ALLOWED - vhost {m.virtual_host} not found", 10, 40)
                return
            c.state = "open"
            c.send(wire.encode_method(0, "connection.open_ok", known_hosts=""))
        elif n == "connection.close":
            c.send(wire.encode_method(0, "connection.close_ok"))
            self._teardown(c)
            c.writer.close()
        elif n == "connection.close_ok":
            self._teardown(c)
            c.writer.close()

    def _ch_method(self, ch: _BChannel, m: Method) -> None:
        c = ch.conn
        n = m.name
        if not ch.open:
            return
        if n == "channel.close":
            c.send(wire.encode_method(ch.id, "channel.close_ok"))
            self._channel_gone(ch)
            c.channels.pop(ch.id, None)
        elif n == "channel.close_ok":
            c.channels.pop(ch.id, None)
        elif n == "channel.flow":
            ch.flow = m.active
            c.send(wire.encode_method(ch.id, "channel.flow_ok", active=m.active))
            if ch.flow:
                for cons in ch.consumers.values():
                    self._pump(cons.queue)
        elif n == "exchange.declare":
            ex = self.exchanges.get(m.exchange)
            if m.passive:
                if ex is None:
                    self._ch_close(ch, wire.NOT_FOUND, f"NOT_FOUND - no exchange '{m.exchange}'", 40, 10)
                    return
            elif ex is None:
                self.exchanges[m.exchange] = _Exchange(m.exchange, m.type, m.durable)
            elif ex.type != m.type:
                self._ch_close(ch, wire.PRECONDITION_FAILED, "PRECONDITION_FAILED - inequivalent arg 'type'",
                               40, 10)
                return
            if not m.nowait:
                c.send(wire.encode_method(ch.id, "exchange.declare_ok"))
        elif n == "queue.declare":
            name = m.queue or f"amq.gen-{id(ch):x}-{next(ch.tags)}"
            q = self.queues.get(name)
            if m.passive:
                if q is None:
                    self._ch_close(ch, wire.NOT_FOUND, f"NOT_FOUND - no queue '{name}'", 50, 10)
                    return
            elif q is None:
                q = self.queues[name] = _Queue(name, m.durable, c if m.exclusive else None, m.auto_delete)
            elif q.durable != m.durable:
                self._ch_close(ch, wire.PRECONDITION_FAILED,
                               f"PRECONDITION_FAILED - inequivalent arg 'durable' for queue '{name}'", 50, 10)
                return
            if not m.nowait:
                c.send(wire.encode_method(ch.id, "queue.declare_ok", queue=name, message_count=len(q.messages),
                                          consumer_count=len(q.consumers)))
        elif n == "queue.bind":
            ex = self.exchanges.get(m.exchange)
            if ex is None or m.queue not in self.queues:
                self._ch_close(ch, wire.NOT_FOUND, "NOT_FOUND - no exchange or queue", 50, 20)
                return
            ex.bindings.append((m.queue, m.routing_key))
            if not m.nowait:
                c.send(wire.encode_method(ch.id, "queue.bind_ok"))
        elif n == "queue.purge":
            q = self.queues.get(m.queue)
            cnt = len(q.messages) if q else 0
            if q:
                q.messages.clear()
            if not m.nowait:
                c.send(wire.encode_method(ch.id, "queue.purge_ok", message_count=cnt))
        elif n == "queue.delete":
            q = self.queues.pop(m.queue, None)
            cnt = len(q.messages) if q else 0
            if q:
                for cons in list(q.consumers):
                    cons.ch.conn.send(wire.encode_method(cons.ch.id, "basic.cancel", consumer_tag=cons.tag,
                                                         nowait=True))
                    cons.ch.consumers.pop(cons.tag, None)
                q.consumers.clear()
            if not m.nowait:
                c.send(wire.encode_method(ch.id, "queue.delete_ok", message_count=cnt))
        elif n == "basic.qos":
            ch.prefetch = m.prefetch_count
            c.send(wire.encode_method(ch.id, "basic.qos_ok"))
            for cons in ch.consumers.values():
                self._pump(cons.queue)
        elif n == "basic.consume":
            q = self.queues.get(m.queue)
            if q is None:
                self._ch_close(ch, wire.NOT_FOUND, f"NOT_FOUND - no queue '{m.queue}'", 60, 20)
                return
            tag = m.consumer_tag or f"amq.ctag-{id(ch):x}-{next(ch.tags)}"
            if tag in ch.consumers:
                self._conn_close(c, wire.COMMAND_INVALID, "NOT_ALLOWED - attempt to reuse consumer tag", 60, 20)
                return
            cons = _Consumer(ch, tag, q, m.no_ack)
            ch.consumers[tag] = cons
            q.consumers.append(cons)
            if not m.nowait:
                c.send(wire.encode_method(ch.id, "basic.consume_ok", consumer_tag=tag))
            self._pump(q)
        elif n == "basic.cancel":
            cons = ch.consumers.pop(m.consumer_tag, None)
            if cons is not None and cons in cons.queue.consumers:
                cons.queue.consumers.remove(cons)
            if not m.nowait:
                c.send(wire.encode_method(ch.id, "basic.cancel_ok", consumer_tag=m.consumer_tag))
        elif n == "basic.publish":
            ch.pub_method = m
            ch.pub_props = {}
            ch.pub_size = -1
            ch.pub_parts = []
            ch.pub_got = 0
        elif n in ("basic.ack", "basic.nack", "basic.reject"):
            self._settle(ch, m)
        elif n == "basic.recover" or n == "basic.recover_async":
            for tag in sorted(ch.unacked, reverse=True):
                q, msg, cons = ch.unacked.pop(tag)
                if cons is not None:
                    cons.unacked -= 1
                q.messages.appendleft((msg, True))
                q.requeued += 1
                self._pump(q)
            if n == "basic.recover":
                c.send(wire.encode_method(ch.id, "basic.recover_ok"))
        elif n == "confirm.select":
            ch.confirm = True
            if not m.nowait:
                c.send(wire.encode_method(ch.id, "confirm.select_ok"))
        else:
            self._ch_close(ch, wire.NOT_IMPLEMENTED, f"NOT_IMPLEMENTED - {n}", m.class_id, m.method_id)

    def _finish_publish(self, ch: _BChannel, body: bytes) -> None:
        m = ch.pub_method
        ch.pub_method = None
        ch.pub_parts = []
        if m.exchange not in self.exchanges:
            self._ch_close(ch, wire.NOT_FOUND, f"NOT_FOUND - no exchange '{m.exchange}'", 60, 40)
            return
        routed = self._route(m.exchange, m.routing_key, (body, ch.pub_props, m.exchange, m.routing_key))
        if routed == 0 and m.mandatory:
            ch.conn.send(wire.encode_method(ch.id, "basic.return", reply_code=wire.NO_ROUTE, reply_text="NO_ROUTE",
                                            exchange=m.exchange, routing_key=m.routing_key)
                         + wire.encode_content(ch.id, 60, body, ch.pub_props, ch.conn.frame_max))
        if ch.confirm:
            ch.pub_seq += 1
            ch.conn.send(wire.encode_method(ch.id, "basic.ack", delivery_tag=ch.pub_seq, multiple=False))

    def _route(self, exchange: str, routing_key: str, msg: Message) -> int:
        ex = self.exchanges.get(exchange)
        targets: List[str] = []
        if exchange == "":
            if routing_key in self.queues:
                targets = [routing_key]
        elif ex is not None:
            for qn, rk in ex.bindings:
                if ex.type == "fanout" or (ex.type == "direct" and rk == routing_key) or \
                        (ex.type == "topic" and _topic_match(rk, routing_key)):
                    if qn not in targets:
                        targets.append(qn)
        for qn in targets:
            q = self.queues.get(qn)
            if q is None:
                continue
            q.messages.append((msg, False))
            q.published += 1
            self._pump(q)
        return len(targets)

    def _settle(self, ch: _BChannel, m: Method) -> None:
        tag = m.delivery_tag
        multiple = m.args.get("multiple", False)
        if multiple:
            tags = [t for t in ch.unacked if t <= tag] if tag else list(ch.unacked)
        else:
            if tag not in ch.unacked:
                self._ch_close(ch, wire.PRECONDITION_FAILED, f"PRECONDITION_FAILED - unknown delivery tag {tag}",
                               m.class_id, m.method_id)
                return
            tags = [tag]
        requeue = m.args.get("requeue", False)
        touched = set()
        for t in sorted(tags):
            q, msg, cons = ch.unacked.pop(t)
            if cons is not None:
                cons.unacked -= 1
            if m.name == "basic.ack":
                q.acked += 1
            elif requeue:
                q.messages.appendleft((msg, True))
                q.requeued += 1
            else:
                q.dead_lettered += 1
            touched.add(q)
        for q in touched:
            self._pump(q)

    def _pump(self, q: _Queue) -> None:
        """Deliver as many queued messages as consumer prefetch windows allow (round-robin)."""
        while q.messages and q.consumers:
            n = len(q.consumers)
            cons = None
            for i in range(n):
                cand = q.consumers[(q.rr + i) % n]
                if cand.can_take() and not cand.ch.conn.closed:
                    cons = cand
                    q.rr = (q.rr + i + 1) % n
                    break
            if cons is None:
                return
            msg, redelivered = q.messages.popleft()
            ch = cons.ch
            tag = next(ch.tags)
            if not cons.no_ack:
                ch.unacked[tag] = (q, msg, cons)
                cons.unacked += 1
            else:
                q.acked += 1
            q.delivered += 1
            body, props, exchange, rk = msg
            ch.conn.send(wire.encode_method(ch.id, "basic.deliver", consumer_tag=cons.tag, delivery_tag=tag,
                                            redelivered=redelivered, exchange=exchange, routing_key=rk)
                         + wire.encode_content(ch.id, 60, body, props, ch.conn.frame_max))


async def serve_forever(host: str = "127.0.0.1", port: int = 5672) -> None:
    b = await AmqpBroker(host, port).start()
    print(f"beholder test broker listening on {b.url}", flush=True)
    try:
        await asyncio.Event().wait()
    finally:
        await b.stop()


class BrokerThread:
    """Runs an :class:`AmqpBroker` on its own event loop in a background thread."""

    def __init__(self, **kw):
        import threading
        self._kw = kw
        self.broker: Optional[AmqpBroker] = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._ready = threading.Event()
        self._thread = threading.Thread(target=self._run, daemon=True, name="amqp-broker")

    def _run(self) -> None:
        self._loop = asyncio.new_event_loop()
        asyncio.set_event_loop(self._loop)
        self.broker = self._loop.run_until_complete(AmqpBroker(**self._kw).start())
        self._ready.set()
        self._loop.run_forever()
        self._loop.run_until_complete(self.broker.stop())
        self._loop.close()

    def start(self) -> "BrokerThread":
        self._thread.start()
        self._ready.wait(10)
        return self

    def call(self, fn, *args):
        """Run ``fn(broker, *args)`` on the broker loop and return its result."""
        import concurrent.futures
        fut: concurrent.futures.Future = concurrent.futures.Future()

        def go():
            try:
                fut.set_result(fn(self.broker, *args))
            except BaseException as e:  # noqa: BLE001
                fut.set_exception(e)

        self._loop.call_soon_threadsafe(go)
        return fut.result(10)

    @property
    def url(self) -> str:
        return self.broker.url

    def stop(self) -> None:
        if self._loop is not None:
            self._loop.call_soon_threadsafe(self._loop.stop)
        self._thread.join(10)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
