"""Asyncio AMQP 0-9-1 client: connection + channels.

Covers what triton-core's amqplib wrapper gives beholder (index.js:43-44,62,127):
connection handshake (PLAIN auth, tune negotiation, vhost open), channels,
``queue.declare``, ``exchange.declare``, ``queue.bind``, ``basic.qos``,
``basic.consume`` / ``basic.cancel``, ``basic.ack`` / ``nack`` / ``reject``,
``basic.publish`` (optionally with publisher confirms), heartbeats and
server-initiated ``connection.close`` / ``channel.close``.

Outgoing frames are coalesced: writes issued during one event-loop iteration
(e.g. the acks of a whole delivery batch) go out in a single ``send``.
"""
from __future__ import annotations

import asyncio
import itertools
import os
import time
from typing import Any, Callable, Dict, List, Optional

from . import wire
from .wire import AmqpError, Method

CLIENT_PROPERTIES = {
    "product": "beholder_amd",
    "version": "1.0.0",
    "platform": "python-asyncio",
    "capabilities": {"publisher_confirms": True, "consumer_cancel_notify": True,
                     "basic.nack": True, "connection.blocked": True},
}


def _negotiate(server: int, client: int) -> int:
    if server == 0 or client == 0:
        return max(server, client)
    return min(server, client)


class Channel:
    def __init__(self, conn: "Connection", cid: int):
        self.conn = conn
        self.id = cid
        self.is_open = False
        self._rpc_lock = asyncio.Lock()
        self._waiter: Optional[asyncio.Future] = None
        self._expect: tuple = ()
        self._consumers: Dict[str, Callable] = {}
        # content assembly state
        self._cmethod: Optional[Method] = None
        self._cprops: Dict[str, Any] = {}
        self._csize = 0
        self._cparts: list = []
        self._cgot = 0
        # publisher confirms
        self._confirm = False
        self._pub_seq = 0
        self._unconfirmed: Dict[int, asyncio.Future] = {}
        self.on_close: Optional[Callable[["Channel", Optional[AmqpError]], None]] = None
        self.on_return: Optional[Callable[[Method, Dict[str, Any], bytes], None]] = None
        self.close_reason: Optional[AmqpError] = None
        self.flow_active = True

    # ---------------------------------------------------------------- rpc ---
    async def _rpc(self, name: str, expect: tuple, **args) -> Method:
        if not self.is_open and name != "channel.open":
            raise AmqpError(f"channel {self.id} is closed", wire.CHANNEL_ERROR)
        async with self._rpc_lock:
            fut = asyncio.get_running_loop().create_future()
            self._waiter = fut
            self._expect = expect
            self.conn._write(wire.encode_method(self.id, name, **args))
            try:
                return await fut
            finally:
                self._waiter = None

    async def open(self) -> "Channel":
        await self._rpc("channel.open", ("channel.open_ok",), out_of_band="")
        self.is_open = True
        return self

    async def close(self, reply_code: int = wire.REPLY_SUCCESS, reply_text: str = "bye") -> None:
        if not self.is_open:
            return
        try:
            await asyncio.wait_for(self._rpc("channel.close", ("channel.close_ok",), reply_code=reply_code,
                                             reply_text=reply_text, class_id=0, method_id=0), 5)
        except (asyncio.TimeoutError, AmqpError, ConnectionError):
            pass
        self._closed(None)

    async def exchange_declare(self, exchange: str, type: str = "direct", durable: bool = True,
                               auto_delete: bool = False, passive: bool = False, arguments=None) -> None:
        await self._rpc("exchange.declare", ("exchange.declare_ok",), exchange=exchange, type=type, passive=passive,
                        durable=durable, auto_delete=auto_delete, arguments=arguments or {})

    async def queue_declare(self, queue: str = "", durable: bool = True, exclusive: bool = False,
                            auto_delete: bool = False, passive: bool = False, arguments=None) -> Method:
        return await self._rpc("queue.declare", ("queue.declare_ok",), queue=queue, passive=passive,
                               durable=durable, exclusive=exclusive, auto_delete=auto_delete,
                               arguments=arguments or {})

    async def queue_bind(self, queue: str, exchange: str, routing_key: str = "", arguments=None) -> None:
        await self._rpc("queue.bind", ("queue.bind_ok",), queue=queue, exchange=exchange, routing_key=routing_key,
                        arguments=arguments or {})

    async def queue_purge(self, queue: str) -> int:
        m = await self._rpc("queue.purge", ("queue.purge_ok",), queue=queue)
        return m.message_count

    async def queue_delete(self, queue: str) -> int:
        m = await self._rpc("queue.delete", ("queue.delete_ok",), queue=queue)
        return m.message_count

    async def basic_qos(self, prefetch_count: int, prefetch_size: int = 0, global_: bool = False) -> None:
        await self._rpc("basic.qos", ("basic.qos_ok",), prefetch_size=prefetch_size, prefetch_count=prefetch_count,
                        global_=global_)

    async def basic_consume(self, queue: str, on_message: Callable, consumer_tag: str = "",
                            no_ack: bool = False, exclusive: bool = False, arguments=None,
                            native_topic: Optional[int] = None) -> str:
        """``on_message(channel, deliver_method, properties, body)`` runs in the reader task.

        The consumer tag is chosen client-side and the callback registered
        *before* ``basic.consume`` is sent: the broker may deliver in the same
        TCP segment as ``consume_ok``.
        """
        tag = consumer_tag or f"beholder.ctag-{self.conn._ctag_prefix}-{next(self.conn._ctags)}"
        self._consumers[tag] = on_message
        demux = self.conn._demux
        if native_topic is not None and demux is not None:
            # deliveries for this consumer are assembled natively into Delivery objects
            # (extra = this channel, so settling routes the ack back here)
            demux.add_consumer(self.id, tag, int(native_topic), self)
        try:
            await self._rpc("basic.consume", ("basic.consume_ok",), queue=queue, consumer_tag=tag,
                            no_local=False, no_ack=no_ack, exclusive=exclusive, arguments=arguments or {})
        except BaseException:
            self._consumers.pop(tag, None)
            if demux is not None:
                demux.remove_consumer(self.id, tag)
            raise
        return tag

    async def basic_cancel(self, consumer_tag: str) -> None:
        if self.is_open:
            await self._rpc("basic.cancel", ("basic.cancel_ok",), consumer_tag=consumer_tag)
        self._consumers.pop(consumer_tag, None)
        if self.conn._demux is not None:
            self.conn._demux.remove_consumer(self.id, consumer_tag)

    def basic_ack(self, delivery_tag: int, multiple: bool = False) -> None:
        self.conn._write(wire.encode_ack(self.id, delivery_tag, multiple))

    def basic_nack(self, delivery_tag: int, multiple: bool = False, requeue: bool = True) -> None:
        self.conn._write(wire.encode_method(self.id, "basic.nack", delivery_tag=delivery_tag, multiple=multiple,
                                            requeue=requeue))

    def basic_reject(self, delivery_tag: int, requeue: bool = False) -> None:
        self.conn._write(wire.encode_method(self.id, "basic.reject", delivery_tag=delivery_tag, requeue=requeue))

    async def confirm_select(self) -> None:
        await self._rpc("confirm.select", ("confirm.select_ok",), nowait=False)
        self._confirm = True

    async def basic_publish(self, body: bytes, routing_key: str, exchange: str = "",
                            properties: Optional[Dict[str, Any]] = None, mandatory: bool = False,
                            wait_confirm: bool = False) -> Optional[asyncio.Future]:
        if not self.is_open:
            raise AmqpError(f"channel {self.id} is closed", wire.CHANNEL_ERROR)
        frames = (wire.encode_method(self.id, "basic.publish", exchange=exchange, routing_key=routing_key,
                                     mandatory=mandatory, immediate=False)
                  + wire.encode_content(self.id, 60, body, properties, self.conn.frame_max))
        fut = None
        if self._confirm:
            self._pub_seq += 1
            fut = asyncio.get_running_loop().create_future()
            self._unconfirmed[self._pub_seq] = fut
        self.conn._write(frames)
        await self.conn._maybe_drain()
        if wait_confirm and fut is not None:
            await fut
        return fut

    async def wait_confirms(self) -> None:
        if self._unconfirmed:
            await asyncio.gather(*list(self._unconfirmed.values()))

    # ----------------------------------------------------------- inbound ---
    def _on_method(self, m: Method) -> None:
        name = m.name
        if m.has_content:
            self._cmethod = m
            self._cparts = []
            self._cgot = 0
            self._csize = -1
            return
        if name == "channel.close":
            err = AmqpError(f"channel closed by broker: {m.reply_code} {m.reply_text}", m.reply_code,
                            m.class_id, m.method_id)
            self.conn._write(wire.encode_method(self.id, "channel.close_ok"))
            self._closed(err)
            return
        if name == "basic.cancel":  # consumer_cancel_notify (queue deleted, ...)
            self._consumers.pop(m.consumer_tag, None)
            if self.conn._demux is not None:
                self.conn._demux.remove_consumer(self.id, m.consumer_tag)
            if self.on_close:
                self.on_close(self, AmqpError(f"consumer {m.consumer_tag} cancelled by broker"))
            return
        if name in ("basic.ack", "basic.nack") and self._confirm:
            self._settle_confirms(m.delivery_tag, m.multiple, name == "basic.ack")
            return
        if name == "channel.flow":
            self.flow_active = m.active
            self.conn._write(wire.encode_method(self.id, "channel.flow_ok", active=m.active))
            return
        w = self._waiter
        if w is not None and not w.done() and name in self._expect:
            w.set_result(m)
            return
        if name.endswith("_ok") and w is None:
            return  # late reply to a timed-out rpc
        self.conn._protocol_error(f"unexpected {name} on channel {self.id}", wire.UNEXPECTED_FRAME)

    def _on_header(self, payload: bytes) -> None:
        if self._cmethod is None:
            self.conn._protocol_error("content header without method", wire.UNEXPECTED_FRAME)
            return
        _cid, size, props = wire.decode_content_header(payload)
        self._cprops = props
        self._csize = size
        if size == 0:
            self._deliver(b"")

    def _on_body(self, payload: bytes) -> None:
        if self._cmethod is None or self._csize < 0:
            self.conn._protocol_error("body frame without header", wire.UNEXPECTED_FRAME)
            return
        self._cparts.append(payload)
        self._cgot += len(payload)
        if self._cgot >= self._csize:
            body = self._cparts[0] if len(self._cparts) == 1 else b"".join(self._cparts)
            self._deliver(body)

    def _deliver(self, body: bytes) -> None:
        m = self._cmethod
        props = self._cprops
        self._cmethod = None
        self._cparts = []
        if m.name == "basic.deliver":
            cb = self._consumers.get(m.consumer_tag)
            if cb is not None:
                cb(self, m, props, body)
            # a delivery for a cancelled consumer stays un-acked -> requeued on close
        elif m.name == "basic.return" and self.on_return is not None:
            self.on_return(m, props, body)

    def _settle_confirms(self, tag: int, multiple: bool, ok: bool) -> None:
        tags = [t for t in self._unconfirmed if t <= tag] if multiple else [tag]
        for t in tags:
            fut = self._unconfirmed.pop(t, None)
            if fut is not None and not fut.done():
                if ok:
                    fut.set_result(True)
                else:
                    fut.set_exception(AmqpError(f"message {t} nacked by broker"))

    def _closed(self, err: Optional[AmqpError]) -> None:
        if not self.is_open and self.close_reason is not None:
            return
        self.is_open = False
        self.close_reason = err
        self.conn._channels.pop(self.id, None)
        if self.conn._demux is not None:
            self.conn._demux.reset_channel(self.id)
        w = self._waiter
        if w is not None and not w.done():
            w.set_exception(err or AmqpError(f"channel {self.id} closed", wire.CHANNEL_ERROR))
        for fut in self._unconfirmed.values():
            if not fut.done():
                fut.set_exception(err or AmqpError("channel closed before confirm"))
        self._unconfirmed.clear()
        if self.on_close is not None:
            cb, self.on_close = self.on_close, None
            cb(self, err)


class _Protocol(asyncio.Protocol):
    """The socket side of a :class:`Connection`: bytes go to ``Connection._on_data`` as they
    arrive (no StreamReader buffer, no read-loop coroutine resumed per read: one callback per
    socket read, the way the loop delivers them), writes go to the transport directly, and
    ``pause_writing`` / ``resume_writing`` give the publisher its back-pressure."""

    def __init__(self, conn: "Connection"):
        self.conn = conn
        self.transport: Optional[asyncio.Transport] = None
        self.paused = False
        self._drain: List[asyncio.Future] = []
        self.closed: Optional[asyncio.Future] = None

    def connection_made(self, transport) -> None:
        self.transport = transport
        self.closed = asyncio.get_running_loop().create_future()

    def data_received(self, data: bytes) -> None:
        self.conn._on_data(data)

    def eof_received(self):
        return False  # close the transport: connection_lost follows

    def connection_lost(self, exc) -> None:
        if self.closed is not None and not self.closed.done():
            self.closed.set_result(None)
        self._wake_drain()
        self.conn._on_transport_lost(exc)

    def pause_writing(self) -> None:
        self.paused = True

    def resume_writing(self) -> None:
        self.paused = False
        self._wake_drain()

    def _wake_drain(self) -> None:
        for f in self._drain:
            if not f.done():
                f.set_result(None)
        self._drain.clear()

    async def drain(self) -> None:
        if self.paused and self.transport is not None and not self.transport.is_closing():
            f = asyncio.get_running_loop().create_future()
            self._drain.append(f)
            await f


class Connection:
    def __init__(self, url: str, *, heartbeat: Optional[int] = None, connect_timeout: float = 10.0,
                 logger=None, on_lost: Optional[Callable[[Optional[BaseException]], None]] = None,
                 native_settler=None, on_deliveries: Optional[Callable[[List[Any]], None]] = None,
                 capture_headers: bool = False):
        """``native_settler`` + ``on_deliveries`` enable the native delivery path
        (:class:`~beholder_amd.ops.AmqpDemux`): deliveries for consumers
        registered with ``native_topic`` arrive as native ``Delivery`` objects
        through ``on_deliveries`` (a list per socket read); all other frames take the Python path."""
        self.params = wire.parse_url(url)
        if heartbeat is not None:
            self.params["heartbeat"] = heartbeat
        self.url = url
        self.connect_timeout = connect_timeout
        self.log = logger
        self.on_lost = on_lost
        self.frame_max = self.params["frame_max"]
        self.channel_max = self.params["channel_max"]
        self.heartbeat = self.params["heartbeat"]
        self.server_properties: Dict[str, Any] = {}
        self.is_open = False
        self.blocked = False
        self._proto: Optional[_Protocol] = None
        self._transport: Optional[asyncio.Transport] = None
        self._aborting = False  # the transport is being closed on purpose: its loss is not reported
        self._parser = wire.FrameParser(0)
        self._channels: Dict[int, Channel] = {}
        self._ids = itertools.count(1)
        self._ctags = itertools.count(1)
        self._ctag_prefix = f"{os.getpid()}-{id(self):x}"
        self._hb_task: Optional[asyncio.Task] = None
        self._wbuf = bytearray()
        self._flush_scheduled = False
        self._last_rx = 0.0
        self._last_tx = 0.0
        self._handshake: Optional[asyncio.Future] = None
        self._close_waiter: Optional[asyncio.Future] = None
        self._lost_reported = False
        self.bytes_in = 0
        self.bytes_out = 0
        self.reads = 0  # data_received calls (one socket read each)
        self.writes = 0  # transport.write calls
        self.on_deliveries = on_deliveries
        self._demux = None
        if native_settler is not None and on_deliveries is not None:
            from ...ops import AmqpDemux
            self._demux = AmqpDemux(native_settler, 0)
            self._demux.capture_headers = capture_headers  # Delivery.headers (trace context)

    # ------------------------------------------------------------- open ----
    async def open(self) -> "Connection":
        p = self.params
        loop = asyncio.get_running_loop()
        ssl_ctx = None
        server_hostname = None
        if p["ssl"]:
            import ssl
            ssl_ctx = ssl.create_default_context(cafile=p.get("cafile"))
            if p.get("certfile"):
                ssl_ctx.load_cert_chain(p["certfile"], p.get("keyfile"))
            if not p.get("verify", True):
                ssl_ctx.check_hostname = False
                ssl_ctx.verify_mode = ssl.CERT_NONE
            server_hostname = p.get("server_name") or p["host"]
        self._handshake = loop.create_future()
        self._transport, self._proto = await asyncio.wait_for(
            loop.create_connection(lambda: _Protocol(self), p["host"], p["port"], ssl=ssl_ctx,
                                   server_hostname=server_hostname),
            self.connect_timeout)
        self._transport.write(wire.PROTOCOL_HEADER)
        self._last_rx = self._last_tx = time.monotonic()
        try:
            await asyncio.wait_for(asyncio.shield(self._handshake), self.connect_timeout)
        except BaseException:
            await self._abort()
            raise
        self.is_open = True
        if self.heartbeat:
            self._hb_task = loop.create_task(self._heartbeat_loop())
        return self

    async def channel(self) -> Channel:
        if not self.is_open:
            raise AmqpError("connection is closed", wire.CONNECTION_FORCED)
        cid = next(self._ids)
        if self.channel_max and cid > self.channel_max:
            raise AmqpError("channel_max exceeded", wire.CHANNEL_ERROR)
        ch = Channel(self, cid)
        self._channels[cid] = ch
        return await ch.open()

    async def close(self, reply_text: str = "bye") -> None:
        if not self.is_open:
            await self._abort()
            return
        self.is_open = False
        self._close_waiter = asyncio.get_running_loop().create_future()
        self._write(wire.encode_method(0, "connection.close", reply_code=wire.REPLY_SUCCESS, reply_text=reply_text,
                                       class_id=0, method_id=0))
        try:
            await asyncio.wait_for(self._close_waiter, 5)
        except (asyncio.TimeoutError, ConnectionError, AmqpError):
            pass
        self._lost_reported = True  # orderly close: not a loss
        await self._abort()

    # ------------------------------------------------------------ writes ---
    def _write(self, data: bytes) -> None:
        self._wbuf += data
        if not self._flush_scheduled:
            self._flush_scheduled = True
            asyncio.get_running_loop().call_soon(self._flush)

    def _write_now(self, data: bytes) -> None:
        """Append and send at once (with anything already queued, in order): the ack flush runs
        once per loop iteration already, so it need not wait for another one."""
        if self._aborting:  # closing on purpose: a late write (an ack) is dropped, not a loss
            return
        t = self._transport
        if not self._wbuf and t is not None and not t.is_closing():  # nothing queued: no copy
            try:
                t.write(data)
            except (ConnectionError, RuntimeError) as e:
                self._lost(e)
                return
            self.bytes_out += len(data)
            self.writes += 1
            self._last_tx = time.monotonic()
            return
        self._wbuf += data
        self._flush()

    def _flush(self) -> None:
        self._flush_scheduled = False
        t = self._transport
        if not self._wbuf or t is None:
            return
        if self._aborting:  # the transport is being closed on purpose (_abort): not a loss
            self._wbuf.clear()
            return
        if t.is_closing():
            self._wbuf.clear()
            self._lost(ConnectionError("connection is closed"))
            return
        data = bytes(self._wbuf)
        self._wbuf.clear()
        try:
            t.write(data)
        except (ConnectionError, RuntimeError) as e:
            self._lost(e)
            return
        self.bytes_out += len(data)
        self.writes += 1
        self._last_tx = time.monotonic()

    async def _maybe_drain(self) -> None:
        t = self._transport
        if t is not None and t.get_write_buffer_size() > (4 << 20):
            self._flush()
            await self._proto.drain()

    # ------------------------------------------------------------- reads ---
    def _on_data(self, data: bytes) -> None:
        """One socket read (``_Protocol.data_received``): frames to the native delivery demux or
        the Python parser. A protocol error ends the connection as a loss."""
        if self._aborting:
            return
        self.bytes_in += len(data)
        self.reads += 1
        self._last_rx = time.monotonic()
        try:
            demux = self._demux
            if demux is not None:
                before = demux.passthrough
                try:
                    items = demux.feed(data)
                except ValueError as e:
                    raise wire.FrameError(str(e), wire.FRAME_ERROR) from None
                if demux.passthrough == before:
                    if items:
                        self.on_deliveries(items)  # only deliveries: hand over the whole list
                else:
                    on_deliveries = self.on_deliveries
                    for it in items:  # control frames interleaved: keep stream order
                        if type(it) is tuple:
                            self._dispatch(*it)
                        else:
                            on_deliveries([it])
            else:
                for ftype, ch, payload in self._parser.feed(data):
                    self._dispatch(ftype, ch, payload)
        except (ConnectionError, OSError, AmqpError) as e:
            self._lost(e)

    def _on_transport_lost(self, exc: Optional[BaseException]) -> None:
        if self._aborting:
            return
        self._lost(exc if exc is not None else ConnectionError("connection closed by peer"))

    def _dispatch(self, ftype: int, ch: int, payload: bytes) -> None:
        if ftype == wire.FRAME_HEARTBEAT:
            return
        if ch == 0:
            if ftype != wire.FRAME_METHOD:
                raise wire.FrameError("non-method frame on channel 0", wire.COMMAND_INVALID)
            self._on_conn_method(wire.decode_method(payload))
            return
        chan = self._channels.get(ch)
        if chan is None:
            return  # frames for a channel we already closed
        if ftype == wire.FRAME_METHOD:
            chan._on_method(wire.decode_method(payload))
        elif ftype == wire.FRAME_HEADER:
            chan._on_header(payload)
        elif ftype == wire.FRAME_BODY:
            chan._on_body(payload)
        else:
            raise wire.FrameError(f"unknown frame type {ftype}", wire.FRAME_ERROR)

    def _on_conn_method(self, m: Method) -> None:
        p = self.params
        name = m.name
        if name == "connection.start":
            mechs = m.mechanisms.decode() if isinstance(m.mechanisms, bytes) else m.mechanisms
            if "PLAIN" not in mechs.split():
                self._fail_handshake(AmqpError(f"broker does not offer PLAIN auth ({mechs})", wire.ACCESS_REFUSED))
                return
            self.server_properties = m.server_properties
            resp = b"\x00" + p["user"].encode() + b"\x00" + p["password"].encode()
            self._write(wire.encode_method(0, "connection.start_ok", client_properties=CLIENT_PROPERTIES,
                                           mechanism="PLAIN", response=resp, locale="en_US"))
        elif name == "connection.tune":
            self.channel_max = _negotiate(m.channel_max, p["channel_max"]) or 65535
            self.frame_max = _negotiate(m.frame_max, p["frame_max"]) or 131072
            self.heartbeat = _negotiate(m.heartbeat, p["heartbeat"])
            self._parser.frame_max = self.frame_max
            if self._demux is not None:
                self._demux.set_frame_max(self.frame_max)
            self._write(wire.encode_method(0, "connection.tune_ok", channel_max=self.channel_max,
                                           frame_max=self.frame_max, heartbeat=self.heartbeat))
            self._write(wire.encode_method(0, "connection.open", virtual_host=p["vhost"], capabilities="",
                                           insist=False))
        elif name == "connection.open_ok":
            if self._handshake and not self._handshake.done():
                self._handshake.set_result(True)
        elif name == "connection.close":
            err = AmqpError(f"connection closed by broker: {m.reply_code} {m.reply_text}", m.reply_code,
                            m.class_id, m.method_id)
            self._write(wire.encode_method(0, "connection.close_ok"))
            self._flush()
            self._fail_handshake(err)
            self._lost(err)
        elif name == "connection.close_ok":
            if self._close_waiter and not self._close_waiter.done():
                self._close_waiter.set_result(True)
        elif name == "connection.blocked":
            self.blocked = True
        elif name == "connection.unblocked":
            self.blocked = False

    def _fail_handshake(self, err: BaseException) -> None:
        if self._handshake and not self._handshake.done():
            self._handshake.set_exception(err)

    def _protocol_error(self, text: str, code: int) -> None:
        self._write(wire.encode_method(0, "connection.close", reply_code=code, reply_text=text[:255],
                                       class_id=0, method_id=0))
        self._lost(AmqpError(text, code))

    async def _heartbeat_loop(self) -> None:
        hb = float(self.heartbeat)
        try:
            while self.is_open:
                await asyncio.sleep(hb / 2)
                now = time.monotonic()
                if now - self._last_tx >= hb / 2:
                    self._write(wire.encode_heartbeat())
                if now - self._last_rx > 2 * hb:
                    self._lost(AmqpError("missed heartbeats from broker", wire.CONNECTION_FORCED))
                    return
        except asyncio.CancelledError:
            pass

    # -------------------------------------------------------------- loss ---
    def _lost(self, err: Optional[BaseException]) -> None:
        was_open = self.is_open
        self.is_open = False
        self._fail_handshake(err or ConnectionError("connection lost"))
        for ch in list(self._channels.values()):
            ch._closed(err if isinstance(err, AmqpError) else AmqpError(str(err or "connection lost")))
        if self._close_waiter and not self._close_waiter.done():
            self._close_waiter.set_result(True)
        if self._transport is not None:
            try:
                self._transport.close()
            except Exception:  # noqa: BLE001
                pass
        if self._hb_task is not None:
            self._hb_task.cancel()
        if not self._lost_reported and not self._aborting and (was_open or err is not None):
            self._lost_reported = True
            if self.on_lost is not None:
                self.on_lost(err)

    async def _abort(self) -> None:
        self.is_open = False
        if self._hb_task is not None:
            self._hb_task.cancel()
        t, proto = self._transport, self._proto
        if t is not None:
            try:
                self._flush()
            except Exception:  # noqa: BLE001
                pass
            self._aborting = True  # from here on, reads and the transport's loss are ours
            try:
                t.close()
                if proto is not None and proto.closed is not None:
                    await asyncio.wait_for(asyncio.shield(proto.closed), 2)
            except Exception:  # noqa: BLE001
                pass
            self._transport = None


async def connect(url: str, **kw) -> Connection:
    return await Connection(url, **kw).open()


__all__ = ["Connection", "Channel", "connect", "AmqpError"]
