"""Hand-derived protocol vectors for what the clients DECODE (server -> client bytes).

tests/test_wire_conformance.py pins what the clients send. These pin what they receive: every
vector below is written out byte by byte from the specifications (AMQP 0-9-1, amqp0-9-1.xml +
the RabbitMQ errata; PostgreSQL v3 frontend/backend protocol), never produced by
``transport/amqp/wire.py`` or ``store/pgwire.py``, and is fed through the production decode
paths: the Python AMQP frame parser + method / content-header decoders, the native
``AmqpDemux`` (delivery assembly on the consumer channel), the native ``PgReader`` and a
``Pool`` talking to a scripted Postgres server. An encoder and decoder that drift together
(the in-repo broker and Postgres fake share the client's codecs) fail here.
"""
from __future__ import annotations

import asyncio

import pytest

from beholder_amd.ops import AmqpDemux, PgReader, Settler
from beholder_amd.store import pgwire
from beholder_amd.transport.amqp import wire


def h(s: str) -> bytes:
    """Hex with spaces and ``|`` separators (field boundaries) allowed."""
    return bytes.fromhex(s.replace(" ", "").replace("|", "").replace("\n", ""))


# ------------------------------------------------------------------ AMQP 0-9-1 -----------------
# basic.deliver (class 60 = 0x003c, method 60 = 0x003c) on channel 1:
#   consumer-tag "c1" | delivery-tag 7 | redelivered (bit) 1 | exchange "ex" | routing-key "rk"
DELIVER = h("01 | 0001 | 00000016 | 003c 003c | 02 6331 | 0000000000000007 | 01 | 02 6578 | 02 726b | ce")
# content header (frame type 2): class 60, weight 0, body-size 10, property flags 0xfffc (all 14
# basic properties present, bit 15 = content-type ... bit 2 = cluster-id), then in order:
#   content-type "ct", content-encoding "gz", headers {"k": longstr "v"}, delivery-mode 2,
#   priority 5, correlation-id "ci", reply-to "rt", expiration "60", message-id "mi",
#   timestamp 1700000000 (0x6553f100), type "ty", user-id "ui", app-id "ai", cluster-id "cl"
HEADERS_TABLE = h("00000008 | 01 6b | 53 | 00000001 | 76")
HEADER = h("02 | 0001 | 00000042 | 003c | 0000 | 000000000000000a | fffc"
           "| 02 6374 | 02 677a") + HEADERS_TABLE + h(
           "| 02 | 05 | 02 6369 | 02 7274 | 02 3630 | 02 6d69 | 000000006553f100 | 02 7479 | 02 7569 | 02 6169"
           "| 02 636c | ce")
# the 10-byte body "0123456789" split over two body frames (type 3)
BODY = h("03 | 0001 | 00000004 | 30313233 | ce") + h("03 | 0001 | 00000006 | 343536373839 | ce")
# server-initiated basic.cancel (consumer cancel notify): class 60 method 30 (0x1e), "c1", no-wait 1
CANCEL = h("01 | 0001 | 00000008 | 003c 001e | 02 6331 | 01 | ce")
# channel.close: class 20 (0x14) method 40 (0x28): 406 PRECONDITION_FAILED "PF", caused by
# class 60 method 80 (basic.ack)
CHANNEL_CLOSE = h("01 | 0001 | 0000000d | 0014 0028 | 0196 | 02 5046 | 003c | 0050 | ce")
# connection.close on channel 0: class 10 method 50 (0x32): 320 CONNECTION_FORCED "bye", 0, 0
CONNECTION_CLOSE = h("01 | 0000 | 0000000e | 000a 0032 | 0140 | 03 627965 | 0000 | 0000 | ce")
# connection.blocked (10, 60) "low memory" / connection.unblocked (10, 61)
BLOCKED = h("01 | 0000 | 0000000f | 000a 003c | 0a 6c6f77206d656d6f7279 | ce")
UNBLOCKED = h("01 | 0000 | 00000004 | 000a 003d | ce")
HEARTBEAT = h("08 | 0000 | 00000000 | ce")

ALL_PROPS = {"content_type": "ct", "content_encoding": "gz", "headers": {"k": "v"}, "delivery_mode": 2,
             "priority": 5, "correlation_id": "ci", "reply_to": "rt", "expiration": "60", "message_id": "mi",
             "timestamp": 1700000000, "type": "ty", "user_id": "ui", "app_id": "ai", "cluster_id": "cl"}
STREAM = DELIVER + HEADER + BODY + HEARTBEAT + CANCEL + BLOCKED + UNBLOCKED + CHANNEL_CLOSE + CONNECTION_CLOSE


def _python_decode(data: bytes, chunk: int):
    p = wire.FrameParser(frame_max=131072)
    frames = []
    for i in range(0, len(data), chunk):
        frames += p.feed(data[i:i + chunk])
    out = []
    for ftype, ch, payload in frames:
        if ftype == 1:
            m = wire.decode_method(payload)
            out.append(("method", ch, m.name, dict(m.args)))
        elif ftype == 2:
            out.append(("header", ch, wire.decode_content_header(payload)))
        else:
            out.append((ftype, ch, payload))
    return out


@pytest.mark.parametrize("chunk", [1, 3, 7, len(STREAM)])
def test_amqp_python_parser_decodes_server_frames(chunk):
    got = _python_decode(STREAM, chunk)
    assert got == [
        ("method", 1, "basic.deliver", {"consumer_tag": "c1", "delivery_tag": 7, "redelivered": True,
                                        "exchange": "ex", "routing_key": "rk"}),
        ("header", 1, (60, 10, ALL_PROPS)),
        (3, 1, b"0123"), (3, 1, b"456789"),
        (8, 0, b""),
        ("method", 1, "basic.cancel", {"consumer_tag": "c1", "nowait": True}),
        ("method", 0, "connection.blocked", {"reason": "low memory"}),
        ("method", 0, "connection.unblocked", {}),
        ("method", 1, "channel.close", {"reply_code": 406, "reply_text": "PF", "class_id": 60, "method_id": 80}),
        ("method", 0, "connection.close", {"reply_code": 320, "reply_text": "bye", "class_id": 0,
                                           "method_id": 0}),
    ]


@pytest.mark.parametrize("chunk", [1, 5, len(STREAM)])
def test_amqp_native_demux_assembles_the_delivery_and_passes_the_rest(chunk):
    s = Settler()
    dm = AmqpDemux(s, 0)
    dm.capture_headers = True
    dm.add_consumer(1, "c1", 2, None)
    out = []
    for i in range(0, len(STREAM), chunk):
        out += dm.feed(STREAM[i:i + chunk])
    d = out[0]
    assert (d.tag, d.topic_id, d.content, d.redelivered) == (7, 2, b"0123456789", True)
    assert d.headers == HEADERS_TABLE  # the raw `headers` table, found past the two shortstrs before it
    rest = [(t, ch, wire.decode_method(p).name if t == 1 else p) for t, ch, p in out[1:]]
    assert rest == [(1, 1, "basic.cancel"), (1, 0, "connection.blocked"), (1, 0, "connection.unblocked"),
                    (1, 1, "channel.close"), (1, 0, "connection.close")]


def test_amqp_client_channel_and_connection_react_to_server_methods():
    """The client's own dispatch (Connection._dispatch) on the vectors: a consumer-cancel
    notification drops the consumer and reports it, blocked/unblocked flip the flag, a
    channel.close is answered with close-ok and fails the channel, a connection.close is
    answered with close-ok and ends the connection."""
    from beholder_amd.transport.amqp.connection import Channel, Connection

    conn = Connection("amqp://guest:guest@127.0.0.1:1/")
    written = []
    conn._write = written.append
    conn._flush = lambda: None
    lost = []
    conn._lost = lost.append
    ch = Channel(conn, 1)
    conn._channels[1] = ch
    ch._consumers["c1"] = lambda *a: None
    closed = []
    ch.on_close = lambda c, err: closed.append(str(err))
    for ftype, chn, payload in wire.FrameParser().feed(CANCEL + BLOCKED):
        conn._dispatch(ftype, chn, payload)
    assert "c1" not in ch._consumers and closed == ["consumer c1 cancelled by broker"] and conn.blocked
    for ftype, chn, payload in wire.FrameParser().feed(UNBLOCKED + CHANNEL_CLOSE + CONNECTION_CLOSE):
        conn._dispatch(ftype, chn, payload)
    assert not conn.blocked
    # close-ok replies: channel.close_ok (20, 41) on channel 1, connection.close_ok (10, 51) on 0
    assert h("01 0001 00000004 0014 0029 ce") in written and h("01 0000 00000004 000a 0033 ce") in written
    assert [type(e).__name__ for e in lost] == ["AmqpError"] and "320 bye" in str(lost[0])


# ----------------------------------------------------------------- PostgreSQL v3 ---------------
AUTH_OK = h("52 | 00000008 | 00000000")                                   # AuthenticationOk
PS_VERSION = h("53 | 00000018 | 7365727665725f76657273696f6e00 | 31362e3200")  # server_version=16.2
KEYDATA = h("4b | 0000000c | 00000007 | 0000002a")                        # BackendKeyData pid 7
READY = h("5a | 00000005 | 49")                                           # ReadyForQuery idle
PARSE_OK, BIND_OK = h("31 00000004"), h("32 00000004")
# RowDescription: 1 field "v", table 0, attnum 0, type int4 (23), typlen 4, typmod -1, text
ROWDESC = h("54 | 0000001a | 0001 | 7600 | 00000000 | 0000 | 00000017 | 0004 | ffffffff | 0000")
ROW_42 = h("44 | 0000000c | 0001 | 00000002 | 3432")
ROW_7 = h("44 | 0000000b | 0001 | 00000001 | 37")
SELECT_1 = h("43 | 0000000d | 53454c4543542031 00")                       # CommandComplete "SELECT 1"
# NoticeResponse in the middle of a result: S "NOTICE", C "00000", M "hello"
NOTICE = h("4e | 0000001b | 53 4e4f5449434500 | 43 303030303000 | 4d 68656c6c6f00 | 00")
# ParameterStatus in the middle of a result (e.g. after SET): application_name=beh
PS_APP = h("53 | 00000019 | 6170706c69636174696f6e5f6e616d6500 | 62656800")
# ErrorResponse: S/V "ERROR", C "42P01", M "no such table"
ERROR = h("45 | 00000029 | 53 4552524f5200 | 56 4552524f5200 | 43 343250303100 | 4d 6e6f2073756368207461626c6500"
          "| 00")
# one pipeline of three Sync groups: a result with a notice and a parameter status inside it, a
# failed Parse (the server skips to Sync), a result on the cached statement
PIPELINE = (PARSE_OK + BIND_OK + ROWDESC + ROW_42 + NOTICE + SELECT_1 + PS_APP + READY
            + ERROR + READY
            + BIND_OK + ROWDESC + ROW_7 + SELECT_1 + READY)


@pytest.mark.parametrize("chunk", [1, 4, 9, len(PIPELINE)])
def test_pg_reader_on_a_pipeline_with_async_messages_and_an_error(chunk):
    r = PgReader()
    r.query_mode = True  # after startup: Sync groups are assembled into results
    out = []
    for i in range(0, len(PIPELINE), chunk):
        out += r.feed(PIPELINE[i:i + chunk])
    assert out == [
        (b"N", NOTICE[5:]),
        (b"S", PS_APP[5:]),
        ([(42,)], "SELECT 1", None, True),
        ([], "", {"S": "ERROR", "V": "ERROR", "C": "42P01", "M": "no such table"}, False),
        ([(7,)], "SELECT 1", None, False),
    ]
    assert r.buffered == 0


class _ScriptedPg:
    """Answers the startup with literal bytes, waits for three Sync messages, then sends PIPELINE
    in small pieces. Reads nothing else of what the client sends."""

    async def start(self):
        self.server = await asyncio.start_server(self._serve, "127.0.0.1", 0)
        self.port = self.server.sockets[0].getsockname()[1]
        return self

    async def _serve(self, reader, writer):
        n = int.from_bytes(await reader.readexactly(4), "big")
        await reader.readexactly(n - 4)  # StartupMessage
        writer.write(AUTH_OK + PS_VERSION + KEYDATA + READY)
        buf = b""
        while buf.count(h("53 00000004")) < 3:  # Sync
            chunk = await reader.read(65536)
            if not chunk:
                return
            buf += chunk
        for i in range(0, len(PIPELINE), 5):
            writer.write(PIPELINE[i:i + 5])
            await writer.drain()
        try:
            await reader.read()
        finally:
            writer.close()

    async def stop(self):
        self.server.close()
        await self.server.wait_closed()


@pytest.mark.parametrize("native_io", ["1", "0"])
def test_pg_pool_on_scripted_server(native_io, monkeypatch):
    monkeypatch.setenv("BEHOLDER_NATIVE_IO", native_io)

    async def go():
        srv = await _ScriptedPg().start()
        try:
            pool = await pgwire.Pool(f"postgres://u@127.0.0.1:{srv.port}/db?sslmode=disable", size=1).open()
            res = await asyncio.gather(pool.execute("SELECT $1::int4", (42,)), pool.execute("SELECT * FROM x"),
                                       pool.execute("SELECT $1::int4", (7,)), return_exceptions=True)
            c = pool._conns[0]
            out = (res, dict(c.server_params), list(c.notices), c.backend_pid, c._net is not None)
            await pool.close()
            return out
        finally:
            await srv.stop()
    res, params, notices, pid, native = asyncio.run(asyncio.wait_for(go(), 20))
    assert res[0] == ([(42,)], "SELECT 1") and res[2] == ([(7,)], "SELECT 1")
    assert isinstance(res[1], pgwire.PgError) and str(res[1]) == "ERROR 42P01: no such table"
    assert res[1].sqlstate == "42P01"
    assert params == {"server_version": "16.2", "application_name": "beh"}
    assert notices == [{"S": "NOTICE", "C": "00000", "M": "hello"}]
    assert pid == 7 and native == (native_io == "1")
