"""AMQP 0-9-1 client/broker over real TCP: protocol, prefetch, acks, redelivery, reconnect.

The reference's transport is RabbitMQ via triton-core/amqplib (index.js:43-44,62,127).
These tests run our client against our broker on 127.0.0.1.
"""
import asyncio
import datetime
import decimal

import pytest

from beholder_amd.transport.amqp import AmqpBroker, AmqpError, AmqpPublisher, AmqpSource, Connection, wire
from beholder_amd.topics import PROGRESS, STATUS


def run(coro, timeout=30):
    return asyncio.run(asyncio.wait_for(coro, timeout))


def test_wire_table_roundtrip():
    t = {"s": "str", "i": 5, "big": 2**40, "neg": -3, "f": 1.5, "b": True, "n": None, "bytes": b"\x00\x01",
         "nested": {"a": [1, "x", False]}, "dec": decimal.Decimal("1.25"),
         "ts": datetime.datetime.fromtimestamp(1700000000, datetime.timezone.utc)}
    enc = wire.encode_table(t)
    dec = wire._Reader(enc).table()
    assert dec == t


def test_wire_method_bits_roundtrip():
    raw = wire.encode_method(3, "queue.declare", queue="q", passive=False, durable=True, exclusive=True,
                             auto_delete=False, nowait=True, arguments={"x-max-length": 10})
    fr = wire.FrameParser().feed(raw)
    assert fr[0][:2] == (wire.FRAME_METHOD, 3)
    m = wire.decode_method(fr[0][2])
    assert m.name == "queue.declare" and m.durable and m.exclusive and m.nowait and not m.passive
    assert m.arguments == {"x-max-length": 10}


def test_parse_url():
    p = wire.parse_url("amqp://u%40x:p%2F@mq:5673/v%2Fh?heartbeat=5")
    assert (p["user"], p["password"], p["host"], p["port"], p["vhost"], p["heartbeat"]) == \
        ("u@x", "p/", "mq", 5673, "v/h", 5)
    assert wire.parse_url("amqp://h")["vhost"] == "/"


def test_frame_parser_rejects_bad_frame_end():
    bad = b"\x08\x00\x00\x00\x00\x00\x00\x00"
    with pytest.raises(wire.FrameError):
        wire.FrameParser().feed(bad)


def test_connect_auth_failure():
    async def go():
        b = await AmqpBroker(users={"u": "right"}).start()
        try:
            with pytest.raises(AmqpError) as ei:
                await Connection(f"amqp://u:wrong@127.0.0.1:{b.port}/").open()
            assert ei.value.reply_code == wire.ACCESS_REFUSED
        finally:
            await b.stop()
    run(go())


def test_unknown_vhost_refused():
    async def go():
        b = await AmqpBroker().start()
        try:
            with pytest.raises(AmqpError):
                await Connection(f"amqp://guest:guest@127.0.0.1:{b.port}/nope").open()
        finally:
            await b.stop()
    run(go())


def test_publish_consume_large_body_multiple_frames():
    async def go():
        b = await AmqpBroker(frame_max=4096).start()
        got = asyncio.get_running_loop().create_future()
        try:
            c = await Connection(b.url).open()
            assert c.frame_max == 4096
            ch = await c.channel()
            await ch.queue_declare("q")
            await ch.basic_consume("q", lambda ch_, m, p, body: got.set_result((m, p, body)))
            body = bytes(range(256)) * 100  # 25600 bytes -> 7 body frames
            await ch.basic_publish(body, "q", properties={"content_type": "application/x-protobuf",
                                                          "headers": {"k": "v"}, "delivery_mode": 2})
            m, p, rbody = await got
            assert rbody == body and p["content_type"] == "application/x-protobuf" and p["headers"] == {"k": "v"}
            ch.basic_ack(m.delivery_tag)
            await asyncio.sleep(0.05)
            assert b.stats("q")["acked"] == 1
            await c.close()
        finally:
            await b.stop()
    run(go())


def test_prefetch_window_enforced_and_ack_releases():
    """basic.qos(100) (index.js:43): never more than `prefetch` un-acked per consumer."""
    async def go():
        b = await AmqpBroker().start()
        try:
            b.declare_queue("q")
            for i in range(50):
                b.publish("q", b"m%d" % i)
            c = await Connection(b.url).open()
            ch = await c.channel()
            await ch.basic_qos(10)
            seen = []
            await ch.basic_consume("q", lambda ch_, m, p, body: seen.append(m.delivery_tag))
            await asyncio.sleep(0.1)
            assert len(seen) == 10 and b.unacked("q") == 10 and b.depth("q") == 40
            ch.basic_ack(seen[4], multiple=True)  # acks tags 1..5
            await asyncio.sleep(0.1)
            assert len(seen) == 15 and b.unacked("q") == 10
            await c.close()
        finally:
            await b.stop()
    run(go())


def test_nack_requeue_redelivers_and_reject_drops():
    async def go():
        b = await AmqpBroker().start()
        try:
            b.declare_queue("q")
            b.publish("q", b"a")
            c = await Connection(b.url).open()
            ch = await c.channel()
            got = asyncio.Queue()
            await ch.basic_consume("q", lambda ch_, m, p, body: got.put_nowait((m, body)))
            m1, body = await got.get()
            assert not m1.redelivered
            ch.basic_nack(m1.delivery_tag, requeue=True)
            m2, body2 = await got.get()
            assert m2.redelivered and body2 == b"a"
            ch.basic_reject(m2.delivery_tag, requeue=False)
            await asyncio.sleep(0.05)
            assert b.stats("q")["dead_lettered"] == 1 and b.depth("q") == 0
            await c.close()
        finally:
            await b.stop()
    run(go())


def test_unknown_delivery_tag_closes_channel():
    async def go():
        b = await AmqpBroker().start()
        try:
            c = await Connection(b.url).open()
            ch = await c.channel()
            closed = asyncio.get_running_loop().create_future()
            ch.on_close = lambda ch_, err: closed.set_result(err)
            ch.basic_ack(999)
            err = await closed
            assert err.reply_code == wire.PRECONDITION_FAILED and not ch.is_open
            await c.close()
        finally:
            await b.stop()
    run(go())


def test_unacked_requeued_on_connection_close():
    async def go():
        b = await AmqpBroker().start()
        try:
            b.declare_queue("q")
            for i in range(3):
                b.publish("q", b"%d" % i)
            c = await Connection(b.url).open()
            ch = await c.channel()
            await ch.basic_consume("q", lambda *a: None)  # never acks
            await asyncio.sleep(0.05)
            assert b.unacked("q") == 3
            await c.close()
            await asyncio.sleep(0.05)
            assert b.depth("q") == 3 and b.stats("q")["requeued"] == 3
            assert [m[0][0] for m in b.queues["q"].messages] == [b"0", b"1", b"2"]  # order kept
        finally:
            await b.stop()
    run(go())


def test_publisher_confirms_and_mandatory_return():
    async def go():
        b = await AmqpBroker().start()
        try:
            pub = await AmqpPublisher(b.url).connect()
            fut = await pub.publish(STATUS, b"x", wait=True)
            assert fut.result() is True and b.depth(STATUS) == 1
            returned = asyncio.get_running_loop().create_future()
            pub._ch.on_return = lambda m, p, body: returned.set_result((m.reply_code, body))
            await pub._ch.basic_publish(b"lost", routing_key="no-such-queue", mandatory=True)
            assert await returned == (wire.NO_ROUTE, b"lost")
            await pub.close()
        finally:
            await b.stop()
    run(go())


def test_topic_and_fanout_exchanges():
    async def go():
        b = await AmqpBroker().start()
        try:
            c = await Connection(b.url).open()
            ch = await c.channel()
            await ch.exchange_declare("telemetry", "topic")
            await ch.queue_declare("all")
            await ch.queue_declare("prog")
            await ch.queue_bind("all", "telemetry", "v1.#")
            await ch.queue_bind("prog", "telemetry", "v1.telemetry.progress")
            await ch.basic_publish(b"p", "v1.telemetry.progress", exchange="telemetry")
            await ch.basic_publish(b"s", "v1.telemetry.status", exchange="telemetry")
            await asyncio.sleep(0.05)
            assert b.depth("all") == 2 and b.depth("prog") == 1
            with pytest.raises(AmqpError):
                await ch.exchange_declare("telemetry", "fanout")  # inequivalent type
            await c.close()
        finally:
            await b.stop()
    run(go())


def test_missed_heartbeats_detected():
    async def go():
        b = await AmqpBroker(heartbeat=1).start()
        b.mute_heartbeats = True
        try:
            lost = asyncio.get_running_loop().create_future()
            c = Connection(b.url, heartbeat=1, on_lost=lambda e: lost.done() or lost.set_result(e))
            await c.open()
            # stop our own heartbeats/acks reaching the broker too: the client must notice silence
            err = await asyncio.wait_for(lost, 6)
            assert err is not None
        finally:
            await b.stop()
    run(go(), timeout=20)


def test_source_consumes_topics_and_acks():
    async def go():
        b = await AmqpBroker().start()
        try:
            src = AmqpSource(b.url, prefetch=100)
            await src.start([STATUS, PROGRESS])
            b.publish(STATUS, b"s1")
            b.publish(PROGRESS, b"p1")
            batches = src.batches()
            got = []
            while len(got) < 2:
                got.extend(await batches.__anext__())
            assert sorted((d.topic, d.content) for d in got) == [(PROGRESS, b"p1"), (STATUS, b"s1")]
            for d in got:
                d.ack()
            await asyncio.sleep(0.05)
            assert b.stats(STATUS)["acked"] == 1 and b.stats(PROGRESS)["acked"] == 1
            await src.close()
        finally:
            await b.stop()
    run(go())


def test_source_startup_retries_then_fails_fast():
    """Q10 fix: retries+1 attempts, then the error propagates."""
    async def go():
        src = AmqpSource("amqp://guest:guest@127.0.0.1:1/", retries=2, backoff_initial=0.01)
        with pytest.raises(OSError):
            await src.start([STATUS])
    run(go())


def test_source_reconnects_after_broker_drop_and_redelivers():
    async def go():
        b = await AmqpBroker().start()
        try:
            src = AmqpSource(b.url, prefetch=10, backoff_initial=0.05)
            await src.start([STATUS])
            b.publish(STATUS, b"m1")
            it = src.batches()
            first = await it.__anext__()
            assert first[0].content == b"m1" and not first[0].redelivered
            await b.drop_connections()  # broker "crash" before the ack
            while src.ready():
                await asyncio.sleep(0.01)
            first[0].ack()  # stale: a no-op, the broker requeued it
            again = []
            while not again:
                again = await asyncio.wait_for(it.__anext__(), 10)
            assert again[0].content == b"m1" and again[0].redelivered
            again[0].ack()
            await asyncio.sleep(0.05)
            assert src.reconnects == 1 and src.stale_settles == 1 and b.stats(STATUS)["acked"] == 1
            await src.close()
        finally:
            await b.stop()
    run(go())


def _acks(frames: bytes):
    """basic.ack frames -> [(tag, multiple), ...]"""
    import struct
    out = []
    for i in range(0, len(frames), 21):
        ftype, ch, size, cls, meth, tag, bits, end = struct.unpack(">BHIHHQBB", frames[i:i + 21])
        assert (ftype, size, cls, meth, end) == (1, 13, 60, 80, 0xCE)
        out.append((tag, bool(bits)))
    return out


class _Token:
    pass


def _batcher():
    from beholder_amd.ops import AckBatcher
    scheduled = []
    b = AckBatcher(lambda: scheduled.append(1))
    ch = _Token()
    b.bind(ch, 1)
    return b, ch, scheduled


def test_ack_batcher_prefix_gap_and_nack():
    b, ch, scheduled = _batcher()  # tags 1..10 delivered on a fresh channel
    for t in (1, 2, 3, 5, 6):      # 4 still pending
        b.ack(t)
    assert len(scheduled) == 1     # one flush per burst
    assert _acks(b.flush()) == [(3, True), (5, False), (6, False)]
    b.settled_elsewhere(4)         # 4 nacked (sent immediately elsewhere)
    for t in (7, 8):
        b.ack(t)
    assert _acks(b.flush()) == [(8, True)]  # 4..8 contiguous now; never covers 9, 10
    b.ack(10)
    assert _acks(b.flush()) == [(10, False)]  # 9 outstanding -> no multiple
    assert b.flush() == b"" and len(scheduled) == 3


def test_ack_batcher_never_covers_an_unhandled_delivery():
    """A delivery received but never handled (connection.py `_deliver` for a cancelled
    consumer) stays un-acked even when later tags are acked: `multiple` stops at the gap."""
    b, ch, _ = _batcher()
    for t in (1, 2, 4, 5):
        b.ack(t)
    assert _acks(b.flush()) == [(2, True), (4, False), (5, False)]


def test_ack_batcher_abandoned_tag_stops_multiple_and_bounds_memory():
    """Q1: a status message left un-acked (its Delivery is freed pending) can never be covered
    by basic.ack(multiple); everything after it is acked singly and nothing is tracked."""
    b, ch, _ = _batcher()
    b.ack(1)
    b.abandon(2)
    for t in range(3, 1003):
        b.ack(t)
    frames = _acks(b.flush())
    assert frames[0] == (1, True) and all(not m for _, m in frames[1:]) and len(frames) == 1001
    assert b.stuck == 2 and b.tracked == 0


def test_ack_batcher_bounds_tracking_without_an_abandon_report():
    from beholder_amd.ops import AckBatcher
    b = AckBatcher(lambda: None, max_settled=100)
    b.bind(_Token(), 1)
    for t in range(2, 500):  # tag 1 never settles and is never reported
        b.ack(t)
    assert b.tracked <= 100 and b.stuck == 1
    assert all(not m for _, m in _acks(b.flush()))


def test_ack_batcher_native_settle_path():
    """Delivery.ack() of a bound channel's delivery is queued in C (no on_settle call); other
    channels and nacks take the Python callback; a freed pending delivery marks its tag stuck."""
    import gc

    from beholder_amd.ops import Delivery, Settler
    b, ch, _ = _batcher()
    calls = []
    s = Settler(on_settle=lambda d, kind, rq: calls.append((d.tag, kind)))
    s.ack_batcher = b
    Delivery(b"x", 1, 1, s, None, False, ch).ack()
    Delivery(b"x", 1, 2, s, None, False, ch).nack(True)
    Delivery(b"x", 1, 3, s, None, False, _Token()).ack()  # a stale channel's delivery
    d4 = Delivery(b"x", 1, 4, s, None, False, ch)
    del d4
    gc.collect()
    assert calls == [(2, "nack"), (3, "ack")] and b.acks == 1 and b.stuck == 4
    assert _acks(b.flush()) == [(1, True)]
    assert s.acked == 2 and s.nacked == 1 and s.abandoned == 1


def test_amqps_tls_with_ca_verification(tmp_path):
    """amqps:// with a private CA (?cafile=...) and hostname verification."""
    import shutil
    import ssl
    import subprocess
    if shutil.which("openssl") is None:
        pytest.skip("needs openssl")
    key, crt = tmp_path / "k.pem", tmp_path / "c.pem"
    r = subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out",
                        str(crt), "-days", "1", "-subj", "/CN=localhost", "-addext", "subjectAltName=DNS:localhost"],
                       capture_output=True)
    assert r.returncode == 0, r.stderr

    async def go():
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(str(crt), str(key))
        b = await AmqpBroker(ssl_context=ctx).start()
        try:
            url = f"amqps://guest:guest@127.0.0.1:{b.port}/?cafile={crt}&server_name=localhost"
            src = AmqpSource(url, prefetch=10)
            await src.start([STATUS])
            b.publish(STATUS, b"secure")
            got = await src.batches().__anext__()
            assert got[0].content == b"secure"
            got[0].ack()
            await src.close()
            with pytest.raises((ssl.SSLError, OSError)):  # untrusted without the CA
                await Connection(f"amqps://guest:guest@127.0.0.1:{b.port}/?server_name=localhost").open()
        finally:
            await b.stop()
    run(go())


def test_protocol_write_backpressure_and_loss_wake_the_publisher():
    """connection._Protocol: a publisher waits in drain() while the transport is paused, resumes
    on resume_writing(), and is woken (not left hanging) when the connection is lost meanwhile."""
    from beholder_amd.transport.amqp.connection import _Protocol

    class Conn:
        lost = None
        data = []

        def _on_data(self, b):
            self.data.append(b)

        def _on_transport_lost(self, exc):
            self.lost = exc

    class Transport:
        closing = False

        def is_closing(self):
            return self.closing

    async def go():
        c = Conn()
        p = _Protocol(c)
        p.connection_made(Transport())
        await p.drain()  # not paused: returns at once
        p.pause_writing()
        t = asyncio.ensure_future(p.drain())
        await asyncio.sleep(0.01)
        blocked = not t.done()
        p.resume_writing()
        await asyncio.wait_for(t, 1)
        p.pause_writing()
        t2 = asyncio.ensure_future(p.drain())
        await asyncio.sleep(0.01)
        err = ConnectionResetError("gone")
        p.connection_lost(err)
        await asyncio.wait_for(t2, 1)
        p.data_received(b"x")
        return blocked, c.lost is err, p.closed.done(), c.data
    blocked, lost, closed, data = asyncio.run(go())
    assert blocked and lost and closed and data == [b"x"]


def test_a_write_while_closing_on_purpose_is_not_a_loss():
    """an ack flushed in _abort's window (the transport already closing on purpose,
    ``_aborting`` set) is dropped; it must not reach ``on_lost`` as a connection loss (AmqpSource
    guards itself, but any other on_lost user would take a clean close for a failure)."""
    async def go():
        b = await AmqpBroker().start()
        try:
            lost = []
            c = Connection(b.url, on_lost=lost.append)
            await c.open()
            await c.channel()
            t = c._transport
            c._aborting = True  # what _abort sets right before it closes the transport
            t.close()
            c._write_now(b"\x01" * 21)  # an ack frame's size: the direct path
            c._write(b"\x01" * 21)      # and the scheduled flush
            await asyncio.sleep(0.05)  # the scheduled flush and the transport's connection_lost ran
            return list(lost)
        finally:
            await b.stop()
    assert run(go()) == []
