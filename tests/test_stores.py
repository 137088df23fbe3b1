"""Media stores (triton-core/db parity, index.js:42,68,76,140): memory, sqlite, postgres (wire protocol)."""
import asyncio

import pytest

from beholder_amd.store import Media, MediaNotFound, MemoryStore, open_store
from beholder_amd.store.pgwire import PgConnection, PgError, PgProtocolError
from beholder_amd.store.postgres import PostgresStore

from pg_fake import FakePg

M1 = Media(id="m1", name="Bebop", creator=1, creatorId="card", metadataId="1", status=2)


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


async def _contract(st):
    await st.connect()
    try:
        await st.upsert(M1)
        await st.upsert(Media(id="m2", name="Trigun"))
        assert await st.count() == 2
        assert await st.get_by_id("m1") == M1
        await st.update_status("m1", 4)
        assert (await st.getByID("m1")).status == 4
        await st.updateStatus("missing", 3)  # UPDATE of zero rows: no error
        with pytest.raises(MediaNotFound):
            await st.get_by_id("missing")
        await st.upsert(M1._replace(name="Cowboy Bebop"))
        got = await st.get_by_id("m1")
        assert got.name == "Cowboy Bebop" and got.status == 2 and await st.count() == 2
    finally:
        await st.close()


def test_memory_store_contract():
    run(_contract(MemoryStore()))


def test_sqlite_store_contract(tmp_path):
    run(_contract(open_store("sqlite", str(tmp_path / "media.db"))))


@pytest.mark.parametrize("auth", ["scram", "md5", "cleartext", "trust"])
def test_postgres_store_contract_over_wire(auth):
    async def go():
        pg = await FakePg(auth=auth).start()
        try:
            await _contract(PostgresStore(pg.dsn, create_schema=True, pool_size=2))
            # prepared statements are parsed once per connection and reused
            assert pg.statements_parsed <= 2 * 8
        finally:
            await pg.stop()
    run(go())


def test_postgres_bad_password():
    async def go():
        pg = await FakePg(auth="scram").start()
        try:
            bad = pg.dsn.replace("s3cret", "nope")
            with pytest.raises(PgError) as ei:
                await PgConnection(bad).connect()
            assert ei.value.sqlstate == "28P01"
        finally:
            await pg.stop()
    run(go())


def test_postgres_bad_params_do_not_poison_the_statement():
    """Parameters that cannot be encoded fail that call only: the statement (first seen in that
    call) is parsed again by the next one instead of being bound to a name never sent."""
    class Unprintable:
        def __str__(self):
            raise ValueError("no text form")

    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            c = await PgConnection(pg.dsn).connect()
            with pytest.raises((TypeError, ValueError)):
                await c.execute("SELECT 2 + $1", 5)  # not a sequence
            with pytest.raises(ValueError):
                await c.execute("SELECT 3 + $1", (Unprintable(),))
            a = await c.execute("SELECT 2 + $1", (40,))
            b = await c.execute("SELECT 3 + $1", (39,))
            await c.close()
            return a, b
        finally:
            await pg.stop()
    a, b = run(go())
    assert a == ([(42,)], "SELECT 1") and b == ([(42,)], "SELECT 1")


def test_postgres_error_then_connection_still_usable():
    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            c = await PgConnection(pg.dsn).connect()
            with pytest.raises(PgError) as ei:
                await c.execute("this is a syntax error")
            assert ei.value.sqlstate == "42601"
            rows, tag = await c.execute("SELECT 1 + $1", (41,))
            assert rows == [(42,)] and tag == "SELECT 1"
            await c.close()
            with pytest.raises(PgProtocolError):
                await c.execute("SELECT 1")
        finally:
            await pg.stop()
    run(go())


def test_postgres_store_in_service():
    """The status handler's UPDATE + SELECT go over the wire (index.js:68,76)."""
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    from beholder_amd.topics import STATUS
    from beholder_amd.transport.memory import MemoryBroker
    from beholder_amd.utils.log import Logger, MemoryStream

    from helpers import cfg, status_msg

    async def go():
        pg = await FakePg().start()
        try:
            st = PostgresStore(pg.dsn, create_schema=True)
            await st.connect()
            await st.upsert(M1)
            b = MemoryBroker()
            http = RecordingHttpClient()
            svc = Service(cfg(), source=b.consumer(), store=st, http=http, logger=Logger(stream=MemoryStream()),
                          serve_metrics=False)
            await svc.init()
            b.publish(STATUS, status_msg("m1", "DEPLOYED"))
            b.finish()
            await svc.run()
            row = await st.get_by_id("m1")
            await svc.close()
            return row, http
        finally:
            await pg.stop()
    row, http = run(go())
    assert row.status == 4 and http.count == 3  # move + telegram + emby


# ------------------------------------------------- pipelining (store/pgwire.py) --

def test_pipelined_queries_share_one_connection():
    """Concurrent lookups (as many as prefetch allows, index.js:43) go out back to back on
    one connection and are answered in order."""
    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            st = PostgresStore(pg.dsn, create_schema=True, pool_size=1)
            await st.connect()
            for i in range(50):
                await st.upsert(Media(id=f"m{i}", name=f"Show {i}", creator=i % 2, status=i % 5))
            c = st._pool._conns[0]
            futs = [asyncio.ensure_future(st.get_by_id(f"m{i}")) for i in range(50)]
            await asyncio.sleep(0)
            peak = c.pending
            got = await asyncio.gather(*futs)
            assert [m.name for m in got] == [f"Show {i}" for i in range(50)]
            assert [m.status for m in got] == [i % 5 for i in range(50)]
            await st.close()
            return peak
        finally:
            await pg.stop()
    assert run(go()) == 50


def test_pipeline_error_isolated_to_its_query():
    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            c = await PgConnection(pg.dsn).connect()
            res = await asyncio.gather(c.execute("SELECT 1 + $1", (1,)), c.execute("this is a syntax error"),
                                       c.execute("SELECT 2 + $1", (2,)), return_exceptions=True)
            assert res[0] == ([(2,)], "SELECT 1") and res[2] == ([(4,)], "SELECT 1")
            assert isinstance(res[1], PgError) and res[1].sqlstate == "42601"
            assert "this is a syntax error" not in c._stmts  # failed Parse evicted from the cache
            assert await c.execute("SELECT 1 + $1", (9,)) == ([(10,)], "SELECT 1")  # cached statement reused
            await c.close()
            return pg.statements_parsed
        finally:
            await pg.stop()
    assert run(go()) == 2  # the two good statements; the bad one failed to parse


async def _dropping_server(after_bytes: int):
    """Accepts one connection, completes trust auth, reads `after_bytes` of queries, drops it."""
    import struct

    async def serve(r, w):
        n = struct.unpack("!I", await r.readexactly(4))[0]
        await r.readexactly(n - 4)
        w.write(b"R" + struct.pack("!II", 8, 0) + b"Z" + struct.pack("!I", 5) + b"I")
        await r.readexactly(after_bytes)
        w.transport.abort()
    srv = await asyncio.start_server(serve, "127.0.0.1", 0)
    return srv, srv.sockets[0].getsockname()[1]


def test_connection_loss_fails_every_pending_query():
    async def go():
        srv, port = await _dropping_server(10)
        try:
            c = await PgConnection(f"postgres://u@127.0.0.1:{port}/db").connect()
            futs = [c.execute("SELECT $1", (i,)) for i in range(5)]
            res = await asyncio.gather(*futs, return_exceptions=True)
            assert all(isinstance(e, PgProtocolError) for e in res)
            assert c.closed
            with pytest.raises(PgProtocolError):
                c.execute("SELECT 1")
        finally:
            srv.close()
    run(go())


def test_pool_spreads_load_and_replaces_broken_connections():
    from beholder_amd.store.pgwire import Pool

    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            pool = await Pool(pg.dsn, size=3, spread_at=2).open()
            assert pool.connections == 1
            # the pool grows in the background, one connection at a time, while bursts keep
            # every open connection at spread_at or more
            for _ in range(50):
                res = await asyncio.gather(*[pool.execute("SELECT $1 + 0", (i,)) for i in range(30)])
                assert [r[0][0][0] for r in res] == list(range(30))
                if pool.connections == 3:
                    break
                await asyncio.sleep(0.005)
            spread = pool.connections
            assert pool.grows == 2 and pool.grow_errors == 0
            pool._conns[0].abort()  # a broken connection is dropped and replaced
            await asyncio.sleep(0.01)
            res = await asyncio.gather(*[pool.execute("SELECT $1 + 0", (i,)) for i in range(10)])
            assert [r[0][0][0] for r in res] == list(range(10))
            await pool.close()
            return spread
        finally:
            await pg.stop()
    assert run(go()) == 3


def test_pool_grow_never_delays_a_query_and_backs_off_after_a_failure(monkeypatch):
    from beholder_amd.store import pgwire
    from beholder_amd.store.pgwire import Pool

    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            pool = await Pool(pg.dsn, size=4, spread_at=1).open()
            real = pgwire.PgConnection.connect
            gate = asyncio.Event()

            async def slow_connect(self):  # a grow whose connect takes as long as the test wants
                await gate.wait()
                return await real(self)
            monkeypatch.setattr(pgwire.PgConnection, "connect", slow_connect)
            res = await asyncio.wait_for(asyncio.gather(*[pool.execute("SELECT $1 + 0", (i,)) for i in range(20)]), 5)
            assert [r[0][0][0] for r in res] == list(range(20))  # served while the grow still waits
            assert pool.connections == 1 and pool._growing is not None
            gate.set()
            await asyncio.sleep(0.05)
            assert pool.connections == 2 and pool.grows == 1

            async def failing_connect(self):
                raise OSError("connection refused")
            monkeypatch.setattr(pgwire.PgConnection, "connect", failing_connect)
            await asyncio.gather(*[pool.execute("SELECT 1") for _ in range(10)])
            await asyncio.sleep(0.01)
            await asyncio.gather(*[pool.execute("SELECT 1") for _ in range(10)])
            await asyncio.sleep(0.01)
            errors = pool.grow_errors  # one failed attempt, then no retry inside GROW_RETRY_S
            monkeypatch.setattr(pgwire.PgConnection, "connect", real)
            await pool.close()
            return errors, pool.connections
        finally:
            await pg.stop()
    assert run(go()) == (1, 0)


def test_pool_close_cancels_a_grow_in_progress(monkeypatch):
    from beholder_amd.store import pgwire
    from beholder_amd.store.pgwire import Pool

    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            pool = await Pool(pg.dsn, size=2, spread_at=1).open()

            async def never(self):
                await asyncio.sleep(3600)
            monkeypatch.setattr(pgwire.PgConnection, "connect", never)
            await asyncio.gather(*[pool.execute("SELECT 1") for _ in range(4)])
            assert pool._growing is not None
            await asyncio.wait_for(pool.close(), 2)
            return pool._growing, pool.connections
        finally:
            await pg.stop()
    assert run(go()) == (None, 0)


def test_pg_reader_decoding_matches_python_reference():
    from beholder_amd.ops import native
    from beholder_amd.store.pgwire import DECODERS
    cases = [(16, b"t"), (16, b"f"), (20, b"-9223372036854775808"), (21, b"7"), (23, b"42"), (26, b"4294967295"),
             (700, b"1.5"), (701, b"-2.25e-10"), (701, b"Infinity"), (1700, b"12345678901234567890"),
             (1700, b"3.14"), (25, "héllo".encode()), (1043, b""), (114, b'{"a": 1}'), (17, b"\\x00ff10")]
    for oid, raw in cases:
        assert native.pg_decode_text(oid, raw) == DECODERS[oid](raw.decode()), (oid, raw)
    assert native.pg_decode_text(99999, b"unknown type") == "unknown type"


def test_pg_reader_split_feeding_and_malformed_input():
    import struct

    from beholder_amd.ops import PgReader

    def m(t, b):
        return t + struct.pack("!I", len(b) + 4) + b
    rd = struct.pack("!H", 1) + b"x\x00" + struct.pack("!IhIhih", 0, 0, 23, 4, -1, 0)
    stream = (m(b"1", b"") + m(b"2", b"") + m(b"T", rd) + m(b"D", struct.pack("!Hi", 1, 2) + b"42") +
              m(b"C", b"SELECT 1\x00") + m(b"Z", b"I")) * 3
    for step in (1, 5, 13, len(stream)):
        r = PgReader()
        r.query_mode = True
        out = []
        for i in range(0, len(stream), step):
            out += r.feed(stream[i:i + step])
        assert out == [([(42,)], "SELECT 1", None, True)] * 3 and r.buffered == 0
    r = PgReader()
    r.query_mode = True
    with pytest.raises(ValueError):
        r.feed(b"D" + struct.pack("!I", 2))  # length < 4
    with pytest.raises(ValueError):
        r.feed(m(b"D", struct.pack("!Hi", 1, 50) + b"short"))


def test_pg_reader_fuzz_never_crashes():
    from hypothesis import given, settings, strategies as st

    from beholder_amd.ops import PgReader

    @settings(max_examples=400, deadline=None)
    @given(st.lists(st.tuples(st.sampled_from(b"12TDCZENSnIA"), st.binary(max_size=40)), max_size=8),
           st.booleans())
    def check(msgs, query_mode):
        import struct
        r = PgReader(max_message=1 << 16)
        r.query_mode = query_mode
        data = b"".join(bytes([t]) + struct.pack("!I", len(b) + 4) + b for t, b in msgs)
        try:
            r.feed(data)
        except ValueError:
            pass
    check()


def test_pg_bind_matches_python_encoding():
    """The native Bind encoder (ops/csrc/py_pg.cpp) against encode_param, the Python reference."""
    import struct

    from hypothesis import given, settings, strategies as st

    from beholder_amd.ops import native
    from beholder_amd.store.pgwire import encode_param

    def ref(name, params):
        parts = [b"\x00", name, b"\x00\x00\x00", struct.pack("!H", len(params))]
        for v in params:
            e = encode_param(v)
            parts.append(struct.pack("!i", -1) if e is None else struct.pack("!i", len(e)) + e)
        parts.append(b"\x00\x00")
        b = b"".join(parts)
        return (b"B" + struct.pack("!I", len(b) + 4) + b + b"D" + struct.pack("!I", 6) + b"P\x00" +
                b"E" + struct.pack("!I", 9) + b"\x00" + struct.pack("!I", 0) + b"S" + struct.pack("!I", 4))

    value = st.one_of(st.none(), st.booleans(), st.integers(), st.floats(allow_nan=False), st.text(),
                      st.binary(max_size=20))

    @settings(max_examples=300, deadline=None)
    @given(st.binary(min_size=1, max_size=8).filter(lambda b: b"\x00" not in b), st.lists(value, max_size=12))
    def check(name, params):
        assert native.pg_bind(name, tuple(params)) == ref(name, params)
    check()


def test_postgres_tls_sslmodes(tmp_path):
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
    sctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    sctx.load_cert_chain(str(crt), str(key))

    async def go():
        tls = await FakePg(auth="scram", ssl_context=sctx).start()
        plain = await FakePg(auth="trust").start()
        try:
            base = tls.dsn.replace("127.0.0.1", "localhost")
            for mode in ("require", "prefer", f"verify-full&sslrootcert={crt}"):
                c = await PgConnection(f"{base}?sslmode={mode}").connect()
                assert c.tls and await c.execute("SELECT 1 + $1", (1,)) == ([(2,)], "SELECT 1")
                await c.close()
            with pytest.raises(ssl.SSLError):  # verify-full against an unknown CA
                await PgConnection(f"{base}?sslmode=verify-full").connect()
            c = await PgConnection(plain.dsn + "?sslmode=prefer").connect()  # server says 'N': plaintext
            assert not c.tls
            await c.close()
            with pytest.raises(PgProtocolError, match="does not support SSL"):
                await PgConnection(plain.dsn + "?sslmode=require").connect()
            with pytest.raises(PgProtocolError, match="invalid sslmode"):
                await PgConnection(plain.dsn + "?sslmode=bogus").connect()
            return tls.tls_sessions
        finally:
            await tls.stop()
            await plain.stop()
    assert run(go()) == 3  # the failed verification never completes a handshake


def test_service_survives_a_postgres_restart():
    """Connections dropped mid-stream (failover / restart): lookups in flight fail like any
    DB error (progress handlers warn and ack, Q7), the pool reconnects, and later events
    are handled normally again."""
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    from beholder_amd.topics import PROGRESS
    from beholder_amd.transport.memory import MemoryBroker
    from beholder_amd.utils.log import Logger, MemoryStream

    from helpers import cfg, progress_msg

    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            st = PostgresStore(pg.dsn, create_schema=True, pool_size=2)
            await st.connect()
            await st.upsert(M1)  # a Trello-created media: every progress event comments
            b = MemoryBroker()
            http = RecordingHttpClient()
            log = MemoryStream()
            svc = Service(cfg(), source=b.consumer(), store=st, http=http, logger=Logger(stream=log),
                          serve_metrics=False)
            await svc.init()
            run = asyncio.ensure_future(svc.run())
            for i in range(20):
                b.publish(PROGRESS, progress_msg("m1", "CONVERTING", i))
            while http.count < 20:
                await asyncio.sleep(0.005)
            dropped = pg.drop_connections()
            for i in range(20, 60):
                b.publish(PROGRESS, progress_msg("m1", "CONVERTING", i))
                await asyncio.sleep(0.002)
            b.finish()
            stats = await run
            await svc.close()
            return dropped, http.count, stats, log.records(), pg.connections
        finally:
            await pg.stop()
    dropped, comments, stats, records, conns = run(go())
    assert dropped >= 1 and conns > dropped  # reconnected after the drop
    assert stats["source"]["acked"] == 60  # Q7: progress always acks, even on DB errors
    failed = [r for r in records if r["msg"].startswith("failed to update media progress")]
    assert comments + len(failed) == 60 and comments >= 50, (comments, len(failed))


def test_compiled_handlers_pick_the_postgres_connection_in_c(monkeypatch):
    """The compiled handlers issue the stock store's queries through the native pick
    (ops pg_pool_execute, called directly): Pool.execute in Python runs only when the pick
    declines (pool growth). The results are those of the Python pick."""
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    from beholder_amd.store import pgwire
    from beholder_amd.topics import PROGRESS
    from beholder_amd.transport.memory import MemoryBroker
    from beholder_amd.utils.log import Logger, MemoryStream

    from helpers import cfg, progress_msg

    calls = []
    orig = pgwire.Pool.execute

    def counting(self, sql, params=()):
        calls.append(sql)
        return orig(self, sql, params)

    monkeypatch.setattr(pgwire.Pool, "execute", counting)

    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            st = PostgresStore(pg.dsn, create_schema=True, pool_size=1)
            await st.connect()
            await st.upsert(M1)
            calls.clear()
            b = MemoryBroker()
            http = RecordingHttpClient()
            svc = Service(cfg(), source=b.consumer(), store=st, http=http, logger=Logger(stream=MemoryStream()),
                          serve_metrics=False)
            await svc.init()
            run = asyncio.ensure_future(svc.run())
            for i in range(30):
                b.publish(PROGRESS, progress_msg("m1", "CONVERTING", i))
            b.finish()
            stats = await run
            await svc.close()
            return stats, http.count, svc.handler_impl
        finally:
            await pg.stop()
    stats, comments, impl = run(go())
    assert stats["source"]["acked"] == 30 and comments == 30
    assert type(impl).__name__ == "NativeHandlers"
    assert calls == []  # every lookup went through the direct native pick


def test_pool_metrics_render_postgres_connections_and_grows():
    from beholder_amd.metrics import parse_exposition
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    from beholder_amd.transport.memory import MemoryBroker
    from beholder_amd.utils.log import Logger, MemoryStream

    from helpers import cfg

    async def go():
        pg = await FakePg().start()
        try:
            st = PostgresStore(pg.dsn, create_schema=True, pool_size=2)
            svc = Service(cfg(), source=MemoryBroker().consumer(), store=st, http=RecordingHttpClient(),
                          logger=Logger(stream=MemoryStream()), serve_metrics=False)
            await svc.init()
            text = svc.registry.render()
            await svc.close()
            return parse_exposition(text)
        finally:
            await pg.stop()
    m = run(go())
    assert m['beholder_pool{pool="postgres",field="open"}'] == 2  # min_connections: the whole pool at startup
    assert m['beholder_pool{pool="postgres",field="grows"}'] == 0
    assert m['beholder_pool{pool="postgres",field="grow_errors"}'] == 0


def test_pool_regrows_after_a_connection_breaks():
    """A broken connection left in the pool's list does not count toward ``size``: the next
    burst that finds the open ones busy grows the pool back (native pick and Python path)."""
    from beholder_amd.store.pgwire import Pool

    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            pool = await Pool(pg.dsn, size=2, spread_at=1).open()
            for _ in range(50):
                await asyncio.gather(*[pool.execute("SELECT 1") for _ in range(4)])
                if pool.connections == 2:
                    break
                await asyncio.sleep(0.005)
            assert pool.connections == 2
            pool._conns[1].abort()
            await asyncio.sleep(0.01)
            assert pool.connections == 1
            for _ in range(50):
                res = await asyncio.gather(*[pool.execute("SELECT $1 + 0", (i,)) for i in range(4)])
                assert [r[0][0][0] for r in res] == list(range(4))
                if pool.connections == 2:
                    break
                await asyncio.sleep(0.005)
            n = pool.connections
            await pool.close()
            return n
        finally:
            await pg.stop()
    assert run(go()) == 2


def test_store_pool_knobs_reach_the_pool_and_are_validated():
    from beholder_amd.config import ConfigError
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    from beholder_amd.transport.memory import MemoryBroker
    from beholder_amd.utils.log import Logger, MemoryStream

    from helpers import cfg

    for bad in ({"spread_at": 0}, {"pool_size": "4"}, {"spread_at": True}):
        with pytest.raises(ConfigError, match="service.store"):
            cfg({"service": {"store": bad}})

    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            c = cfg({"service": {"store": {"dsn": pg.dsn, "pool_size": 3, "spread_at": 2}}})
            svc = Service(c, source=MemoryBroker().consumer(), http=RecordingHttpClient(),
                          logger=Logger(stream=MemoryStream()), serve_metrics=False)
            await svc.init()
            pool = svc.store._pool
            got = (pool.size, pool.spread_at)
            await svc.close()
            return got
        finally:
            await pg.stop()
    assert run(go()) == (3, 2)


@pytest.mark.parametrize("native_io", ["1", "0"])
def test_server_closing_right_after_startup_is_a_failed_connect(native_io, monkeypatch):
    """A server that closes the socket right behind its ReadyForQuery (a restart, a pooler
    recycling the backend): the connection is lost before connect() returns. connect() must fail
    (the pool then reconnects) instead of reporting an open connection whose queries are never
    answered (found by the chaos test: 100 handlers waiting on a dead asyncio-path connection)."""
    import struct

    monkeypatch.setenv("BEHOLDER_NATIVE_IO", native_io)

    async def serve(reader, writer):
        n = int.from_bytes(await reader.readexactly(4), "big")
        await reader.readexactly(n - 4)
        writer.write(b"R" + struct.pack("!II", 8, 0) + b"Z" + struct.pack("!I", 5) + b"I")
        await writer.drain()
        writer.close()

    async def go():
        srv = await asyncio.start_server(serve, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        try:
            c = PgConnection(f"postgres://u@127.0.0.1:{port}/db?sslmode=disable")
            try:
                await c.connect()
                await asyncio.sleep(0.05)
                try:  # if connect() won the race, the query must fail fast, never hang
                    await asyncio.wait_for(c.execute("SELECT 1"), 2)
                    return "answered"
                except (PgProtocolError, ConnectionError):
                    return "query failed"
            except PgProtocolError:
                return "connect failed"
        finally:
            srv.close()
    assert run(go()) in ("connect failed", "query failed")


@pytest.mark.parametrize("native_io", ["1", "0"])
def test_pool_drops_a_connection_whose_replies_stopped(native_io, monkeypatch):
    """A server that stops answering (a half-open TCP connection: the peer vanished without a
    FIN or RST) must not hold queries -- and the handlers awaiting them -- forever: after
    ``stall_timeout_s`` without a reply the pool drops the connection and the queries fail."""
    import struct

    from beholder_amd.store.pgwire import Pool

    monkeypatch.setenv("BEHOLDER_NATIVE_IO", native_io)

    async def serve(reader, writer):
        n = int.from_bytes(await reader.readexactly(4), "big")
        await reader.readexactly(n - 4)
        writer.write(b"R" + struct.pack("!II", 8, 0) + b"Z" + struct.pack("!I", 5) + b"I")
        await writer.drain()
        await reader.read()  # reads the queries, never answers

    async def go():
        srv = await asyncio.start_server(serve, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        try:
            pool = await Pool(f"postgres://u@127.0.0.1:{port}/db?sslmode=disable", size=1,
                              stall_timeout_s=0.3).open()
            t0 = asyncio.get_running_loop().time()
            with pytest.raises(PgProtocolError, match="no reply from Postgres for 0.3 s"):
                await asyncio.wait_for(pool.execute("SELECT 1"), 5)
            took = asyncio.get_running_loop().time() - t0
            stalls = pool.stalls
            await pool.close()
            return took, stalls
        finally:
            srv.close()
    took, stalls = run(go())
    assert stalls == 1 and 0.3 <= took < 1.5


def test_stall_timeout_config():
    from beholder_amd.config import ConfigError
    from helpers import cfg
    assert cfg().data["service"]["store"]["stall_timeout_s"] == 30.0
    cfg({"service": {"store": {"stall_timeout_s": None}}})  # off
    with pytest.raises(ConfigError, match="stall_timeout_s"):
        cfg({"service": {"store": {"stall_timeout_s": 0}}})


def test_pool_opens_min_connections_at_startup_and_tolerates_a_failed_extra():
    """``min_open``: open() makes that many connections together (the startup burst is spread at
    once). The first must succeed; a failed extra one is counted and left to the background grow."""
    from beholder_amd.store.pgwire import Pool, PgConnection

    async def go():
        pg = await FakePg().start()
        try:
            pool = await Pool(pg.dsn, size=4, min_open=3).open()
            assert pool.connections == 3 and pool.grow_errors == 0
            await pool.close()
            real, calls = PgConnection.connect, []

            async def flaky(self):
                calls.append(1)
                if len(calls) == 2:
                    raise OSError("refused")
                return await real(self)
            PgConnection.connect = flaky
            try:
                pool = await Pool(pg.dsn, size=4, min_open=3).open()
            finally:
                PgConnection.connect = real
            assert pool.connections == 2 and pool.grow_errors == 1
            rows, _ = await pool.execute("SELECT 1")
            await pool.close()
            st = PostgresStore(pg.dsn, pool_size=3)
            assert st.min_connections == 3
            assert PostgresStore(pg.dsn, pool_size=3, min_connections=1).min_connections == 1
        finally:
            await pg.stop()
    run(go())
