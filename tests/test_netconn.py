"""Native plain-TCP connections (ops/csrc/py_netconn.cpp, utils/netconn.py).

The H1 sink client and the Postgres client hand their plain-TCP sockets to a NetConn once
connected; tests/test_h1.py and tests/test_stores.py therefore exercise the native path. This
file adds what only the native path has (multi-recv replies, send backpressure, fd ownership),
and re-runs the network tests of both clients with BEHOLDER_NATIVE_IO=0, so the asyncio
transport path stays covered too.
"""
import asyncio
import inspect
import os
import socket

import pytest

import test_h1
import test_stores
import test_tls
from beholder_amd.ops import H1Parser, IOFuture
from beholder_amd.sinks import H1Client
from beholder_amd.store.pgwire import PgConnection
from beholder_amd.utils import netconn

from pg_fake import FakePg


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


def _no_arg_tests(mod, prefix):
    return [f for n, f in sorted(vars(mod).items())
            if n.startswith(prefix) and callable(f) and not inspect.signature(f).parameters]


ASYNCIO_PATH = ([f for f in _no_arg_tests(test_h1, "test_")
                 if "H1Client" in inspect.getsource(f) or "Scripted" in inspect.getsource(f)]
                + [f for f in _no_arg_tests(test_stores, "test_")
                   if any(k in inspect.getsource(f) for k in ("PgConnection", "PostgresStore", "Pool"))])


@pytest.mark.parametrize("fn", ASYNCIO_PATH, ids=[f"{f.__module__}.{f.__name__}" for f in ASYNCIO_PATH])
def test_asyncio_transport_path(fn, monkeypatch):
    monkeypatch.setenv("BEHOLDER_NATIVE_IO", "0")
    fn()


class _NoPollerLoop(asyncio.SelectorEventLoop):
    """A loop that cannot hold the NetPoller (as a loop type without an instance dict): each
    NetConn then registers its own socket with loop.add_reader / add_writer and runs its TLS
    handshake on the loop (py_netpoll.cpp netpoll_for, py_netconn.cpp tls_start)."""

    def __setattr__(self, name, value):
        if name == "_beholder_netpoller":
            raise AttributeError(name)
        super().__setattr__(name, value)


class _NoPollerPolicy(asyncio.DefaultEventLoopPolicy):
    def new_event_loop(self):
        return _NoPollerLoop()


# (the TLS tests of the handshake threads need a NetPoller to take the socket out of)
PER_SOCKET_PATH = ASYNCIO_PATH + [f for f in _no_arg_tests(test_tls, "test_")
                                  if "reactor" not in f.__name__ and "handshake_threads" not in f.__name__
                                  and "churn" not in f.__name__]


@pytest.mark.parametrize("fn", PER_SOCKET_PATH, ids=[f"{f.__module__}.{f.__name__}" for f in PER_SOCKET_PATH])
def test_per_socket_reader_path(fn):
    """The network tests of both clients and the TLS suite, on loops with no NetPoller."""
    if not netconn.enabled():
        pytest.skip("BEHOLDER_NATIVE_IO=0")
    old = asyncio.get_event_loop_policy()
    asyncio.set_event_loop_policy(_NoPollerPolicy())
    try:
        fn()
    finally:
        asyncio.set_event_loop_policy(old)


def test_per_socket_readers_register_each_socket_with_the_loop():
    """Without a NetPoller every NetConn's fd is in the loop's selector itself, and leaves it on close."""
    if not netconn.enabled():
        pytest.skip("BEHOLDER_NATIVE_IO=0")

    async def go():
        loop = asyncio.get_running_loop()
        s = await test_h1.Scripted(lambda n, m, t, h: test_h1.OK).start()
        try:
            c = H1Client(timeout_s=5)
            await asyncio.gather(*[c.request("GET", f"http://127.0.0.1:{s.port}/{i}") for i in range(3)])
            fds = {conn.net.fd for o in c._origins.values() for conn in o.idle}
            registered = set(loop._selector.get_map())
            out = (hasattr(loop, "_beholder_netpoller"), bool(fds) and fds <= registered)
            await c.close()
            return out + (bool(fds & set(loop._selector.get_map())),)
        finally:
            await s.stop()
    old = asyncio.get_event_loop_policy()
    asyncio.set_event_loop_policy(_NoPollerPolicy())
    try:
        assert run(go()) == (False, True, False)
    finally:
        asyncio.set_event_loop_policy(old)


def test_both_clients_adopt_plain_tcp_connections():
    async def go():
        s = await test_h1.Scripted(lambda n, m, t, h: test_h1.OK).start()
        pg = await FakePg(auth="md5").start()
        try:
            c = H1Client(timeout_s=5)
            await c.request("GET", f"http://127.0.0.1:{s.port}/x")
            conn = next(iter(c._origins.values())).idle[0]
            p = await PgConnection(pg.dsn).connect()
            rows, tag = await p.execute("SELECT $1 + 1", (1,))
            out = (type(conn.net).__name__, conn.transport, type(p._net).__name__, p._transport, rows, tag)
            await c.close()
            await p.close()
            assert p.closed and conn.net.closed
            return out
        finally:
            await s.stop()
            await pg.stop()
    assert run(go()) == ("NetConn", None, "NetConn", None, [(2,)], "SELECT 1")


def test_process_io_counts_follow_the_connections():
    """ops.io_counts(): the process-wide socket call counts (the bench's ``*_io_per_event``) move
    with each NetConn's own sends / receives, by kind."""
    from beholder_amd.ops import native

    async def go():
        s = await test_h1.Scripted(lambda n, m, t, h: test_h1.OK).start()
        pg = await FakePg(auth="md5").start()
        try:
            c0 = dict(native.io_counts())
            h = H1Client(timeout_s=5)
            for _ in range(3):
                await h.request("GET", f"http://127.0.0.1:{s.port}/x")
            p = await PgConnection(pg.dsn).connect()
            for i in range(2):
                await p.execute("SELECT $1 + 1", (i,))
            c1 = dict(native.io_counts())
            hs = next(iter(h._origins.values())).idle[0].net.stats
            ps = p._net.stats
            await h.close()
            await p.close()
            return c0, c1, hs, ps
        finally:
            await s.stop()
            await pg.stop()
    c0, c1, hs, ps = run(go())
    d = {k: c1[k] - c0[k] for k in c0}
    assert d["h1_sends"] == hs["sends"] >= 3 and d["h1_recvs"] == hs["recvs"] >= 3
    assert d["pg_sends"] >= 2 and d["pg_recvs"] >= 2 and ps["sends"] <= d["pg_sends"]
    assert d["poll_runs"] >= 5 and d["poll_ready"] >= d["poll_runs"]


def test_large_response_spans_many_recvs():
    body = os.urandom(3 << 20).hex().encode()  # 6 MiB: 24+ reads of 256 KiB

    def respond(n, m, t, h):
        return b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(body) + body

    async def go():
        s = await test_h1.Scripted(respond).start()
        c = H1Client(timeout_s=10)
        try:
            r1 = await c.request("GET", f"http://127.0.0.1:{s.port}/a")
            r2 = await c.request("GET", f"http://127.0.0.1:{s.port}/b")  # same connection, reused
            conn = next(iter(c._origins.values())).idle[0]
            return r1.body == body and r2.body == body, conn.net.stats, s.connections
        finally:
            await c.close()
            await s.stop()
    ok, stats, conns = run(go())
    assert ok and conns == 1 and stats["recvs"] > 24 and stats["bytes_in"] > 2 * len(body)


def test_write_backpressure_keeps_order():
    """A peer that reads slowly: what the kernel refuses is queued and sent from the writer
    callback, in order, and the fd is unregistered at close."""
    payload = bytes(range(256)) * (64 << 10)  # 16 MiB

    async def go():
        loop = asyncio.get_running_loop()
        a, b = socket.socketpair()
        a.setblocking(False)
        b.setblocking(False)
        fd = os.dup(a.fileno())
        a.close()
        lost = []

        class Owner:
            def _net_lost(self, exc):
                lost.append(exc)

        nc = netconn.NetConn(fd, loop, "h1", Owner(), H1Parser())
        nc.write(payload[: len(payload) // 2])
        nc.write(payload[len(payload) // 2:])
        assert nc.buffered > 0  # the socket buffer cannot hold 16 MiB
        got = bytearray()
        while len(got) < len(payload):
            await asyncio.sleep(0.001)
            try:
                got += b.recv(1 << 20)
            except BlockingIOError:
                pass
        assert nc.buffered == 0
        nc.close()
        b.close()
        return bytes(got) == payload, nc.fd, nc.closed, lost
    ok, fd, closed, lost = run(go())
    assert ok and fd == -1 and closed and lost == []


def test_peer_close_reports_loss_and_fails_the_waiter():
    async def go():
        loop = asyncio.get_running_loop()
        a, b = socket.socketpair()
        lost = []

        class Owner:
            def _net_lost(self, exc):
                lost.append(exc)
                w = nc.take_waiter()
                if w is not None:
                    w.set_exception(ConnectionResetError("peer closed"))

        fd = os.dup(a.fileno())
        a.close()
        os.set_blocking(fd, False)
        nc = netconn.NetConn(fd, loop, "h1", Owner(), H1Parser())
        w = IOFuture(loop)
        nc.request(b"GET / HTTP/1.1\r\n\r\n", w, False)
        assert b.recv(100).startswith(b"GET /")
        b.close()
        with pytest.raises(ConnectionResetError):
            await w
        with pytest.raises(ConnectionError):
            nc.write(b"x")
        return lost, nc.closed
    lost, closed = run(go())
    assert lost == [None] and closed


def test_bad_arguments():
    async def go():
        loop = asyncio.get_running_loop()
        with pytest.raises(ValueError):
            netconn.NetConn(0, loop, "smtp", object(), H1Parser())
        with pytest.raises(TypeError):
            netconn.NetConn(0, loop, "pg", object(), H1Parser())  # no stmts / pg_error
        with pytest.raises(ValueError):
            netconn.NetConn(-1, loop, "h1", object(), H1Parser())
    run(go())


def test_disabled_by_env(monkeypatch):
    monkeypatch.setenv("BEHOLDER_NATIVE_IO", "0")

    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            p = await PgConnection(pg.dsn).connect()
            r = await p.execute("SELECT 1")
            kind = p._net
            await p.close()
            return kind, r
        finally:
            await pg.stop()
    assert run(go()) == (None, ([(1,)], "SELECT 1"))


def test_native_pool_pick_matches_python_pick(monkeypatch):
    """store/pgwire.py Pool.execute: the native pick (ops pg_pool_execute) sends each query to the
    same connection the Python loop would (fewest in flight, first on ties, grow only when every
    open one has spread_at or more) and the answers are the same."""
    from beholder_amd.store import pgwire

    async def one(native_pick):
        pg = await FakePg(auth="md5").start()
        try:
            pool = pgwire.Pool(pg.dsn, size=3, spread_at=4)
            pool.native_pick = pgwire._native.pg_pool_execute if native_pick else None
            await pool.open()
            seq, futs = [], []
            for wave in range(3):
                for i in range(10):
                    futs.append(pool.execute("SELECT $1 * 2", (wave * 10 + i,)))
                    seq.append(tuple(c.pending for c in pool._conns))
                await asyncio.sleep(0)
            res = await asyncio.gather(*futs)
            kinds = {type(f).__name__ for f in futs}
            await pool.close()
            return seq, [r[0] for r in res], len(pool._conns), kinds
        finally:
            await pg.stop()

    nat = run(one(True))
    py = run(one(False))
    assert nat[1] == py[1] == [[(2 * i,)] for i in range(30)]
    assert nat[0] == py[0]
    assert nat[2] == py[2]
    assert "IOFuture" in nat[3]


def test_native_connect_refused_localhost_and_ready_future():
    """ops netconn_connect: the TCP connect made in C (sinks/h1.py _connect_native). A refused
    connect rejects the ready future with ECONNREFUSED (Node's message via _connect_error); a
    name tries every resolved address in order (localhost: ::1 then 127.0.0.1 against a server
    on 127.0.0.1 only); the connection in the pool is a NetConn with no asyncio transport."""
    import errno as _errno

    from beholder_amd.ops import native
    from beholder_amd.sinks import HttpError

    async def go():
        loop = asyncio.get_running_loop()
        probe = socket.socket()
        probe.bind(("127.0.0.1", 0))
        dead_port = probe.getsockname()[1]
        probe.close()  # nothing listens there now
        net = native.netconn_connect("127.0.0.1", dead_port, loop, "h1", None, H1Parser())
        try:
            await net.handshake
            refused = None
        except OSError as e:
            refused = e.errno
        s = await test_h1.Scripted(lambda n, m, t, h: test_h1.OK).start()
        try:
            c = H1Client(timeout_s=5)
            r = await c.request("GET", f"http://localhost:{s.port}/x")
            conn = next(iter(c._origins.values())).idle[0]
            kinds = (type(conn.net).__name__, conn.transport, conn.net.tls)
            with pytest.raises(HttpError, match=f"^connect ECONNREFUSED 127.0.0.1:{dead_port}$"):
                await c.request("GET", f"http://127.0.0.1:{dead_port}/x")
            await c.close()
            return refused, r.status, kinds
        finally:
            await s.stop()
    refused, status, kinds = run(go())
    assert refused == _errno.ECONNREFUSED
    assert status == 200 and kinds == ("NetConn", None, None)


def test_native_connect_ipv6_literal():
    """An IPv6 literal origin (``http://[::1]:port``) connects natively over AF_INET6."""
    async def go():
        async def serve(r, w):
            await r.readuntil(b"\r\n\r\n")
            w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nv6")
            await w.drain()
            w.close()
        try:
            srv = await asyncio.start_server(serve, "::1", 0)
        except OSError:
            return None
        port = srv.sockets[0].getsockname()[1]
        c = H1Client(timeout_s=5)
        try:
            r = await c.request("GET", f"http://[::1]:{port}/x")
            return r.status, r.body
        finally:
            await c.close()
            srv.close()
    res = run(go())
    if res is None:
        pytest.skip("no IPv6 loopback")
    assert res == (200, b"v6")


def test_native_io_off_still_works():
    """BEHOLDER_NATIVE_IO=0 (the one native-I/O switch; replies on plain asyncio futures, read at
    import) leaves working clients: the H1 and TLS suites pass with it."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-x",
                        "tests/test_h1.py", "tests/test_tls.py"], cwd=root, capture_output=True, text=True,
                       env=dict(os.environ, BEHOLDER_NATIVE_IO="0"), timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


def test_netconns_share_one_epoll_set_per_loop():
    """ops/csrc/py_netpoll.cpp: every NetConn of a loop sits in one epoll set whose fd is the only
    one registered with the loop; it is closed (and leaves the loop) with its last socket."""
    if not netconn.enabled():
        pytest.skip("BEHOLDER_NATIVE_IO=0")

    async def go():
        loop = asyncio.get_running_loop()
        s = await test_h1.Scripted(lambda n, m, t, h: test_h1.OK).start()
        pg = await FakePg(auth="md5").start()
        try:
            c = H1Client(timeout_s=5)
            await asyncio.gather(*[c.request("GET", f"http://127.0.0.1:{s.port}/{i}") for i in range(5)])
            p = await PgConnection(pg.dsn).connect()
            poller = loop._beholder_netpoller
            sizes = [poller.size]
            client_fds = {conn.net.fd for o in c._origins.values() for conn in o.idle} | {p._net.fd}
            registered = set(loop._selector.get_map())
            readers = (poller.fd in registered, bool(client_fds & registered))
            await p.close()
            sizes.append(poller.size)
            await c.close()
            sizes.append(poller.size)
            return sizes, poller.fd, hasattr(loop, "_beholder_netpoller"), readers
        finally:
            await s.stop()
            await pg.stop()
    sizes, fd, attached, readers = run(go())
    assert sizes == [6, 5, 0] and fd == -1 and not attached
    assert readers == (True, False)  # the loop watches the epoll fd, not the client sockets


def test_failed_flush_scheduling_forgets_the_new_statement():
    """when execute() cannot schedule its flush (loop.call_soon raises), the queued
    Parse is dropped, and so is the statement name: the next execute of that SQL parses it again
    instead of binding a name the server never saw."""
    if not netconn.enabled():
        pytest.skip("BEHOLDER_NATIVE_IO=0")

    async def go():
        loop = asyncio.get_running_loop()
        pg = await FakePg(auth="trust").start()
        try:
            p = await PgConnection(pg.dsn).connect()
            assert p._net is not None

            def refuse(*a, **k):
                raise RuntimeError("loop refuses callbacks")
            loop.call_soon = refuse
            try:
                with pytest.raises(RuntimeError, match="refuses"):
                    p.execute("SELECT 5 + $1", (1,))
            finally:
                del loop.call_soon
            r = await p.execute("SELECT 5 + $1", (37,))
            await p.close()
            return r
        finally:
            await pg.stop()
    assert run(go()) == ([(42,)], "SELECT 1")


def test_scoped_ipv6_address_and_bad_port_are_http_errors_or_work():
    """getaddrinfo can return a scoped IPv6 address ("fe80::1%eth0") that the native
    connect (inet_pton) cannot parse: it connects through asyncio instead; an address that fails
    to connect is an HttpError, never a raw ValueError. A port outside 1-65535 is an invalid URI."""
    from beholder_amd.sinks import HttpError

    async def go():
        loop = asyncio.get_running_loop()

        async def serve(r, w):
            await r.readuntil(b"\r\n\r\n")
            w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nv6")
            await w.drain()
            w.close()
        try:
            srv = await asyncio.start_server(serve, "::1", 0)
        except OSError:
            return None
        port = srv.sockets[0].getsockname()[1]
        real = loop.getaddrinfo

        async def scoped(host, *a, **k):
            if host == "scoped.test":
                return [(socket.AF_INET6, socket.SOCK_STREAM, 6, "", ("::1", port, 0, 1))]  # scope id 1
            if host == "deadscope.test":
                return [(socket.AF_INET6, socket.SOCK_STREAM, 6, "", ("fe80::dead", port, 0, 1))]
            return await real(host, *a, **k)
        loop.getaddrinfo = scoped
        c = H1Client(timeout_s=2)
        try:
            r = await c.request("GET", f"http://scoped.test:{port}/x")
            out = [(r.status, r.body)]
            for url in (f"http://deadscope.test:{port}/x", "http://127.0.0.1:70000/x"):
                try:
                    await c.request("GET", url)
                    out.append("no error")
                except HttpError as e:
                    out.append(type(e).__name__ + ": " + str(e).split(" ")[0])
            return out
        finally:
            del loop.getaddrinfo
            await c.close()
            srv.close()
    res = run(go())
    if res is None:
        pytest.skip("no IPv6 loopback")
    assert res[0] == (200, b"v6")
    assert res[1].startswith("HttpError") and res[2] == "HttpError: Invalid"
