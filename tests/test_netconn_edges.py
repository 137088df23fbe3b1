"""NetConn (ops/csrc/py_netconn.cpp) on a socket pair: the paths a real peer rarely takes.

The H1 sink client and the Postgres pool drive NetConns against well-behaved servers (test_h1*,
test_stores, test_netconn). Here the peer is the other end of a socketpair, written byte by byte
by the test, so each odd case is exact: a response nobody asked for, a malformed one, a
ReadyForQuery with no query outstanding, a parser that is a Python object (fed through its
``feed`` / ``start`` methods), queries queued when the connection closes, and every argument
check of the constructor, ``netconn_connect`` and ``pg_pool_execute``. The owner's callbacks
(``_net_error`` / ``_net_lost`` / ``_net_message``) must report exactly what happened.
"""
import asyncio
import os
import socket

import pytest

from beholder_amd.ops import H1Parser, IOFuture, PgReader, native
from beholder_amd.utils import netconn

pytestmark = pytest.mark.skipif(not netconn.enabled(), reason="BEHOLDER_NATIVE_IO=0")

OK = b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\n{}"


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 20))


class Owner:
    def __init__(self):
        self.errors, self.lost, self.messages = [], [], []

    def _net_error(self, exc):
        self.errors.append(exc)

    def _net_lost(self, exc):
        self.lost.append(exc)

    def _net_message(self, typ, body):
        self.messages.append((typ, bytes(body)))


class PyH1Parser:
    """The stock parser behind Python methods: the NetConn feeds it a memoryview per read."""

    def __init__(self):
        self.p = H1Parser()
        self.fed = 0

    def start(self, head=False):
        self.p.start(head=head)

    def feed(self, data):
        self.fed += 1
        return self.p.feed(bytes(data))


class PgError(Exception):
    pass


def _pair():
    a, b = socket.socketpair()
    fd = os.dup(a.fileno())
    a.close()
    os.set_blocking(fd, False)
    b.setblocking(False)
    return fd, b


async def _read(sock, n=65536):
    loop = asyncio.get_running_loop()
    return await loop.sock_recv(sock, n)


async def _until(pred, t=2.0):
    for _ in range(int(t / 0.005)):
        if pred():
            return True
        await asyncio.sleep(0.005)
    return pred()


def test_h1_reply_through_a_python_parser():
    async def go():
        fd, peer = _pair()
        owner, parser = Owner(), PyH1Parser()
        c = native.NetConn(fd, asyncio.get_running_loop(), "h1", owner, parser)
        w = IOFuture(asyncio.get_running_loop())
        assert not c.waiting
        c.request(b"GET /x HTTP/1.1\r\nHost: h\r\n\r\n", w, False)
        assert c.waiting
        req = await _read(peer)
        peer.send(OK)
        status, reason, raw, body, keep = await w
        c.close()
        peer.close()
        return req, status, body, keep, parser.fed > 0, owner.errors
    req, status, body, keep, fed, errors = run(go())
    assert req.startswith(b"GET /x HTTP/1.1") and status == 200 and body == b"{}" and keep and fed
    assert errors == []


def test_h1_unsolicited_and_malformed_responses_are_reported():
    async def go():
        loop = asyncio.get_running_loop()
        fd, peer = _pair()
        owner = Owner()
        c = native.NetConn(fd, loop, "h1", owner, H1Parser())
        w = IOFuture(loop)
        c.request(b"GET / HTTP/1.1\r\n\r\n", w, False)
        await _read(peer)
        assert c.take_waiter() is w and not c.waiting  # the request given up (an owner's timeout)
        peer.send(OK)  # its reply now answers nothing
        await _until(lambda: owner.errors)
        unsolicited = list(owner.errors)
        c.abort()
        peer.close()
        fd, peer = _pair()
        owner2 = Owner()
        c2 = native.NetConn(fd, loop, "h1", owner2, H1Parser())
        c2.request(b"GET / HTTP/1.1\r\n\r\n", IOFuture(loop), False)
        await _read(peer)
        peer.send(b"NOT HTTP AT ALL\r\n\r\n")
        await _until(lambda: owner2.errors)
        c2.abort()
        peer.close()
        return unsolicited, owner2.errors
    unsolicited, malformed = run(go())
    assert unsolicited == [None]
    assert len(malformed) == 1 and isinstance(malformed[0], Exception)


def test_h1_peer_closing_is_a_loss():
    async def go():
        loop = asyncio.get_running_loop()
        fd, peer = _pair()
        owner = Owner()
        c = native.NetConn(fd, loop, "h1", owner, H1Parser())
        w = IOFuture(loop)
        c.request(b"GET / HTTP/1.1\r\n\r\n", w, False)
        await _read(peer)
        peer.close()
        await _until(lambda: owner.lost)
        took = c.take_waiter()
        return owner.lost, took is w, c.closed
    lost, took, closed = run(go())
    assert len(lost) == 1 and took and closed


def _rfq() -> bytes:
    return b"Z\x00\x00\x00\x05I"


def test_pg_replies_notices_and_a_ready_for_query_nobody_waits_for():
    async def go():
        loop = asyncio.get_running_loop()
        fd, peer = _pair()
        owner = Owner()
        reader = PgReader()
        assert reader.query_mode is False  # startup / authentication: raw messages
        reader.query_mode = True
        c = native.NetConn(fd, loop, "pg", owner, reader, stmts={}, pg_error=PgError)
        f = c.execute("SELECT 1", ())
        assert c.pending == 1
        sent = await _read(peer)  # Parse, Bind, Execute, Sync
        notice = b"N" + (4 + 6).to_bytes(4, "big") + b"Mhi\x00\x00\x00"
        complete = b"C" + (4 + 9).to_bytes(4, "big") + b"SELECT 1\x00"
        peer.send(notice + b"1\x00\x00\x00\x04" + b"2\x00\x00\x00\x04" + b"n\x00\x00\x00\x04" + complete
                  + _rfq())
        rows, tag = await f
        peer.send(_rfq())  # nothing outstanding
        await _until(lambda: owner.errors)
        c.abort()
        peer.close()
        return sent[:1], rows, tag, owner.messages, owner.errors
    first, rows, tag, messages, errors = run(go())
    assert first == b"P" and rows == [] and tag == "SELECT 1"
    assert messages and messages[0][0] in (b"N", "N")
    assert errors == [None]


def test_pg_queries_queued_at_close_are_dropped():
    """execute() queues the query for the loop's flush; close() in the same iteration sends what is
    queued (best effort); the outstanding futures stay for the owner, whose fail_all() rejects them."""
    async def go():
        loop = asyncio.get_running_loop()
        fd, peer = _pair()
        c = native.NetConn(fd, loop, "pg", Owner(), PgReader(), stmts={}, pg_error=PgError)
        futs = [c.execute("SELECT $1::int", (i,)) for i in range(3)]
        c.close()
        got = await _read(peer)
        peer.close()
        queued = c.pending
        c.fail_all(PgError("connection closed"))  # what the owner does on a loss
        errs = [type(e).__name__ for e in await asyncio.gather(*futs, return_exceptions=True)]
        return c.closed, queued, c.pending, got.count(b"P"), errs
    closed, queued, pending, parses, errs = run(go())
    assert closed and queued == 3 and pending == 0 and parses >= 1 and errs == ["PgError"] * 3


def test_wrong_kind_calls_and_closed_calls_raise():
    async def go():
        loop = asyncio.get_running_loop()
        fd, peer = _pair()
        h = native.NetConn(fd, loop, "h1", Owner(), H1Parser())
        fd2, peer2 = _pair()
        p = native.NetConn(fd2, loop, "pg", Owner(), PgReader(), stmts={}, pg_error=PgError)
        out = []
        for call in (lambda: h.execute("SELECT 1"), lambda: p.request(b"x", IOFuture(loop), False),
                     lambda: h.request(b"x", IOFuture(loop))):
            with pytest.raises(TypeError) as e:
                call()
            out.append(str(e.value))
        h.close()
        p.close()
        with pytest.raises(ConnectionError, match="closed"):
            h.request(b"x", IOFuture(loop), False)
        with pytest.raises(ConnectionError, match="closed"):
            p.execute("SELECT 1")
        peer.close()
        peer2.close()
        return out
    out = run(go())
    assert "on a pg NetConn" in out[0] and "on an h1 NetConn" in out[1] and "on an h1 NetConn" in out[2]


def test_constructor_checks_its_arguments():
    async def go():
        loop = asyncio.get_running_loop()
        fd, peer = _pair()
        cases = [
            (dict(tls=object(), server_hostname="h"), TypeError, "TlsContext"),
            (dict(closed_exc=42), TypeError, "exception class"),
            (dict(kind="smtp"), ValueError, "kind must be"),
            (dict(kind="pg"), TypeError, "needs stmts"),
            (dict(fd=-1), ValueError, "invalid fd"),
        ]
        for over, exc, match in cases:
            kw = dict(fd=fd, loop=loop, kind="h1", owner=Owner(), parser=H1Parser())
            kw.update(over)
            with pytest.raises(exc, match=match):
                native.NetConn(**kw)
        c = native.NetConn(fd, loop, "h1", Owner(), H1Parser())
        with pytest.raises(RuntimeError, match="already initialised"):
            c.__init__(fd, loop, "h1", Owner(), H1Parser())
        c.close()
        peer.close()
    run(go())


def test_netconn_connect_checks_its_arguments():
    async def go():
        loop = asyncio.get_running_loop()
        with pytest.raises(ValueError, match="not an IP address"):
            native.netconn_connect("example.com", 80, loop, "h1", Owner(), H1Parser())
        for port in (0, 70000):
            with pytest.raises(ValueError, match="bad port"):
                native.netconn_connect("127.0.0.1", port, loop, "h1", Owner(), H1Parser())
        srv = socket.socket()
        srv.bind(("127.0.0.1", 0))
        srv.listen()
        port = srv.getsockname()[1]
        before = len(os.listdir("/proc/self/fd"))
        with pytest.raises(ValueError, match="kind must be"):  # refused after the socket was made: closed again
            native.netconn_connect("127.0.0.1", port, loop, "smtp", Owner(), H1Parser())
        after = len(os.listdir("/proc/self/fd"))
        srv.close()
        return before, after
    before, after = run(go())
    assert after <= before


def test_pg_pool_execute_checks_its_arguments():
    with pytest.raises(TypeError, match="pg_pool_execute"):
        native.pg_pool_execute([], "SELECT 1")
    with pytest.raises(TypeError, match="list of NetConn or None"):
        native.pg_pool_execute((1,), "SELECT 1", (), 1, 1)
    assert native.pg_pool_execute(None, "SELECT 1", (), 1, 1) is None  # the Python path


def test_pg_malformed_reply_and_ownerless_notices():
    """A Postgres reply the reader cannot parse is reported to the owner as a protocol error;
    with no owner, notices are dropped quietly."""
    async def go():
        loop = asyncio.get_running_loop()
        fd, peer = _pair()
        owner = Owner()
        r = PgReader()
        r.query_mode = True
        c = native.NetConn(fd, loop, "pg", owner, r, stmts={}, pg_error=PgError)
        c.execute("SELECT 1")
        await _read(peer)
        peer.send(b"C\x00\x00\x00\x02")  # a length below the header's own 4 bytes
        await _until(lambda: owner.errors)
        c.abort()
        peer.close()
        fd, peer = _pair()
        r2 = PgReader()
        r2.query_mode = True
        c2 = native.NetConn(fd, loop, "pg", None, r2, stmts={}, pg_error=PgError)
        peer.send(b"N" + (4 + 6).to_bytes(4, "big") + b"Mhi\x00\x00\x00")
        await asyncio.sleep(0.05)
        open_after_notice = not c2.closed
        c2.close()
        peer.close()
        return owner.errors, open_after_notice
    errors, still_open = run(go())
    assert len(errors) == 1 and isinstance(errors[0], Exception) and still_open


def test_an_owner_callback_that_raises_is_reported_not_raised():
    """The owner's _net_* callbacks run from the loop's read callback: an exception there goes to
    sys.unraisablehook, and the NetConn carries on (here: it is closed as the peer went away)."""
    import sys
    seen = []
    old = sys.unraisablehook
    sys.unraisablehook = lambda u: seen.append(type(u.exc_value).__name__)

    class Bad(Owner):
        def _net_lost(self, exc):
            raise LookupError("owner failed")

    async def go():
        loop = asyncio.get_running_loop()
        fd, peer = _pair()
        c = native.NetConn(fd, loop, "h1", Bad(), H1Parser())
        peer.close()
        await _until(lambda: c.closed)
        return c.closed
    try:
        assert run(go())
    finally:
        sys.unraisablehook = old
    assert "LookupError" in seen


def test_writing_to_a_peer_that_is_gone_is_a_loss():
    async def go():
        loop = asyncio.get_running_loop()
        fd, peer = _pair()
        owner = Owner()
        c = native.NetConn(fd, loop, "h1", owner, H1Parser())
        peer.close()
        try:
            for _ in range(4):
                c.write(b"x" * 65536)
                await asyncio.sleep(0.01)
        except ConnectionError:
            pass
        await _until(lambda: owner.lost or c.closed)
        return bool(owner.lost) or c.closed
    assert run(go())


def test_constructor_rejects_wrong_argument_types():
    async def go():
        with pytest.raises(TypeError):
            native.NetConn("not an fd", asyncio.get_running_loop(), "h1", Owner(), H1Parser())
    run(go())
