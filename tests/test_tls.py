"""Native TLS (`ops/csrc/py_tls.cpp` TlsContext, the TLS mode of `ops/csrc/py_netconn.cpp`
NetConn) for the HTTPS sinks (`sinks/h1.py` `_connect`) and for Postgres sslmodes
(`store/pgwire.py` `_negotiate_tls`). Trello and Telegram are HTTPS in production
(index.js:53,83,99); with H1Client's own SSL context (the default one or ``ssl_cafile``) the
handshake and the record layer run in C on the socket. Every behaviour is checked against the
asyncio TLS path (``BEHOLDER_NATIVE_IO=0``)."""
import asyncio
import os
import shutil
import ssl
import subprocess

import pytest

from beholder_amd.bench.http_sink_server import TLS_CERT, server_ssl_context
from beholder_amd.sinks import H1Client, HttpError


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


class TlsServer:
    """HTTPS keep-alive server; ``respond(target) -> bytes | None`` (None: close the connection
    cleanly after reading the request); "hang" never answers."""

    def __init__(self, respond, ctx=None, handshake=True):
        self.respond = respond
        self.ctx = ctx or server_ssl_context()
        self.handshake = handshake
        self.connections = 0
        self.requests = []

    async def start(self):
        self.server = await asyncio.start_server(self._serve, "127.0.0.1", 0,
                                                 ssl=self.ctx if self.handshake else None)
        self.port = self.server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        self.server.close()
        await self.server.wait_closed()

    async def _serve(self, r, w):
        self.connections += 1
        try:
            if not self.handshake:  # accept TCP, never answer the ClientHello
                await asyncio.sleep(3600)
            while True:
                try:
                    head = await r.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, ConnectionError, ssl.SSLError):
                    return
                self.requests.append(head)
                out = self.respond(head.split(b" ", 2)[1].decode())
                if out == "hang":
                    await asyncio.sleep(3600)
                if out is None:
                    return
                w.write(out)
                await w.drain()
        finally:
            w.close()


requires_native_tls = pytest.mark.skipif(os.environ.get("BEHOLDER_NATIVE_IO", "1") == "0",
                                         reason="inspects native TLS state; BEHOLDER_NATIVE_IO=0")


def ok(body=b"{}"):
    return b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(body) + body


def native_tls(c):
    return [conn.net.tls for o in c._origins.values() for conn in o.idle if conn.net is not None]


def test_native_tls_requests_take_the_fast_path():
    if not H1Client().native_call:
        pytest.skip("native I/O switched off (BEHOLDER_NATIVE_IO=0)")

    async def go():
        s = await TlsServer(lambda t: ok()).start()
        c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
        url = f"https://127.0.0.1:{s.port}/1/cards/abc/actions/comments"
        first = await c.request("POST", url, params={"text": "hi ü", "key": "k"})
        aw = c.request("POST", url, params={"text": "again"})
        second = await aw
        kind = "H1Call" if aw.native else "python"
        tls = native_tls(c)
        st = dict(c.counts)
        await c.close()
        await s.stop()
        return first.status, second.status, kind, tls, st, s.connections, s.requests[0].split(b"\r\n")[0]
    a, b, kind, tls, st, conns, line = run(go())
    assert (a, b, kind, conns) == (200, 200, "H1Call", 1)
    assert tls == ["TLSv1.3"] and st["reused"] == 1
    assert line == b"POST /1/cards/abc/actions/comments?text=hi%20%C3%BC&key=k HTTP/1.1"


def _both(fn):
    """fn(native: bool) run with native I/O (native TLS connections) and with asyncio's TLS
    (``BEHOLDER_NATIVE_IO=0``, read per connection); returns both results."""
    out = {}
    for native in (True, False):
        old = os.environ.get("BEHOLDER_NATIVE_IO")
        os.environ["BEHOLDER_NATIVE_IO"] = "1" if native else "0"
        try:
            out[native] = run(fn(native))
        finally:
            if old is None:
                os.environ.pop("BEHOLDER_NATIVE_IO", None)
            else:
                os.environ["BEHOLDER_NATIVE_IO"] = old
    return out[True], out[False]


def test_large_bodies_and_many_requests_match_asyncio_tls():
    big = os.urandom(700_000).hex().encode()  # 1.4 MB: ~90 TLS records, many reads

    async def go(native):
        s = await TlsServer(lambda t: ok(big if t.startswith("/big") else t.encode())).start()
        c = H1Client(timeout_s=10, ssl_cafile=TLS_CERT)
        base = f"https://127.0.0.1:{s.port}"
        rs = await asyncio.gather(*[c.request("GET", f"{base}/p{i}", params={"i": i}) for i in range(60)])
        b = await c.request("GET", base + "/big")
        kinds = native_tls(c)
        await c.close()
        await s.stop()
        return [(r.status, r.body) for r in rs], b.body == big, bool(kinds) and all(kinds)
    nat, py = _both(go)
    assert nat[0] == py[0] and nat[1] and py[1]
    assert nat[2] is True and py[2] is False  # native connections only with the native path


class DribbleServer(TlsServer):
    """Answers in one-byte TLS records (one write + drain per byte) after reading the request
    head slowly; the request targets may be far larger than a socket buffer."""

    async def _serve(self, r, w):
        self.connections += 1
        try:
            while True:
                try:
                    head = await r.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, asyncio.LimitOverrunError, ConnectionError, ssl.SSLError):
                    return
                self.requests.append(len(head))
                target = head.split(b" ", 2)[1]
                body = b"%d:%s" % (len(target), target[-16:])
                for i, ch in enumerate(ok(body)):
                    w.write(bytes([ch]))
                    if i % 7 == 0:
                        await w.drain()
                        await asyncio.sleep(0)
                await w.drain()
        finally:
            w.close()


def test_one_byte_records_and_requests_larger_than_the_socket_buffer():
    """Replies split into one-byte records, and request heads of several MB (partial TLS writes
    that wait for the socket to drain), on the native path and on asyncio's: same results."""
    async def go(native):
        s = DribbleServer(None)
        s.server = await asyncio.start_server(s._serve, "127.0.0.1", 0, ssl=s.ctx, limit=16 * 1024 * 1024)
        s.port = s.server.sockets[0].getsockname()[1]
        c = H1Client(timeout_s=20, ssl_cafile=TLS_CERT)
        base = f"https://127.0.0.1:{s.port}"
        out = []
        for i in range(6):
            params = {"i": i, "text": ("x%d" % i) * (2_200_000 if i % 3 == 2 else 10)}
            r = await c.request("POST", f"{base}/c{i}", params=params)
            out.append((r.status, r.body))
        kinds = native_tls(c)
        st = dict(c.counts)
        await c.close()
        await s.stop()
        return out, bool(kinds) and all(kinds), st["connections"], s.requests
    nat, py = _both(go)
    assert nat[0] == py[0] and nat[3] == py[3]
    assert max(nat[3]) > 4_000_000 and nat[2] == py[2] == 1
    assert nat[1] is True and py[1] is False


def test_verification_failures_match_asyncio_tls(tmp_path):
    if shutil.which("openssl") is None:
        pytest.skip("needs openssl")
    key, crt = tmp_path / "k.pem", tmp_path / "c.pem"
    r = subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1",
                        "-nodes", "-keyout", str(key), "-out", str(crt), "-days", "1", "-subj", "/CN=other.example",
                        "-addext", "subjectAltName=DNS:other.example"], capture_output=True)
    assert r.returncode == 0, r.stderr
    wrong_name = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    wrong_name.load_cert_chain(str(crt), str(key))

    async def go(native):
        errs = []
        for ctx, cafile in ((None, None), (wrong_name, str(crt))):
            s = await TlsServer(lambda t: ok(), ctx=ctx).start()
            c = H1Client(timeout_s=5, ssl_cafile=cafile)  # no cafile: default trust, self-signed refused
            try:
                await c.request("GET", f"https://127.0.0.1:{s.port}/x")
                errs.append("no error")
            except HttpError as e:
                errs.append(str(e))
            await c.close()
            await s.stop()
        return errs
    nat, py = _both(go)
    assert nat == py == ["CERTIFICATE_VERIFY_FAILED", "CERTIFICATE_VERIFY_FAILED"]


def test_plain_http_server_and_handshake_timeout():
    async def plain(native):
        s = await TlsServer(lambda t: ok(), handshake=True).start()
        s.server.close()
        await s.server.wait_closed()
        srv = await asyncio.start_server(lambda r, w: w.write(b"HTTP/1.1 400 Bad\r\n\r\n"), "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
        try:
            await c.request("GET", f"https://127.0.0.1:{port}/x")
            err = "no error"
        except HttpError as e:
            err = str(e)
        await c.close()
        srv.close()
        await srv.wait_closed()
        return err
    nat, py = _both(plain)
    assert nat == py and nat in ("WRONG_VERSION_NUMBER", "RECORD_LAYER_FAILURE", "PACKET_LENGTH_TOO_LONG")

    async def silent():
        s = await TlsServer(lambda t: ok(), handshake=False).start()
        c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
        with pytest.raises(HttpError, match=r"^ETIMEDOUT: GET https://127\.0\.0\.1:\d+/x$"):
            await c.request("GET", f"https://127.0.0.1:{s.port}/x", timeout=0.3)
        await asyncio.sleep(0.1)  # the queue's background connect shares the request's deadline
        open_ = sum(o.open for o in c._origins.values())
        await c.close()
        s.server.close()
        return open_
    assert run(silent()) == 0


@requires_native_tls
def test_server_close_then_reconnect_resumes_the_session():
    async def go():
        n = {"i": 0}

        def respond(t):
            n["i"] += 1
            return ok() if n["i"] % 2 else None  # every second request: the server closes instead
        s = await TlsServer(respond).start()
        c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
        url = f"https://127.0.0.1:{s.port}/x"
        statuses = []
        for _ in range(6):
            statuses.append((await c.request("GET", url)).status)  # GET: retried on a fresh connection
            await asyncio.sleep(0.01)
        stats = c._native_tls().stats
        st = dict(c.counts)
        cs = c.stats()
        assert (cs["tls_handshakes"], cs["tls_resumed"]) == (stats["handshakes"], stats["resumed"])
        await c.close()
        await s.stop()
        return statuses, stats, st, s.connections
    statuses, stats, st, conns = run(go())
    assert statuses == [200] * 6 and st["retries"] >= 4
    assert stats["handshakes"] == conns and stats["resumed"] >= conns - 2  # tickets reused on reconnect


@requires_native_tls
def test_tls12_server_and_caller_context_keeps_asyncio_path():
    ctx12 = server_ssl_context()
    ctx12.maximum_version = ssl.TLSVersion.TLSv1_2

    async def go():
        s = await TlsServer(lambda t: ok(), ctx=ctx12).start()
        c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
        r = await c.request("GET", f"https://127.0.0.1:{s.port}/x")
        tls = native_tls(c)
        await c.close()
        own = H1Client(timeout_s=5, ssl_context=ssl.create_default_context(cafile=TLS_CERT))
        r2 = await own.request("GET", f"https://127.0.0.1:{s.port}/y")
        own_native = native_tls(own)
        await own.close()
        await s.stop()
        return r.status, tls, r2.status, own_native
    assert run(go()) == (200, ["TLSv1.2"], 200, [])


def test_postgres_sslmodes_on_native_tls():
    """store/pgwire.py: after the SSLRequest's 'S' the socket goes to a TLS NetConn; startup,
    authentication (SCRAM) and the pipelined queries run over it. sslmode require / verify-ca /
    verify-full behave as libpq (and as the asyncio path)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pg_fake import FakePg

    from beholder_amd.store.pgwire import PgConnection, Pool

    async def go(native):
        srv = await FakePg(auth="scram", ssl_context=server_ssl_context()).start()
        out = []
        try:
            for mode in ("require", f"verify-ca&sslrootcert={TLS_CERT}", f"verify-full&sslrootcert={TLS_CERT}"):
                c = await PgConnection(f"{srv.dsn}?sslmode={mode}").connect()
                rows = await asyncio.gather(*[c.execute("SELECT $1 + 1", (i,)) for i in range(50)])
                out.append((mode.split("&")[0], c.tls, c._net.tls if c._net is not None else None,
                            [r[0][0][0] for r in rows][:3]))
                await c.close()
            for mode in ("verify-full", "verify-ca"):  # unknown CA: refused before any query
                try:
                    await PgConnection(f"{srv.dsn}?sslmode={mode}").connect()
                    out.append("no error")
                except ssl.SSLError as e:
                    out.append(e.reason)
            pool = await Pool(f"{srv.dsn}?sslmode=verify-full&sslrootcert={TLS_CERT}", size=2).open()
            res = await asyncio.gather(*[pool.execute("SELECT $1 * 3", (i,)) for i in range(40)])
            out.append([r[0][0][0] for r in res][-1])
            await pool.close()
            return out, srv.tls_sessions
        finally:
            await srv.stop()
    nat, py = _both(go)
    assert [o if not isinstance(o, tuple) else (o[0], o[1], o[3]) for o in nat[0]] == \
           [o if not isinstance(o, tuple) else (o[0], o[1], o[3]) for o in py[0]]
    assert [o[2] for o in nat[0][:3]] == ["TLSv1.3"] * 3 and [o[2] for o in py[0][:3]] == [None] * 3
    assert nat[0][3:5] == ["CERTIFICATE_VERIFY_FAILED"] * 2 and nat[0][5] == 117
    assert nat[1] == py[1]


@requires_native_tls
def test_tls13_tickets_are_single_use_and_a_reconnect_burst_resumes():
    """Each TLS 1.3 ticket resumes one connection (RFC 8446 C.4); the origin's newest tickets
    (servers send two per connection) let several concurrent reconnects resume."""
    async def go():
        s = await TlsServer(lambda t: ok()).start()
        c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
        url = f"https://127.0.0.1:{s.port}/x"
        await c.request("GET", url)
        await asyncio.sleep(0.02)  # the tickets arrive after the handshake
        t = c._native_tls()
        cached0 = t.stats["cached_sessions"]
        for o in c._origins.values():
            while o.idle:
                c._drop(o.idle.pop())
        await asyncio.gather(*[c.request("GET", url) for _ in range(cached0)])
        for _ in range(200):  # a background connect may finish after the burst was served
            if not c._dials:
                break
            await asyncio.sleep(0.005)
        st = t.stats
        await c.close()
        await s.stop()
        return cached0, st
    cached0, st = run(go())
    assert cached0 >= 2
    assert st["handshakes"] == 1 + cached0 and st["resumed"] == cached0


def test_garbage_on_an_established_tls_connection():
    """Bytes that are not TLS records on an established connection (a broken middlebox): the
    connection is failed, the idempotent request is retried once on a fresh connection (as on
    the asyncio path), a POST fails with an error, and the pool keeps working."""
    state = {"n": 0}

    class Broken(TlsServer):
        async def _serve(self, r, w):
            self.connections += 1
            try:
                while True:
                    try:
                        await r.readuntil(b"\r\n\r\n")
                    except (asyncio.IncompleteReadError, ConnectionError, ssl.SSLError):
                        return
                    state["n"] += 1
                    if state["n"] in (2, 4):  # raw bytes under the TLS layer instead of a record
                        os.write(w.transport.get_extra_info("socket").fileno(), b"\x17\x03\x03\x00\x05junk!" * 3)
                        await asyncio.sleep(0.05)
                        w.transport.abort()
                        return
                    w.write(ok())
                    await w.drain()
            finally:
                w.close()

    async def go(native):
        state["n"] = 0
        s = await Broken(None).start()
        c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
        url = f"https://127.0.0.1:{s.port}/x"
        out = [(await c.request("GET", url)).status]
        out.append((await c.request("GET", url)).status)  # 2nd answered with junk: retried
        try:
            await c.request("POST", url)  # 4th answered with junk: not replayed
            out.append("no error")
        except HttpError:
            out.append("error")
        out.append((await c.request("GET", url)).status)
        st = dict(c.counts)
        await c.close()
        await s.stop()
        return out, st["retries"], st["errors"]
    nat, py = _both(go)
    assert nat == py and nat[0] == [200, 200, "error", 200] and nat[1] == 1 and nat[2] == 1


@pytest.mark.parametrize("max_connecting", [1, 8])
def test_first_burst_admits_at_most_max_connecting_handshakes(max_connecting):
    """100 concurrent first requests to one HTTPS origin (prefetch 100 deliveries at start):
    never more than ``max_connecting`` connects + TLS handshakes in flight; queued requests take
    the first connection that frees up or the next connect slot, and all 100 succeed."""
    async def go():
        s = await TlsServer(lambda t: ok()).start()
        c = H1Client(timeout_s=10, ssl_cafile=TLS_CERT, max_connecting=max_connecting)
        url = f"https://127.0.0.1:{s.port}/x"
        inflight = {"now": 0, "peak": 0}
        real = c._dial

        async def counted(o, deadline, infos=None):
            inflight["now"] += 1
            inflight["peak"] = max(inflight["peak"], inflight["now"])
            try:
                return await real(o, deadline, infos)
            finally:
                inflight["now"] -= 1
        c._dial = counted
        rs = await asyncio.gather(*[c.request("GET", url) for _ in range(100)])
        for _ in range(400):  # background connects may finish after the burst was served
            if not c._dials:
                break
            await asyncio.sleep(0.005)
        st = c.stats()
        await c.close()
        await s.stop()
        return rs, st, inflight["peak"], s.connections
    rs, st, peak, server_conns = run(go())
    assert all(r.status == 200 for r in rs)
    assert peak <= max_connecting and st["connecting_peak"] <= max_connecting
    assert st["connections"] == server_conns < 100 and st["connect_waits"] > 0
    assert st["reused"] >= 100 - st["connections"]


def test_pool_still_grows_past_max_connecting_under_slow_responses():
    """Admission caps connects in flight, not the pool: with slow responses every request needs
    its own connection, and the pool grows to serve them (8 at a time)."""
    async def go():
        s = await TlsServer(lambda t: ok()).start()
        real_serve = s._serve

        async def slow_serve(r, w):
            await asyncio.sleep(0.05)
            await real_serve(r, w)
        s.server.close()
        await s.server.wait_closed()
        s.server = await asyncio.start_server(slow_serve, "127.0.0.1", s.port, ssl=s.ctx)
        c = H1Client(timeout_s=10, ssl_cafile=TLS_CERT, max_connecting=4)
        url = f"https://127.0.0.1:{s.port}/x"
        rs = await asyncio.gather(*[c.request("GET", url) for _ in range(32)])
        st = c.stats()
        await c.close()
        await s.stop()
        return rs, st
    rs, st = run(go())
    assert all(r.status == 200 for r in rs)
    assert st["connecting_peak"] <= 4 and st["connections"] > 4


@requires_native_tls
def test_handshakes_run_on_handshake_threads_and_abort_cleanly():
    """The client half of each TLS handshake runs on a handshake thread (py_netconn.cpp), not on
    the event loop: every handshake of a burst is counted as offloaded. Connections closed while
    their handshake is still on a thread (a server that never answers) release their socket."""
    import gc

    import psutil

    def client_sockets(port):  # this process's sockets connected TO `port` (not the server's own)
        return sum(1 for k in psutil.Process().net_connections(kind="tcp") if k.raddr and k.raddr.port == port)

    async def go():
        s = await TlsServer(lambda t: ok()).start()
        silent = await TlsServer(lambda t: ok(), handshake=False).start()
        c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
        url = f"https://127.0.0.1:{s.port}/x"
        rs = await asyncio.gather(*[c.request("GET", url) for _ in range(40)])
        for _ in range(200):
            if not c._dials:
                break
            await asyncio.sleep(0.005)
        st = dict(c._native_tls().stats)
        await c.close()
        for _ in range(3):  # handshakes that never finish, abandoned by the client
            c2 = H1Client(timeout_s=0.2, ssl_cafile=TLS_CERT)
            res = await asyncio.gather(*[c2.request("GET", f"https://127.0.0.1:{silent.port}/y") for _ in range(8)],
                                       return_exceptions=True)
            assert all(isinstance(x, HttpError) for x in res)
            await c2.close()
        for _ in range(100):  # the threads notice the shutdown and close the sockets
            gc.collect()
            if client_sockets(silent.port) == 0:
                break
            await asyncio.sleep(0.01)
        left = client_sockets(silent.port)
        await s.stop()
        silent.server.close()
        return rs, st, left
    rs, st, left = run(go())
    assert all(r.status == 200 for r in rs)
    assert st["handshakes"] >= 2 and st["offloaded"] == st["handshakes"]
    assert left == 0


def test_first_tls_context_starts_warm_handshake_threads_and_a_warm_up_handshake():
    """Making the first TlsContext starts the handshake threads (each runs one in-memory warm-up
    handshake before taking jobs) and runs the process's one-time warm-up handshake, so the
    first burst of connects pays neither. Fresh process: the pool is process-wide."""
    import sys
    code = (
        "import os, time\n"
        "from beholder_amd.ops import _native\n"
        "before = len(os.listdir('/proc/self/task'))\n"
        f"ctx = _native.TlsContext(cafile={TLS_CERT!r})\n"
        "time.sleep(0.3)\n"
        "after = len(os.listdir('/proc/self/task'))\n"
        f"_native.TlsContext(cafile={TLS_CERT!r})\n"
        "again = len(os.listdir('/proc/self/task'))\n"
        "want = max(1, min(4, os.cpu_count() // 4))\n"
        "print(before, after, again, want)\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr
    before, after, again, want = map(int, out.stdout.split())
    assert after - before == want and again == after  # one pool per process


def test_tls_connection_churn_leaks_no_descriptors_or_threads():
    """Many clients each open a burst of HTTPS connections (handshakes on the handshake threads,
    completions through the poller's channel), use them and close; servers that drop the
    connection (``once``, after a reply, when the client asks) add closes on both sides. Afterwards this process holds the same descriptors
    and threads as after the first round: nothing accumulates per connection."""
    import psutil

    def fds():  # this process's descriptors, less the test servers' own accepted sockets
        server_side = sum(1 for k in psutil.Process().net_connections(kind="tcp")
                          if k.laddr and k.laddr.port in ports and k.raddr)
        return len(os.listdir("/proc/self/fd")) - server_side

    ports = set()

    def tasks():
        return len(os.listdir("/proc/self/task"))

    async def go():
        keep = await TlsServer(lambda t: ok()).start()
        once = await TlsServer(lambda t: ok(b"{}") if not t.endswith("/bye") else None).start()
        ports.update((keep.port, once.port))

        async def cycle():
            c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
            urls = [f"https://127.0.0.1:{keep.port}/a", f"https://127.0.0.1:{once.port}/b"]
            rs = await asyncio.gather(*[c.request("GET", urls[i % 2]) for i in range(24)])
            for _ in range(200):
                if not c._dials:
                    break
                await asyncio.sleep(0.005)
            await c.close()
            return all(r.status == 200 for r in rs)

        assert await cycle()
        await asyncio.sleep(0.05)
        base_fds, base_tasks = fds(), tasks()
        for _ in range(15):
            assert await cycle()
        for _ in range(100):
            await asyncio.sleep(0.01)
            if fds() <= base_fds:
                break
        out = fds(), tasks(), base_fds, base_tasks
        await keep.stop()
        await once.stop()
        return out
    now_fds, now_tasks, base_fds, base_tasks = run(go())
    assert now_fds <= base_fds + 2, (now_fds, base_fds)
    assert now_tasks == base_tasks, (now_tasks, base_tasks)


def test_https_by_host_name_verifies_the_name_and_shares_the_lookup():
    """An HTTPS sink addressed by name (as api.trello.com is): the name is resolved once for the
    burst, sent as SNI and checked against the certificate (the bench certificate names
    localhost); a name the certificate does not carry fails verification."""
    async def go():
        s = await TlsServer(lambda t: ok()).start()
        loop = asyncio.get_running_loop()
        real, calls = loop.getaddrinfo, []

        async def lookup(host, port, **kw):
            calls.append(host)
            return await real("127.0.0.1", port, **kw)
        loop.getaddrinfo = lookup
        try:
            c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
            rs = await asyncio.gather(*[c.request("GET", f"https://localhost:{s.port}/x") for _ in range(20)])
            good = ([r.status for r in rs], len(calls), dict(c.counts)["connections"])
            await c.close()
            c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
            try:
                await c.request("GET", f"https://not-the-name.invalid:{s.port}/x")
                bad = "ok"
            except HttpError as e:
                bad = str(e)
            await c.close()
        finally:
            loop.getaddrinfo = real
            await s.stop()
        return good, bad
    (statuses, lookups, conns), bad = run(go())
    assert statuses == [200] * 20 and conns >= 2
    from beholder_amd.utils import netconn
    if netconn.enabled():
        assert lookups == 1
    assert "CERTIFICATE_VERIFY_FAILED" in bad or "certificate" in bad.lower()


def test_closing_a_connection_whose_handshake_just_finished_reports_nothing():
    """A connection closed right after its handshake finished on a thread (the completion queued,
    not yet taken by the loop), while it is the poller's last socket: closing the poller drains
    the completion channel, and that drain must see the connection as gone (it used to treat it
    as a fresh success and fail re-arming a socket that had left the epoll set, reported as an
    unraisable FileNotFoundError). Many bursts whose clients close at once make the window
    likely; nothing may be reported."""
    import sys
    seen = []
    hook, sys.unraisablehook = sys.unraisablehook, seen.append

    async def go():
        s = await TlsServer(lambda t: ok()).start()
        try:
            for _ in range(60):
                c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)
                rs = await asyncio.gather(*[c.request("GET", f"https://127.0.0.1:{s.port}/x") for _ in range(20)])
                assert all(r.status == 200 for r in rs)
                await c.close()  # background connects still finishing their handshakes
            await asyncio.sleep(0.05)
        finally:
            await s.stop()
    try:
        run(go())
    finally:
        sys.unraisablehook = hook
    assert [f"{u.exc_type.__name__}: {u.exc_value}" for u in seen] == []


@requires_native_tls
def test_handshakes_waiting_for_slow_peers_do_not_hold_the_handshake_threads():
    """The handshake threads only run the CPU steps (hs_reactor.hpp): a handshake waiting for its
    peer holds no thread. 16 connects to a peer that answers each ClientHello 0.3 s late all
    finish in about 0.3 s; with the threads blocked in poll(2) through the wait (the earlier
    design, 4 threads) they took four rounds, about 1.2 s."""
    delay, n = 0.3, 16

    async def go():
        s = await TlsServer(lambda t: ok()).start()

        async def pipe(src, dst, first_delay=0.0):
            try:
                while True:
                    data = await src.read(65536)
                    if not data:
                        break
                    if first_delay:
                        await asyncio.sleep(first_delay)
                        first_delay = 0.0
                    dst.write(data)
                    await dst.drain()
            except ConnectionError:
                pass
            finally:
                dst.close()

        async def slow(r, w):  # delays the server's first flight by `delay`, then relays
            ur, uw = await asyncio.open_connection("127.0.0.1", s.port)
            await asyncio.gather(pipe(r, uw), pipe(ur, w, delay))

        proxy = await asyncio.start_server(slow, "127.0.0.1", 0)
        port = proxy.sockets[0].getsockname()[1]
        c = H1Client(timeout_s=10, ssl_cafile=TLS_CERT, max_per_host=n)
        url = f"https://127.0.0.1:{port}/x"
        before = dict(c._native_tls().stats)
        t0 = asyncio.get_running_loop().time()
        opened, err = await c.preconnect(url, n)
        took = asyncio.get_running_loop().time() - t0
        after = dict(c._native_tls().stats)
        r = await c.request("GET", url)
        await c.close()
        proxy.close()
        await s.stop()
        return opened, err, took, after["offloaded"] - before["offloaded"], r.status
    opened, err, took, offloaded, status = run(go())
    assert err is None and opened == n and status == 200
    assert offloaded == n
    assert delay <= took < 2 * delay + 0.15, took


def test_peer_reset_during_offloaded_handshakes_fails_them_promptly():
    """A peer that resets the connection right after the ClientHello, while the handshake runs on
    a handshake thread (the loop's poller has the socket paused with EPOLLONESHOT, so the reset's
    EPOLLHUP wakes the loop at most once): every request fails with a connection error,
    quickly, and no socket is left behind."""
    import socket
    import struct

    import psutil

    async def go():
        async def rst(r, w):
            await r.read(1)  # the ClientHello has arrived
            so = w.get_extra_info("socket")
            so.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
            w.transport.abort()  # RST

        srv = await asyncio.start_server(rst, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT, max_per_host=16, max_connecting=16)
        t0 = asyncio.get_running_loop().time()
        res = await asyncio.gather(*[c.request("GET", f"https://127.0.0.1:{port}/x") for _ in range(16)],
                                   return_exceptions=True)
        took = asyncio.get_running_loop().time() - t0
        await c.close()
        srv.close()
        await asyncio.sleep(0.05)
        left = sum(1 for k in psutil.Process().net_connections(kind="tcp") if k.raddr and k.raddr.port == port)
        return res, took, left
    res, took, left = run(go())
    assert all(isinstance(x, HttpError) for x in res), res
    assert took < 2.0 and left == 0


def test_tls_after_fork_starts_fresh_handshake_threads(tmp_path):
    """A process that forks after its TLS handshakes ran on the handshake threads (the supervisor's
    workers are spawned, but a library user may fork): the child has none of those threads, so the
    atfork handler drops the reactor (py_netconn.cpp hs_after_fork_child) and the child's first
    handshake starts new ones. Both processes complete their HTTPS requests."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "fork_tls.py"
    script.write_text(
        "import asyncio, os, sys\n"
        f"sys.path[:0] = [{root!r}, {os.path.join(root, 'tests')!r}]\n"
        "from test_tls import TlsServer, ok, TLS_CERT\n"
        "from beholder_amd.sinks import H1Client\n"
        "async def once():\n"
        "    srv = await TlsServer(lambda t: ok()).start()\n"
        "    c = H1Client(timeout_s=5, ssl_cafile=TLS_CERT)\n"
        "    rs = await asyncio.gather(*[c.request('GET', f'https://127.0.0.1:{srv.port}/a') for _ in range(4)])\n"
        "    await c.close()\n"
        "    await srv.stop()\n"
        "    return all(r.status == 200 for r in rs)\n"
        "assert asyncio.run(once())\n"
        "pid = os.fork()\n"
        "if pid == 0:\n"
        "    sys.exit(0 if asyncio.run(once()) else 3)\n"
        "_, st = os.waitpid(pid, 0)\n"
        "sys.exit(os.waitstatus_to_exitcode(st) or (0 if asyncio.run(once()) else 4))\n")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
