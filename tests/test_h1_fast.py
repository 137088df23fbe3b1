"""Native fast path of the keep-alive sink client (`ops/csrc/py_h1call.cpp` `h1_fast`, used by
`sinks/h1.py` `H1Client.request` on a warm pool): the bytes on the wire, the responses, the
pool accounting and every rare path (reset + retry, redirect, timeout, cancellation, abandon)
must be those of the Python request loop (index.js:53,83,99,112 go through this client)."""
import asyncio
import random

import pytest

from beholder_amd.ops import native
from beholder_amd.sinks import H1Client, HttpError
from beholder_amd.sinks import h1 as h1mod

pytestmark = pytest.mark.skipif(h1mod._NATIVE_CALL is None or not H1Client().native_call,
                                reason="native I/O switched off (BEHOLDER_NATIVE_IO=0)")


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


class Raw:
    """HTTP/1.1 server that records every request's exact bytes; ``respond(target) -> bytes | None``
    (None: drop the connection without answering; "hang": never answer)."""

    def __init__(self, respond):
        self.respond = respond
        self.raw = []
        self.connections = 0
        self._tasks = set()

    async def start(self):
        self.server = await asyncio.start_server(self._serve, "127.0.0.1", 0)
        self.port = self.server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        self.server.close()
        await self.server.wait_closed()
        # Python 3.10's Server.close leaves connection handlers running ("hang" ones sleep on):
        # end them while the loop is still open
        for t in list(self._tasks):
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)

    async def _serve(self, r, w):
        self.connections += 1
        me = asyncio.current_task()
        self._tasks.add(me)
        try:
            while True:
                try:
                    head = await r.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, ConnectionError):
                    return
                self.raw.append(head)
                target = head.split(b" ", 2)[1].decode("latin-1")
                out = self.respond(target)
                if out == "hang":
                    await asyncio.sleep(3600)
                if out is None:
                    w.transport.abort()
                    return
                w.write(out)
                await w.drain()
        finally:
            self._tasks.discard(me)
            w.close()


OK = b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\nX-A: 1\r\n\r\n{}"


def _cases(port, n=150, seed=7):
    rnd = random.Random(seed)
    base = [f"http://127.0.0.1:{port}", f"http://u%40s:p%3Aw@127.0.0.1:{port}"]
    paths = ["/1/cards/abc/actions/comments", "/bot123:XYZ/sendMessage?chat_id=5&text=a%20b", "/emby/library/refresh",
             "", "/x y", "/é", "/a#frag", "?q=1", "/p?x=1", "/1/cards/C\r\nX-Evil:1/actions/comments",
             # the shape check reads 8 bytes at a time: odd bytes past the first words
             "/1/cards/abcdefghij/x y", "/1/cards/abcdefghij#frag", "/1/cards/abcdefghij\x7fz",
             "/1/cards/abcdefghij?q=1", "/1/cards/abcdefghijklmnopqrstu/actions"]
    params = [None, {}, {"key": "k", "token": "t", "text": "DEPLOYED: **5%** (_x_) ü"}, {"a": None, "b": 1},
              {"pos": 2, "idList": "L1"}, {"api_key": "x y&z"}, {"v": 1.5, "w": True}]
    for _ in range(n):
        yield (rnd.choice(["GET", "POST", "PUT", "get", "DELETE", "HEAD"]), rnd.choice(base) + rnd.choice(paths),
               rnd.choice(params))


async def _drive(port, fast: bool):
    """Every case on one client, each after a warm-up request so a keep-alive connection is idle."""
    c = H1Client(timeout_s=5)
    if not fast:
        c.native_call = None
    out, kinds = [], []
    for m, url, params in _cases(port):
        try:
            await c.request("GET", f"http://127.0.0.1:{port}/warm")
            await c.request("GET", url.split("?")[0].split("#")[0] or url, params=None)
        except HttpError:
            pass
        aw = c.request(m, url, params=params)
        try:
            r = await aw
            out.append((r.status, r.body, r.headers, r.url))
        except HttpError as e:
            out.append(("error", str(e)))
        kinds.append("native" if getattr(aw, "native", False) else "python")
    counts = dict(c.counts)
    await c.close()
    return out, kinds, counts


def test_fast_path_sends_the_same_bytes_and_returns_the_same_responses():
    async def go():
        res = {}
        for fast in (True, False):
            s = await Raw(lambda t: OK).start()
            out, kinds, counts = await _drive(s.port, fast)
            raw = [r.replace(str(s.port).encode(), b"PORT") for r in s.raw]
            res[fast] = ([tuple(str(x).replace(str(s.port), "PORT") for x in o) for o in out], kinds, counts, raw,
                         s.connections)
            await s.stop()
        return res
    res = run(go())
    f_out, f_kinds, f_counts, f_raw, f_conns = res[True]
    p_out, p_kinds, p_counts, p_raw, p_conns = res[False]
    assert f_raw == p_raw  # byte for byte, request line, Host, Authorization, User-Agent, Content-Length
    assert f_out == p_out
    assert f_counts == p_counts and f_conns == p_conns
    assert "native" in f_kinds and "native" not in p_kinds
    # the shapes the sinks produce take the native path; the others decline before any state changes
    assert f_kinds.count("native") > len(f_kinds) // 4


def test_fast_path_declines_cold_pool_and_foreign_shapes():
    async def go():
        s = await Raw(lambda t: OK).start()
        c = H1Client(timeout_s=5)
        url = f"http://127.0.0.1:{s.port}/a"
        first = c.request("GET", url)
        assert first.native is None  # nothing happens before the first await, as for a coroutine
        await first
        kinds = [first.native]
        for args in (("GET", url), ("get", url), ("GET", url + "#f"), ("GET", url + "/é"), ("POST", url + "?a=1"),
                     ("GET", f"http://127.0.0.1:{s.port + 1 if s.port < 65535 else 1}/b")):
            aw = c.request(*args, params={"k": 1} if args[0] == "POST" else None)
            try:
                await aw
            except HttpError:
                pass
            kinds.append(aw.native)
        await c.close()
        await s.stop()
        return kinds
    kinds = run(go())
    assert kinds[0] is False  # no idle connection yet
    assert kinds[1] is True
    assert kinds[2:] == [False] * 5


def test_fast_path_declines_foreign_argument_types():
    """Arguments outside the sinks' shapes (a Mapping that is not a dict, a non-ASCII host, a
    bytes method) are the Python path's: same results and errors, no native read of them."""
    import types

    async def one(fast):
        s = await Raw(lambda t: OK).start()
        c = H1Client(timeout_s=5)
        if not fast:
            c.native_call = None
        base = f"http://127.0.0.1:{s.port}"
        seen = []
        for m, url, params in [("POST", base + "/a", types.MappingProxyType({"k": "v w"})),
                               ("POST", base + "/b", [("x", 1)]),
                               ("GET", "http://café.invalid/x", None),
                               (b"GET", base + "/c", None),
                               ("GET", base + "/d", {"ok": 1})]:
            await c.request("GET", base + "/warm")
            aw = c.request(m, url, params=params)
            try:
                r = await aw
                seen.append((r.status, r.url.replace(base, "")))
            except Exception as e:  # noqa: BLE001 — the exact outcome is compared
                seen.append((type(e).__name__, str(e).replace(base, "")))
            seen.append(getattr(aw, "native", None) is True)
        await c.close()
        await s.stop()
        return seen, [r.split(b"\r\n")[0] for r in s.raw]

    async def go():
        return await one(True), await one(False)
    (fast, fraw), (slow, sraw) = run(go())
    assert [x for x in fast if not isinstance(x, bool)] == [x for x in slow if not isinstance(x, bool)]
    assert fraw == sraw
    assert fast[1::2] == [False, False, False, False, True]  # only the dict-shaped request is native


def test_fast_path_reset_retry_redirect_and_errors_match_python():
    def respond(t):
        if t.startswith("/old"):
            return b"HTTP/1.1 302 Found\r\nLocation: /new?a=1\r\nContent-Length: 0\r\n\r\n"
        if t.startswith("/drop"):
            return None
        if t.startswith("/bad"):
            return b"SMTP ready\r\n\r\n"
        return b"HTTP/1.1 200 OK\r\nContent-Length: 3\r\n\r\nnew"

    async def one(fast):
        s = await Raw(respond).start()
        c = H1Client(timeout_s=5)
        if not fast:
            c.native_call = None
        base = f"http://127.0.0.1:{s.port}"
        seen = []
        for m, p in [("GET", "/new"), ("GET", "/old"), ("POST", "/old"), ("GET", "/drop"), ("POST", "/drop"),
                     ("GET", "/bad"), ("GET", "/new")]:
            await c.request("GET", base + "/new")  # warm: an idle connection for the fast path
            try:
                r = await c.request(m, base + p)
                seen.append((r.status, r.body, r.url.replace(base, "")))
            except HttpError as e:
                seen.append(str(e).replace(base, ""))
        st = dict(c.counts)
        await c.close()
        await s.stop()
        return seen, st, [r.split(b"\r\n")[0] for r in s.raw]

    async def go():
        return await one(True), await one(False)
    fast, slow = run(go())
    assert fast == slow
    assert fast[1]["retries"] >= 1 and fast[1]["errors"] >= 2


def test_fast_path_timeout_cancel_and_abandon_release_the_connection():
    async def go():
        s = await Raw(lambda t: "hang" if t.startswith("/slow") else OK).start()
        c = H1Client(timeout_s=5)
        base = f"http://127.0.0.1:{s.port}"
        await c.request("GET", base + "/a")
        aw = c.request("GET", base + "/slow", params={"token": "secret"}, timeout=0.2)
        with pytest.raises(HttpError, match=r"^ETIMEDOUT: GET http://127\.0\.0\.1:\d+/slow$"):
            await aw
        assert aw.native is True
        await c.request("GET", base + "/a")
        t = asyncio.ensure_future(c.request("GET", base + "/slow"))
        await asyncio.sleep(0.05)
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        await c.request("GET", base + "/a")
        aw = c.request("GET", base + "/slow")
        assert aw.send(None) is not None and aw.native is True  # sent, suspended on the reply
        aw.close()  # never awaited to the end: like closing the coroutine
        busy = len(c._busy)
        r = await c.request("GET", base + "/a")
        st = dict(c.counts)
        open_ = sum(o.open for o in c._origins.values())
        await c.close()
        await s.stop()
        return busy, r.status, st, open_, s.connections
    busy, status, st, open_, conns = run(go())
    assert busy == 0 and status == 200
    assert st["timeouts"] == 1 and st["errors"] == 1
    assert open_ == 1 and conns == 4  # each abandoned request's connection was dropped, a new one opened


def test_client_close_with_requests_in_flight_matches_python():
    """close() while requests wait for their replies: every waiter ends (no hang), with the
    same outcome on the native path and on the Python one, and nothing stays open."""
    async def one(fast):
        s = await Raw(lambda t: "hang" if t.startswith("/slow") else OK).start()
        c = H1Client(timeout_s=5, max_per_host=4)
        if not fast:
            c.native_call = None
        base = f"http://127.0.0.1:{s.port}"
        await asyncio.gather(*[c.request("GET", f"{base}/w{i}") for i in range(4)])
        tasks = [asyncio.ensure_future(c.request("POST", f"{base}/slow{i}", params={"i": i})) for i in range(4)]
        await asyncio.sleep(0.05)
        await c.close()
        done = await asyncio.wait_for(asyncio.gather(*tasks, return_exceptions=True), 5)
        open_ = sum(o.open for o in c._origins.values())
        await s.stop()
        return [type(x).__name__ + ":" + str(x).replace(base, "") for x in done], open_, len(c._busy)

    async def go():
        return await one(True), await one(False)
    fast, slow = run(go())
    assert fast == slow
    assert fast[1] == 0 and fast[2] == 0


def test_fast_path_under_native_driver_and_gather():
    """Many concurrent requests through gather (Tasks) and through a native Driver."""
    async def go():
        s = await Raw(lambda t: OK).start()
        c = H1Client(timeout_s=5, max_per_host=8)
        base = f"http://127.0.0.1:{s.port}"
        await asyncio.gather(*[c.request("GET", f"{base}/w{i}") for i in range(8)])
        rs = await asyncio.gather(*[c.request("POST", f"{base}/p{i}", params={"i": i}) for i in range(200)])
        done = []

        async def handler(i):
            r = await c.request("PUT", f"{base}/d{i}", params={"pos": 2})
            done.append(r.status)

        for i in range(50):
            coro = handler(i)
            first = coro.send(None)
            native.Driver(coro, lambda d, e: None).start(first)
        while len(done) < 50:
            await asyncio.sleep(0.01)
        st = dict(c.counts)
        await c.close()
        await s.stop()
        return [r.status for r in rs], done, st, s.connections
    statuses, done, st, conns = run(go())
    assert statuses == [200] * 200 and done == [200] * 50
    assert st["requests"] == 258 and conns <= 8


def _script(seed):
    """Server behaviour for the differential run: a function of the request's global index only
    (the same in both runs when the client behaves the same)."""
    rnd = random.Random(seed)
    plan = []
    for _ in range(120):
        kind = rnd.choices(["ok", "cl", "chunked", "close", "redirect", "status", "drop", "drop_mid", "head204"],
                           [30, 10, 10, 8, 6, 10, 6, 4, 4])[0]
        plan.append((kind, rnd.randrange(0, 2000), rnd.choice([200, 201, 204, 404, 500, 503])))
    return plan


def _response(kind, n, status, target):
    body = (b"x%d" % n) * (n % 7)
    if kind == "ok":
        return b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(body) + body
    if kind == "cl":
        return b"HTTP/1.1 %d S\r\nContent-Length: %d\r\nX-N: %d\r\n\r\n" % (status, len(body), n) + body
    if kind == "chunked":
        return (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" + b"%x\r\n" % len(body) + body
                + b"\r\n" if body else b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n") + b"0\r\n\r\n"
    if kind == "close":
        return b"HTTP/1.1 200 OK\r\nConnection: close\r\nContent-Length: %d\r\n\r\n" % len(body) + body
    if kind == "redirect":
        return b"HTTP/1.1 302 Found\r\nLocation: /r%d\r\nContent-Length: 0\r\n\r\n" % n
    if kind == "status":
        return b"HTTP/1.1 %d X\r\nContent-Length: 0\r\n\r\n" % status
    if kind == "head204":
        return b"HTTP/1.1 204 No Content\r\n\r\n"
    if kind == "drop_mid":
        return (b"HTTP/1.1 200 OK\r\nContent-Length: 100\r\n\r\npartial", "close")
    return None  # drop


@pytest.mark.parametrize("seed", range(16))
def test_differential_random_server_behaviour(seed):
    """Random status codes, framings, Connection: close, redirects, drops before and in the
    middle of a response: the fast path and the Python path see the same requests on the same
    connections and produce the same outcomes and counters."""
    plan = _script(seed)

    class Srv(Raw):
        def __init__(self):
            super().__init__(None)
            self.n = 0
            self.trace = []

        async def _serve(self, r, w):
            self.connections += 1
            conn = self.connections
            try:
                while True:
                    try:
                        head = await r.readuntil(b"\r\n\r\n")
                    except (asyncio.IncompleteReadError, ConnectionError):
                        return
                    i = self.n
                    self.n += 1
                    kind, n, status = plan[i % len(plan)]
                    target = head.split(b" ", 2)[1].decode()
                    self.trace.append((conn, head.split(b" ", 1)[0].decode(), target, kind))
                    if target.startswith("/r"):
                        kind = "ok"  # redirect targets answer
                    out = _response(kind, n, status, target)
                    if out is None:
                        w.transport.abort()
                        return
                    close = isinstance(out, tuple)
                    w.write(out[0] if close else out)
                    await w.drain()
                    if close or kind == "close":
                        return
            finally:
                w.close()

    async def one(fast):
        s = await Srv().start()
        c = H1Client(timeout_s=5, max_per_host=4)
        if not fast:
            c.native_call = None
        rnd = random.Random(seed + 100)
        base = f"http://127.0.0.1:{s.port}"
        out = []
        for i in range(80):
            m = rnd.choice(["GET", "POST", "PUT", "HEAD", "DELETE"])
            params = rnd.choice([None, {"i": i}, {"text": "a b ü", "k": None}])
            conc = rnd.choice([1, 1, 1, 3])
            aws = [c.request(m, f"{base}/p{i}_{j}", params=params) for j in range(conc)]
            res = await asyncio.gather(*aws, return_exceptions=True)
            for r in res:
                if isinstance(r, HttpError):
                    out.append(("err", str(r).replace(base, "")))
                elif isinstance(r, BaseException):
                    raise r
                else:
                    out.append((r.status, r.body, r.url.replace(base, ""), sorted(r.headers.items())))
        st = dict(c.counts)
        await c.close()
        await s.stop()
        return out, st, s.trace

    async def go():
        return await one(True), await one(False)
    (fo, fs, ft), (po, ps, pt) = run(go())
    assert ft == pt  # same requests, same connections, same order
    assert fo == po
    assert fs == ps


def test_compiled_handlers_make_h1_calls_directly(monkeypatch):
    """The compiled handlers make the H1Call themselves (no H1Client.request frame); switching
    a client without the `native_call` capability sends them back through the Python method."""
    from beholder_amd.service import Service
    from beholder_amd.store import MemoryStore
    from beholder_amd.topics import PROGRESS
    from beholder_amd.transport.memory import MemoryBroker
    from beholder_amd.utils.log import Logger, MemoryStream

    from helpers import cfg, progress_msg
    from test_stores import M1

    calls = []
    orig = H1Client.request

    def counting(self, *a, **k):
        calls.append(a[0])
        return orig(self, *a, **k)

    monkeypatch.setattr(H1Client, "request", counting)

    async def go(direct):
        s = await Raw(lambda t: OK).start()
        b = MemoryBroker()
        http = H1Client(timeout_s=5)
        if not direct:
            http.native_call = None  # the client hands out no native capability
        url = f"http://127.0.0.1:{s.port}"
        svc = Service(cfg({"service": {"endpoints": {"trello": url, "telegram": url}}}), source=b.consumer(),
                      store=MemoryStore([M1]), http=http, logger=Logger(stream=MemoryStream()), serve_metrics=False)
        await svc.init()
        run_ = asyncio.ensure_future(svc.run())
        for i in range(20):
            b.publish(PROGRESS, progress_msg("m1", "CONVERTING", i))
        b.finish()
        stats = await run_
        await svc.close()
        await http.close()
        await s.stop()
        return stats["source"]["acked"], len(s.raw), type(svc.handler_impl).__name__

    calls.clear()
    acked, served, impl = run(go(True))
    assert (acked, served, impl) == (20, 20, "NativeHandlers") and calls == []
    acked, served, _ = run(go(False))
    assert (acked, served) == (20, 20) and calls.count("POST") == 20


async def _queued_run(fast: bool):
    """A pool of 3 and 60 concurrent requests: most wait in the origin's queue. Returns what the
    client did (responses, counts, the exact requests the server saw, connections made)."""
    s = await Raw(lambda t: OK).start()
    c = H1Client(timeout_s=5, max_per_host=3)
    if not fast:
        c.native_call = None
    base = f"http://127.0.0.1:{s.port}"
    await c.request("GET", base + "/warm")
    shapes = [("POST", "/1/cards/c1/actions/comments", {"text": "DEPLOYED ü", "key": "k"}),
              ("PUT", "/1/cards/c2", {"idList": "L", "pos": 2}), ("GET", "/bot1:X/sendMessage", {"chat_id": 5}),
              ("HEAD", "/emby", None), ("GET", "/plain?x=1", None)]
    aws = [c.request(m, base + p, params=q) for i in range(60) for m, p, q in [shapes[i % len(shapes)]]]
    rs = await asyncio.gather(*aws)
    out = [(r.status, r.body, r.url.replace(base, "")) for r in rs]
    kinds = [getattr(aw, "native", False) for aw in aws]  # the Python path returns coroutines
    counts = dict(c.counts)
    open_ = sum(o.open for o in c._origins.values())
    await c.close()
    await s.stop()
    raw = sorted(r.replace(str(s.port).encode(), b"PORT") for r in s.raw)
    return out, kinds, counts, raw, s.connections, open_


def test_queued_requests_take_the_native_path_and_match_python():
    """No idle connection at the first await: the request waits in the origin's queue
    (H1Client._enqueue) and is sent natively when a connection is handed over. Responses, the
    bytes on the wire, every count and the connections made are those of the Python loop."""
    async def go():
        return await _queued_run(True), await _queued_run(False)
    fast, slow = run(go())
    f_out, f_kinds, f_counts, f_raw, f_conns, f_open = fast
    p_out, p_kinds, p_counts, p_raw, p_conns, p_open = slow
    assert f_out == p_out and f_raw == p_raw
    assert f_counts == p_counts and f_conns == p_conns and f_open == p_open
    assert f_counts["connect_waits"] > 40
    # queued ones too (the origin was known, the pool full); a request handed a freed slot
    # instead of a connection (after a HEAD reply leaves a connection unusable) continues in Python
    assert f_kinds.count(True) >= 40


def test_queued_timeout_cancel_and_close_match_python():
    """A request waiting in the queue: its deadline (ETIMEDOUT), a cancel (its place is given up,
    no connection leaks) and the client closing ("client closed") end it as on the Python path,
    under gather (Tasks) and under the native Driver."""
    async def one(fast):
        s = await Raw(lambda t: "hang" if t.startswith("/slow") else OK).start()
        c = H1Client(timeout_s=5, max_per_host=1)
        if not fast:
            c.native_call = None
        base = f"http://127.0.0.1:{s.port}"
        await c.request("GET", base + "/warm")
        hog = asyncio.ensure_future(c.request("GET", base + "/slow"))  # holds the only connection
        await asyncio.sleep(0.02)
        res = []
        try:
            await c.request("GET", base + "/q", params={"token": "s"}, timeout=0.1)
        except HttpError as e:
            res.append(str(e).replace(base, ""))
        t = asyncio.ensure_future(c.request("GET", base + "/cancelled"))
        await asyncio.sleep(0.02)
        t.cancel()
        res.append(type((await asyncio.gather(t, return_exceptions=True))[0]).__name__)
        got = []

        async def handler():
            try:
                got.append((await c.request("PUT", base + "/d", params={"pos": 2}, timeout=0.1)).status)
            except HttpError as e:
                got.append(str(e).replace(base, ""))
        coro = handler()
        native.Driver(coro, lambda d, e: None).start(coro.send(None))
        while not got:
            await asyncio.sleep(0.01)
        res.append(got[0])
        waiting = [asyncio.ensure_future(c.request("GET", base + f"/w{i}")) for i in range(3)]
        await asyncio.sleep(0.02)
        await c.close()
        done = await asyncio.wait_for(asyncio.gather(hog, *waiting, return_exceptions=True), 5)
        res += [type(x).__name__ + ":" + str(x) for x in done]
        counts = dict(c.counts)
        open_ = sum(o.open for o in c._origins.values())
        await s.stop()
        return res, counts, open_

    async def go():
        return await one(True), await one(False)
    fast, slow = run(go())
    assert fast == slow
    res, counts, open_ = fast
    assert res[0] == "ETIMEDOUT: GET /q" and res[1] == "CancelledError" and res[2] == "ETIMEDOUT: PUT /d"
    assert res[3:] == ["HttpError:client closed"] * 4 and open_ == 0


def test_queued_request_gets_the_connect_error_of_a_failed_background_connect():
    """The first queued request of an origin whose background connect fails gets the connect
    error (as from _acquire), mapped to the Node-style message."""
    import socket as _s

    async def one(fast):
        srv = await Raw(lambda t: OK).start()
        c = H1Client(timeout_s=2, max_per_host=1)
        if not fast:
            c.native_call = None
        base = f"http://127.0.0.1:{srv.port}"
        await c.request("GET", base + "/warm")
        o = c._origins[base]
        conn = o.idle.pop()  # the only connection, gone; new connects go to a closed port
        c._drop(conn)
        await srv.stop()
        probe = _s.socket()
        probe.bind(("127.0.0.1", 0))
        o.port = probe.getsockname()[1]  # nothing listens here
        probe.close()
        try:
            await c.request("GET", base + "/x")
            msg = "ok"
        except HttpError as e:
            msg = str(e).split(":")[0] + ":" + str(e).split(" ")[1]
        await c.close()
        return msg

    async def go():
        return await one(True), await one(False)
    fast, slow = run(go())
    assert fast == slow and fast.startswith("connect ECONNREFUSED")


class Gated(Raw):
    """Raw server whose ``/slow`` requests are answered only once ``gate`` is set."""

    def __init__(self):
        super().__init__(lambda t: OK)
        self.gate = asyncio.Event()

    async def _serve(self, r, w):
        self.connections += 1
        try:
            while True:
                try:
                    head = await r.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, ConnectionError):
                    return
                self.raw.append(head)
                if head.split(b" ", 2)[1].startswith(b"/slow"):
                    await self.gate.wait()
                w.write(OK)
                await w.drain()
        finally:
            w.close()


def test_queued_continuation_waits_at_the_front():
    """A request marked as the continuation of an event (h1_fast's ``front``) that finds no idle
    connection waits at the head of the origin's queue: it is sent on the next freed connection,
    before requests that were queued earlier by other events."""
    async def go():
        s = await Gated().start()
        c = H1Client(timeout_s=5, max_per_host=1)
        base = f"http://127.0.0.1:{s.port}"
        await c.request("GET", base + "/warm")
        hog = asyncio.ensure_future(c.request("GET", base + "/slow"))  # holds the only connection
        await asyncio.sleep(0.02)
        first = [asyncio.ensure_future(c.request("GET", base + f"/n{i}")) for i in range(3)]
        await asyncio.sleep(0.02)
        cont = asyncio.ensure_future(c.native_call(c, "GET", base + "/cont", None, None, True))
        await asyncio.sleep(0.02)
        queued = len(c._origins[base].waiters)
        s.gate.set()
        rs = await asyncio.gather(hog, *first, cont)
        await c.close()
        await s.stop()
        return queued, [r.status for r in rs], [h.split(b" ", 2)[1].decode() for h in s.raw]
    queued, statuses, order = run(go())
    assert queued == 4 and statuses == [200] * 5
    assert order == ["/warm", "/slow", "/cont", "/n0", "/n1", "/n2"]


@pytest.mark.parametrize("trello_retry", [False, True])
def test_compiled_handlers_queue_an_events_later_requests_at_the_front(monkeypatch, trello_retry):
    """The compiled handlers mark an event's second and later sink requests (a DEPLOYED status:
    the Trello move, then the Telegram and Emby hooks, index.js:83,99,112) as continuations; its
    first request queues behind earlier ones as usual. A Trello client with 429 retries sends
    through its own Python method (unmarked), and still counts as the event's first request."""
    from beholder_amd.service import Service
    from beholder_amd.store import MemoryStore
    from beholder_amd.topics import STATUS
    from beholder_amd.transport.memory import MemoryBroker
    from beholder_amd.utils.log import Logger, MemoryStream

    from helpers import cfg, status_msg, trello_media

    seen = []
    orig = H1Client._enqueue

    def recording(self, o, deadline, w, front=False):
        seen.append(front)
        return orig(self, o, deadline, w, front)

    monkeypatch.setattr(H1Client, "_enqueue", recording)

    async def go():
        s = await Raw(lambda t: OK).start()
        b = MemoryBroker()
        # keepalive 0: no idle connection is ever reused, so every request after the origin's
        # first goes through the queue
        http = H1Client(timeout_s=5, keepalive_s=0.0)
        url = f"http://127.0.0.1:{s.port}"
        await http.request("GET", url + "/warm")
        over = {"service": {"endpoints": {"trello": url, "telegram": url}},
                "instance": {"emby": {"host": url}}}
        if trello_retry:
            over["service"]["sinks"] = {"trello": {"retry_429": 1}}
        svc = Service(cfg(over), source=b.consumer(), store=MemoryStore([trello_media("m1", card="C1")]), http=http,
                      logger=Logger(stream=MemoryStream()), serve_metrics=False)
        await svc.init()
        run_ = asyncio.ensure_future(svc.run())
        b.publish(STATUS, status_msg("m1", "DEPLOYED"))
        b.finish()
        stats = await run_
        await svc.close()
        await http.close()
        await s.stop()
        return stats["source"]["acked"], [h.split(b" ", 2)[:2] for h in s.raw], type(svc.handler_impl).__name__
    acked, reqs, impl = run(go())
    assert acked == 1 and impl == "NativeHandlers"
    assert len(reqs) - 1 == len(seen) >= 2, (reqs, seen)
    assert seen[0] is False and all(seen[1:]), seen
