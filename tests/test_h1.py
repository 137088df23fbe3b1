"""Native HTTP/1.1 response parser (`ops/csrc/py_http.cpp`) and the keep-alive sink client
(`sinks/h1.py`) that the service uses by default for Trello / Telegram / Emby
(index.js:53,83,99,112)."""
import asyncio
import socket
import shutil
import ssl
import subprocess
import time

import pytest
from hypothesis import given, settings, strategies as st

from beholder_amd.ops import H1Parser
from beholder_amd.sinks import H1Client, HttpError
from beholder_amd.sinks.http import parse_raw_headers, with_query


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


def feed_all(p, data, step=None):
    """Feeds data in `step`-byte pieces; returns the first completed result."""
    step = step or len(data) or 1
    for i in range(0, len(data), step):
        r = p.feed(data[i:i + step])
        if r is not None:
            return r
    return None


# ---------------------------------------------------------------- parser ----

def test_content_length_split_at_every_byte():
    raw = b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: 13\r\n\r\n{\"id\": \"abc\"}"
    for step in (1, 2, 3, 7, len(raw)):
        p = H1Parser()
        p.start()
        assert feed_all(p, raw, step) == (200, "OK", b"Content-Type: application/json\r\nContent-Length: 13\r\n",
                                          b'{"id": "abc"}', True)
        assert p.idle and p.buffered == 0


def test_chunked_with_extensions_and_trailers():
    raw = (b"HTTP/1.1 201 Created\r\nTransfer-Encoding: gzip, chunked\r\n\r\n"
           b"5;name=v\r\nhello\r\n1\r\n \r\nA\r\n0123456789\r\n0\r\nX-Trailer: 1\r\n\r\n")
    for step in (1, 4, len(raw)):
        p = H1Parser()
        p.start()
        st_, reason, _, body, keep = feed_all(p, raw, step)
        assert (st_, reason, body, keep) == (201, "Created", b"hello 0123456789", True)


def test_interim_100_continue_is_skipped():
    p = H1Parser()
    p.start()
    r = p.feed(b"HTTP/1.1 100 Continue\r\n\r\nHTTP/1.1 103 Early\r\nLink: x\r\n\r\nHTTP/1.1 204 No Content\r\n\r\n")
    assert r[0] == 204 and r[3] == b""


def test_no_body_for_head_204_304():
    p = H1Parser()
    p.start(head=True)
    assert p.feed(b"HTTP/1.1 200 OK\r\nContent-Length: 50\r\n\r\n")[3] == b""
    for code in (204, 304):
        p.start()
        assert p.feed(f"HTTP/1.1 {code} X\r\nContent-Length: 9\r\n\r\n".encode())[:1] == (code,)


def test_close_delimited_body_and_keep_alive_rules():
    p = H1Parser()
    p.start()
    assert p.feed(b"HTTP/1.0 404 Not Found\nServer: x\n\nnot ") is None  # LF-only line ends accepted
    assert p.feed(b"here") is None
    assert p.eof() == (404, "Not Found", b"Server: x\r\n", b"not here", False)
    p.start()
    assert p.feed(b"HTTP/1.1 200 OK\r\nConnection: close\r\nContent-Length: 0\r\n\r\n")[4] is False
    p.start()
    assert p.feed(b"HTTP/1.0 200 OK\r\nConnection: Keep-Alive\r\nContent-Length: 0\r\n\r\n")[4] is True
    p.start()
    assert p.feed(b"HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n")[4] is True


def test_eof_semantics():
    p = H1Parser()
    p.start()
    assert p.eof() is None  # closed before any response byte (stale keep-alive connection)
    p.start()
    p.feed(b"HTTP/1.1 200 OK\r\nContent-Length: 10\r\n\r\nabc")
    assert p.started
    with pytest.raises(ValueError):
        p.eof()  # truncated body


@pytest.mark.parametrize("raw", [
    b"HTTX/1.1 200 OK\r\n\r\n",
    b"HTTP/1.1 2x0 OK\r\n\r\n",
    b"HTTP/2.0 200 OK\r\n\r\n",
    b"HTTP/1.1 200 OK\r\nBad Header\r\n\r\n",
    b"HTTP/1.1 200 OK\r\nNa me: v\r\n\r\n",
    b"HTTP/1.1 200 OK\r\n folded: v\r\n\r\n",
    b"HTTP/1.1 200 OK\r\nContent-Length: 1\r\nContent-Length: 2\r\n\r\n",
    b"HTTP/1.1 200 OK\r\nContent-Length: -1\r\n\r\n",
    b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n",
    b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n1\r\nab\r\n",
    b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nfffffffffffffffff\r\n",
    b"HTTP/1.1 101 Switching Protocols\r\n\r\n",
])
def test_malformed_responses_raise(raw):
    p = H1Parser()
    p.start()
    with pytest.raises(ValueError):
        p.feed(raw)
    assert p.idle  # reset: the connection is discarded by the client


def test_limits():
    p = H1Parser(max_header=128, max_body=10)
    p.start()
    with pytest.raises(ValueError, match="too large"):
        p.feed(b"HTTP/1.1 200 OK\r\n" + b"X: " + b"a" * 200 + b"\r\n")
    p.start()
    with pytest.raises(ValueError, match="max_body"):
        p.feed(b"HTTP/1.1 200 OK\r\nContent-Length: 11\r\n\r\n")
    p.start()
    with pytest.raises(ValueError, match="max_body"):
        p.feed(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n8\r\n12345678\r\n8\r\n")
    with pytest.raises(RuntimeError):
        p.start()
        p.start()  # start() while a response is in progress


def test_leftover_bytes_are_reported():
    p = H1Parser()
    p.start()
    r = p.feed(b"HTTP/1.1 200 OK\r\nContent-Length: 1\r\n\r\nxHTTP/1.1")
    assert r[3] == b"x" and p.buffered == 8


def test_parse_raw_headers_joins_repeats():
    assert parse_raw_headers(b"A: 1\r\nSet-Cookie: x\r\nset-cookie: y\r\n") == {"a": "1", "set-cookie": "x, y"}


@st.composite
def responses(draw):
    status = draw(st.integers(200, 599))
    body = draw(st.binary(max_size=300))
    hdrs = draw(st.lists(st.tuples(st.sampled_from(["X-A", "Server", "ETag", "Vary"]),
                                   st.text("abcdefgh0123 =;", max_size=20)), max_size=4))
    mode = draw(st.sampled_from(["length", "chunked", "close"]))
    eol = draw(st.sampled_from([b"\r\n", b"\n"]))
    head = [f"HTTP/1.1 {status} R".encode()] + [f"{k}: {v}".encode() for k, v in hdrs]
    if mode == "length":
        head.append(f"Content-Length: {len(body)}".encode())
        payload = body
    elif mode == "chunked":
        head.append(b"Transfer-Encoding: chunked")
        cuts = sorted(draw(st.lists(st.integers(0, len(body)), max_size=5)))
        parts, last = [], 0
        for c in cuts + [len(body)]:
            if c > last:
                parts.append(body[last:c])
                last = c
        payload = b"".join(b"%x\r\n%s\r\n" % (len(x), x) for x in parts) + b"0\r\n\r\n"
    else:
        head.append(b"Connection: close")
        payload = body
    if status in (204, 304):
        body = b""
        payload = b"" if mode != "chunked" else payload
        if mode == "chunked":
            payload = b""
    raw = eol.join(head) + eol + eol + payload
    splits = draw(st.lists(st.integers(1, max(1, len(raw))), max_size=6))
    return status, body, mode, raw, splits


@settings(max_examples=300, deadline=None)
@given(responses())
def test_property_any_split_gives_same_result(case):
    status, body, mode, raw, splits = case
    p = H1Parser()
    p.start()
    r = None
    pos = 0
    for s in sorted(set(splits)) + [len(raw)]:
        if s <= pos:
            continue
        r = p.feed(raw[pos:s])
        pos = s
        if r is not None:
            break
    if r is None:
        r = p.eof()
    assert r is not None
    assert r[0] == status and r[3] == body
    assert r[4] == (mode != "close")


@settings(max_examples=500, deadline=None)
@given(st.binary(max_size=400), st.booleans())
def test_fuzz_random_bytes_never_crash(data, head):
    p = H1Parser(max_header=256, max_body=1024)
    p.start(head=head)
    try:
        p.feed(data)
        p.eof()
    except ValueError:
        pass


# ---------------------------------------------------------------- client ----

class Scripted:
    """A tiny HTTP/1.1 server whose per-request behaviour is a Python function.

    ``respond(n_on_conn, method, target, headers) -> bytes | (bytes, "close") | None``
    (None = abort the connection without answering; "hang" = never answer)."""

    def __init__(self, respond):
        self.respond = respond
        self.requests = []
        self.connections = 0
        self.peak = 0
        self.live = 0
        self.server = None
        self.port = 0

    async def start(self, ssl_ctx=None):
        self.server = await asyncio.start_server(self._serve, "127.0.0.1", 0, ssl=ssl_ctx)
        self.port = self.server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        self.server.close()
        await self.server.wait_closed()

    async def _serve(self, r, w):
        self.connections += 1
        self.live += 1
        self.peak = max(self.peak, self.live)
        n = 0
        try:
            while True:
                try:
                    head = await r.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, ConnectionError):
                    return
                lines = head.decode("latin-1").split("\r\n")
                method, target, _ = lines[0].split(" ", 2)
                hdrs = {k.strip().lower(): v.strip() for k, _, v in (ln.partition(":") for ln in lines[1:] if ln)}
                self.requests.append((method, target, hdrs))
                out = self.respond(n, method, target, hdrs)
                n += 1
                if out == "hang":
                    await asyncio.sleep(3600)
                if out is None:
                    w.transport.abort()
                    return
                close = isinstance(out, tuple)
                w.write(out[0] if close else out)
                await w.drain()
                if close:
                    return
        finally:
            self.live -= 1
            w.close()


OK = b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\n{}"


def test_keep_alive_reuses_one_connection_and_target_is_verbatim():
    async def go():
        s = await Scripted(lambda n, m, t, h: OK).start()
        c = H1Client(timeout_s=5)
        for i in range(20):
            r = await c.request("POST", f"http://127.0.0.1:{s.port}/1/cards/C{i}/actions/comments",
                                params={"text": "DEPLOYED: Progress **5%** (_h_) ü", "key": "k"})
            assert r.status == 200 and r.body == b"{}" and r.ok
        r = await c.request("GET", f"http://127.0.0.1:{s.port}/emby/library/refresh", params={"api_key": "x"})
        await c.close()
        await s.stop()
        return s, c, r
    s, c, r = run(go())
    assert s.connections == 1 and c.counts["reused"] == 20
    m, target, hdrs = s.requests[0]
    assert (m, target) == ("POST", "/1/cards/C0/actions/comments?text=DEPLOYED%3A%20Progress%20**5%25**%20(_h_)"
                                   "%20%C3%BC&key=k")
    assert hdrs["content-length"] == "0" and hdrs["host"] == f"127.0.0.1:{s.port}"
    assert s.requests[-1][0] == "GET" and "content-length" not in s.requests[-1][2]
    assert r.headers == {"content-length": "2"}


def test_a_fragment_in_the_url_keeps_the_parameters():
    """A path segment from the database can hold '#' (Trello's /1/cards/{creatorId}): the fragment
    is never sent, and the parameters (the comment text, key and token) join the query before it,
    as Node's url.parse + request put them, instead of being dropped with it."""
    async def go():
        s = await Scripted(lambda n, m, t, h: OK).start()
        c = H1Client(timeout_s=5)
        base = f"http://127.0.0.1:{s.port}/1/cards/"
        await c.request("POST", base + "a&b=c?d#e/actions/comments", params={"text": "x y", "key": "K"})
        await c.request("POST", base + "c#1/actions/comments", params={"text": "x", "key": "K"})
        await c.request("GET", base + "c#1", params=None)
        await c.close()
        await s.stop()
        return [t for _, t, _ in s.requests]
    assert run(go()) == ["/1/cards/a&b=c?d&text=x%20y&key=K", "/1/cards/c?text=x&key=K", "/1/cards/c"]


def test_connection_close_and_http10_open_new_connections():
    def respond(n, m, t, h):
        if t.startswith("/close"):
            return b"HTTP/1.1 200 OK\r\nConnection: close\r\nContent-Length: 1\r\n\r\nx"
        return b"HTTP/1.0 200 OK\r\n\r\nold", "close"  # close-delimited

    async def go():
        s = await Scripted(respond).start()
        c = H1Client(timeout_s=5)
        bodies = [(await c.request("GET", f"http://127.0.0.1:{s.port}/{p}")).body for p in ("close", "close", "x")]
        await c.close()
        await s.stop()
        return s, bodies
    s, bodies = run(go())
    assert bodies == [b"x", b"x", b"old"] and s.connections == 3


def test_redirects_followed_for_get_only():
    def respond(n, m, t, h):
        if t.startswith("/old"):
            return b"HTTP/1.1 302 Found\r\nLocation: /new?a=1\r\nContent-Length: 0\r\n\r\n"
        if t.startswith("/loop"):
            return b"HTTP/1.1 301 Moved\r\nLocation: /loop\r\nContent-Length: 0\r\n\r\n"
        return b"HTTP/1.1 200 OK\r\nContent-Length: 3\r\n\r\nnew"

    async def go():
        s = await Scripted(respond).start()
        c = H1Client(timeout_s=5, max_redirects=3)
        base = f"http://127.0.0.1:{s.port}"
        g = await c.request("GET", base + "/old")
        p = await c.request("POST", base + "/old")
        with pytest.raises(HttpError, match="maxRedirects"):
            await c.request("GET", base + "/loop")
        await c.close()
        await s.stop()
        return g, p, s
    g, p, s = run(go())
    assert (g.status, g.body, g.url.endswith("/old")) == (200, b"new", True)
    assert p.status == 302  # request: followRedirect applies to GET only
    assert ("GET", "/new?a=1") in [(m, t) for m, t, _ in s.requests]


def test_timeout_drops_connection_and_reports_etimedout():
    async def go():
        s = await Scripted(lambda n, m, t, h: "hang" if t.startswith("/slow") else OK).start()
        c = H1Client(timeout_s=5)
        t0 = time.monotonic()
        with pytest.raises(HttpError, match=r"^ETIMEDOUT: GET http://127\.0\.0\.1:\d+/slow$"):
            await c.request("GET", f"http://127.0.0.1:{s.port}/slow", params={"token": "secret"}, timeout=0.2)
        dt = time.monotonic() - t0
        ok = await c.request("GET", f"http://127.0.0.1:{s.port}/fast")
        st_ = c.stats()
        await c.close()
        s.server.close()
        return dt, ok.status, st_
    dt, status, stats = run(go())
    assert 0.2 <= dt < 1.0 and status == 200
    assert stats["timeouts"] == 1 and stats["connections"] == 2


def test_stale_reused_connection_retry_only_for_idempotent_methods():
    # the server answers the first request on each connection, then drops the connection
    # on the second without answering: what a keep-alive timeout race looks like
    async def go():
        s = await Scripted(lambda n, m, t, h: OK if n == 0 else None).start()
        c = H1Client(timeout_s=5)
        url = f"http://127.0.0.1:{s.port}/x"
        await c.request("GET", url)
        r = await c.request("GET", url)  # reused -> reset -> retried on a fresh connection
        with pytest.raises(HttpError, match="socket hang up|ECONNRESET"):
            await c.request("POST", url)  # reuses the retry's connection, which drops: never replayed
        p = await c.request("POST", url)  # the dead connection was discarded: a fresh one works
        st_ = c.stats()
        await c.close()
        await s.stop()
        return r.status, p.status, st_, [m for m, _, _ in s.requests]
    status, pstatus, st_, methods = run(go())
    assert status == 200 and pstatus == 200 and st_["retries"] == 1 and st_["errors"] == 1
    assert methods == ["GET", "GET", "GET", "POST", "POST"]  # the failed POST reached the server once


def test_max_per_host_bounds_connections():
    async def slow(n, m, t, h):
        return OK

    async def go():
        s = Scripted(lambda n, m, t, h: OK)
        orig = s._serve

        async def serve(r, w):
            await asyncio.sleep(0.01)
            await orig(r, w)
        s._serve = serve
        await s.start()
        c = H1Client(timeout_s=5, max_per_host=3)
        rs = await asyncio.gather(*[c.request("GET", f"http://127.0.0.1:{s.port}/{i}") for i in range(40)])
        await c.close()
        await s.stop()
        return s, rs
    s, rs = run(go())
    assert all(r.status == 200 for r in rs) and s.connections <= 3 and len(s.requests) == 40


def test_queue_wait_timestamps_leave_with_their_waiters():
    """Requests that time out in the connection queue keep no enqueue timestamp once their waiter
    is dropped from the queue; the ones handed a connection are in the queue-wait histogram."""
    async def go():
        s = Scripted(lambda n, m, t, h: OK)
        orig = s._serve

        async def serve(r, w):
            await asyncio.sleep(0.15)
            await orig(r, w)
        s._serve = serve
        await s.start()
        c = H1Client(timeout_s=5, max_per_host=1)
        url = f"http://127.0.0.1:{s.port}/"
        first = asyncio.ensure_future(c.request("GET", url + "0"))
        await asyncio.sleep(0.02)
        short = [asyncio.ensure_future(c.request("GET", url + str(i), timeout=0.05)) for i in range(1, 7)]
        await asyncio.sleep(0.08)  # they have timed out, their waiters still queued
        late = asyncio.ensure_future(c.request("GET", url + "late"))  # queues behind them: drops them
        rs = await asyncio.gather(first, *short, late, return_exceptions=True)
        o = next(iter(c._origins.values()))
        left = (len(o.queued_at), len(o.waiters))
        await c.close()
        await s.stop()
        return rs, left, c.queue_wait_ns.count
    rs, (stamps, waiters), waited = run(go())
    assert rs[0].status == 200 and rs[-1].status == 200
    assert all(isinstance(r, HttpError) for r in rs[1:-1])
    assert stamps == 0 and waiters == 0
    assert waited >= 1  # the late request was handed the connection


def test_connection_refused_and_bad_urls():
    async def go():
        c = H1Client(timeout_s=2)
        with pytest.raises(HttpError, match="^connect ECONNREFUSED 127.0.0.1:9$"):  # Node's err.message
            await c.request("GET", "http://127.0.0.1:9/x", params={"api_key": "s3cret"})
        with pytest.raises(HttpError, match="Invalid protocol"):
            await c.request("GET", "ftp://h/x")
        with pytest.raises(HttpError, match="Invalid URI"):
            await c.request("GET", "undefined/emby/library/refresh")  # js_str(undefined host)
        with pytest.raises(HttpError, match="^getaddrinfo ENOTFOUND no-such-host.invalid$"):
            await c.request("GET", "http://no-such-host.invalid/x")
        await c.close()
    run(go())


def test_name_resolution_counts_against_the_request_timeout():
    """A resolver that never answers ends in ETIMEDOUT at the request's deadline (the native
    connect resolves names itself; asyncio's create_connection did it inside the timeout)."""
    async def go():
        loop = asyncio.get_running_loop()

        async def stuck(*a, **k):
            await asyncio.sleep(3600)
        loop.getaddrinfo = stuck
        c = H1Client(timeout_s=5)
        t0 = loop.time()
        with pytest.raises(HttpError, match="^ETIMEDOUT: GET http://resolver-hangs.example/x$"):
            await c.request("GET", "http://resolver-hangs.example/x", timeout=0.2)
        took = loop.time() - t0
        await asyncio.sleep(0.05)  # the queue's background connect ends at the same deadline
        st = dict(c.counts)
        open_ = sum(o.open for o in c._origins.values())
        await c.close()
        return took, st, open_
    took, st, open_ = run(go())
    assert took < 2 and st["timeouts"] == 1 and open_ == 0


def test_invalid_response_is_an_http_error():
    async def go():
        s = await Scripted(lambda n, m, t, h: b"SMTP ready\r\n\r\n").start()
        c = H1Client(timeout_s=5)
        with pytest.raises(HttpError, match="HPE_INVALID_RESPONSE"):
            await c.request("GET", f"http://127.0.0.1:{s.port}/")
        await c.close()
        await s.stop()
    run(go())


def test_basic_auth_from_userinfo_is_sent_and_redacted():
    async def go():
        s = await Scripted(lambda n, m, t, h: OK).start()
        c = H1Client(timeout_s=5)
        await c.request("GET", f"http://us%40er:p%3Ass@127.0.0.1:{s.port}/emby/library/refresh")
        await c.close()
        await s.stop()
        return s.requests[0][2]
    import base64
    assert run(go())["authorization"] == "Basic " + base64.b64encode(b"us@er:p:ss").decode()
    from beholder_amd.sinks import redact
    assert redact("http://user:pw@h:1/x?api_key=1") == "http://***@h:1/x"


def test_https_with_private_ca(tmp_path):
    if shutil.which("openssl") is None:
        pytest.skip("needs openssl")
    key, crt = tmp_path / "k.pem", tmp_path / "c.pem"
    r = subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out",
                        str(crt), "-days", "1", "-subj", "/CN=localhost", "-addext", "subjectAltName=DNS:localhost"],
                       capture_output=True)
    assert r.returncode == 0, r.stderr

    async def go():
        sctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        sctx.load_cert_chain(str(crt), str(key))
        s = await Scripted(lambda n, m, t, h: OK).start(ssl_ctx=sctx)
        cctx = ssl.create_default_context(cafile=str(crt))
        c = H1Client(timeout_s=5, ssl_context=cctx)
        rs = [await c.request("POST", f"https://localhost:{s.port}/1/cards/x/actions/comments") for _ in range(3)]
        untrusted = H1Client(timeout_s=5)
        with pytest.raises(HttpError, match="CERTIFICATE_VERIFY_FAILED|SSL|certificate"):
            await untrusted.request("GET", f"https://localhost:{s.port}/")
        await c.close()
        await untrusted.close()
        await s.stop()
        return rs, s.connections
    rs, conns = run(go())
    assert [r.status for r in rs] == [200, 200, 200] and conns == 1  # keep-alive over TLS; the rejected
    # handshake never reaches the application


def test_service_uses_h1_client_by_default():
    from beholder_amd.service import make_http_client
    from beholder_amd.sinks import AiohttpClient
    assert isinstance(make_http_client({}), H1Client)
    assert isinstance(make_http_client({"client": "aiohttp"}), AiohttpClient)


@settings(max_examples=400, deadline=None)
@given(st.sampled_from(["http://h", "https://u:p@h:8443", "http://[::1]:80"]),
       st.text(alphabet="/ab c%é#?&=-_", max_size=12),
       st.one_of(st.none(), st.dictionaries(st.sampled_from(["text", "key", "a b", "é"]),
                                            st.one_of(st.text(max_size=8), st.integers(), st.none()), max_size=3)))
def test_cached_route_gives_the_uncached_request_target(origin, path, params):
    """The per-URL route cache (query appended after the cached, already quoted path) builds the
    same URL, origin and request line as resolving the full URL from scratch."""
    c = H1Client()
    url = origin + path
    h = url.find("#")  # a fragment is not sent: the parameters join the query before it
    base, frag = (url, "") if h < 0 else (url[:h], url[h:])
    try:
        want = c._resolve(with_query(base, params))
    except HttpError:  # e.g. "https://u:p@h:8443=": both ways refuse it
        with pytest.raises(HttpError):
            c._prepare(url, params)
        return
    for _ in range(2):  # second time from the cache
        full, o, target, rest = c._prepare(url, params)
        assert full == with_query(base, params) + frag
        assert (o, target, rest) == want


def test_connects_of_a_burst_share_one_name_lookup():
    """A burst to a host name opens connections in waves (max_connecting at a time); they share
    one getaddrinfo, in flight or finished within a second, instead of one resolver query each.
    A later burst resolves again. (Native connects; asyncio's create_connection, with native I/O
    off, resolves on its own.)"""
    from beholder_amd.utils import netconn
    if not netconn.enabled():
        return

    async def go():
        s = await Scripted(lambda n, m, t, h: OK).start()
        loop = asyncio.get_running_loop()
        real, calls = loop.getaddrinfo, []

        async def slow_lookup(host, port, **kw):
            calls.append(host)
            await asyncio.sleep(0.05)
            return [(socket.AF_INET, socket.SOCK_STREAM, 6, "", ("127.0.0.1", port))]
        loop.getaddrinfo = slow_lookup
        try:
            c = H1Client(timeout_s=5, max_connecting=8)
            url = f"http://sink.invalid:{s.port}/x"
            rs = await asyncio.gather(*[c.request("GET", url) for _ in range(12)])
            first = len(calls)
            await c.preconnect(url, 20)  # within a second: the same lookup
            second = len(calls)
            c._resolving[("sink.invalid", s.port)] = (c._resolving[("sink.invalid", s.port)][0], 0.0)  # expired
            await c.preconnect(url, 30)  # a later batch resolves again
            third = len(calls)
            st = dict(c.counts)
            await c.close()
        finally:
            loop.getaddrinfo = real
            await s.stop()
        return [r.status for r in rs], first, second, third, st
    statuses, first, second, third, st = run(go())
    assert statuses == [200] * 12 and st["connections"] >= 2
    assert (first, second, third) == (1, 1, 2)


def test_fresh_retry_hands_a_healthy_used_connection_to_the_next_waiter():
    """a retry that needs a fresh connection, queued at max_per_host and handed a
    healthy keep-alive connection, passes it to the next queued request instead of aborting it
    (a connect plus, for HTTPS, a handshake saved); with nobody else queued it still makes room."""
    from beholder_amd.sinks.h1 import _Conn

    class Tracked(_Conn):
        __slots__ = ("aborted",)

        def __init__(self, o):
            super().__init__(o)
            self.aborted = False

        def abort(self):
            self.aborted = True
            self.closed = True

    async def go():
        c = H1Client(timeout_s=5, max_per_host=1)
        o = c._origin("http://127.0.0.1:9")
        o.open = 1  # the pool is full with one busy connection
        used = Tracked(o)
        used.uses = 3
        loop = asyncio.get_running_loop()
        deadline = loop.time() + 5
        retry = asyncio.ensure_future(c._acquire(o, deadline, fresh=True))
        await asyncio.sleep(0)
        other = asyncio.ensure_future(c._acquire(o, deadline))
        await asyncio.sleep(0)
        c._release(used, True)  # the first waiter is the fresh retry
        got = await asyncio.wait_for(other, 1)
        pending = not retry.done()
        retry.cancel()
        # alone in the queue, the retry drops the used connection to make room for its own
        o2 = c._origin("http://127.0.0.1:10")
        o2.open = 1
        used2 = Tracked(o2)
        used2.uses = 1
        retry2 = asyncio.ensure_future(c._acquire(o2, deadline, fresh=True))
        await asyncio.sleep(0)
        c._connect = lambda o, d, infos=None: asyncio.sleep(0, "fresh")  # the retry's own connect
        c._release(used2, True)
        got2 = await asyncio.wait_for(retry2, 1)
        await c.close()
        return got, used, pending, o.open, got2, used2
    got, used, pending, open_, got2, used2 = run(go())
    assert got is used and not used.aborted and pending and open_ == 1
    assert got2 == "fresh" and used2.aborted


def test_fresh_retry_in_a_saturated_pool_is_not_starved():
    """at max_per_host with several requests queued, a fresh retry passes a healthy
    used connection on at most once; the next one it is handed makes room for its own connect,
    so it finishes well before its deadline instead of waiting behind every release."""
    from beholder_amd.sinks.h1 import _Conn

    class Tracked(_Conn):
        __slots__ = ("aborted",)

        def __init__(self, o):
            super().__init__(o)
            self.aborted = False

        def abort(self):
            self.aborted = True
            self.closed = True

    async def go():
        c = H1Client(timeout_s=5, max_per_host=2)
        o = c._origin("http://127.0.0.1:9")
        o.open = 2  # full: two busy connections
        loop = asyncio.get_running_loop()
        deadline = loop.time() + 5
        retry = asyncio.ensure_future(c._acquire(o, deadline, fresh=True))
        await asyncio.sleep(0)
        others = [asyncio.ensure_future(c._acquire(o, deadline)) for _ in range(4)]
        await asyncio.sleep(0)
        connects = []

        async def connect(o_, d, infos=None):
            o_.open += 1
            connects.append(1)
            return "fresh"
        c._connect = connect
        conns = []
        t0 = loop.time()
        for _ in range(2):  # the two busy connections finish; each is released healthy
            used = Tracked(o)
            used.uses = 5
            conns.append(used)
            c._release(used, True)
            await asyncio.sleep(0)
            await asyncio.sleep(0)
        got = await asyncio.wait_for(retry, 1)
        took = loop.time() - t0
        served = [x for x in others if x.done()]
        for x in others:
            x.cancel()
        await c.close()
        return got, took, conns, served, connects, o.open
    got, took, conns, served, connects, open_ = run(go())
    assert got == "fresh" and took < 0.5 and len(connects) == 1
    assert not conns[0].aborted and conns[1].aborted  # passed on once, then its slot was taken
    assert len(served) == 1 and served[0].result() is conns[0]
    assert open_ == 2  # one kept by the other request, one the retry's own
