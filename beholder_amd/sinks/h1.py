"""Keep-alive HTTP/1.1 client for the sinks (default production client).

The reference's outbound calls (index.js:53,83,99,112) go through ``request``.
The service makes one of these per Trello-created progress event, so the
client's per-request CPU bounds production throughput. aiohttp costs about
140 µs of CPU per request on this host. This client is an ``asyncio.Protocol``
per connection. Response framing is done by the native ``H1Parser``
(``ops/csrc/py_http.cpp``), and connections are pooled per origin with
keep-alive. A request costs one ``write`` and one ``data_received`` callback.

Semantics that match ``request`` (the library behind the reference):

* redirects are followed for GET/HEAD only (``followRedirect``; at most 10);
* bodies are not decompressed (no ``Accept-Encoding`` is sent);
* the query string is passed through unmodified (``encodeURIComponent``
  encoding, see :func:`.http.with_query`).

Additions over the reference:

* keep-alive pooling: at most ``max_per_host`` connections per origin, and
  idle connections expire after ``keepalive_s``;
* connect admission: at most ``max_connecting`` connects (TCP + TLS handshake) in
  progress per origin. A request that finds no idle connection and no free connect
  slot queues, and takes whichever comes first: a keep-alive connection released by
  another request, or a connect slot. A burst of first requests after start (prefetch
  100 deliveries at once) therefore shares a few fresh connections instead of running
  ~100 handshakes at once, which made every one of them slow (the warm-up tail);
* one transparent retry on a fresh connection when a *reused* idle connection
  dies before any response byte arrives. This applies to idempotent methods only,
  so a POST (a Trello comment) is never sent twice;
* a per-request deadline that covers connect, TLS, request and response;
* :meth:`H1Client.preconnect` opens connections ahead of the first requests
  (``service.http.preconnect``; one name lookup per batch);
* HTTP proxies (``HTTP_PROXY``) are not supported.
"""
from __future__ import annotations

import asyncio
import base64
import collections
import functools
import ipaddress
import socket
import ssl as _ssl
import time
from typing import Deque, Dict, Optional, Tuple
from urllib.parse import quote, unquote, urljoin

from ..ops import H1Parser
from ..ops import IOFuture as _IOFuture
from ..ops import encode_query as _encode_query
from ..ops import native as _native

_netconn_connect = _native.netconn_connect
from ..utils import netconn
from .http import HttpClient, HttpError, HttpResponse, encode_query, redact, with_query

_IDEMPOTENT = frozenset(("GET", "HEAD", "PUT", "DELETE", "OPTIONS"))
_BODY_METHODS = frozenset(("POST", "PUT", "PATCH", "DELETE"))
_REDIRECTS = frozenset((301, 302, 303, 307, 308))
_TICK = 0.05  # deadline sweep period (s): timeouts fire at most this late
_PATH_SAFE = "".join(chr(c) for c in range(0x21, 0x7F) if chr(c) not in '"<>\\^`{|}')


def _is_token_text(s: str) -> bool:
    """Every character in 0x21-0x7E (printable ASCII, no space): safe in a request line."""
    return s.isascii() and s.isprintable() and " " not in s


class _Reset(Exception):
    """The connection closed before the response completed (``started``: bytes of it seen)."""

    def __init__(self, started: bool, detail: str = ""):
        super().__init__(detail or "socket hang up")
        self.started = started


class _Conn(asyncio.Protocol):
    """One keep-alive connection. Normally its socket is a native ``NetConn`` (``net``) that
    connected it (and runs its TLS) in C (``ops netconn_connect``): replies are parsed and
    delivered in C and the methods below only see its rare paths (``_net_lost``,
    ``_net_error``). With native connections off, or a caller-supplied ``ssl.SSLContext``, it
    is an asyncio protocol on an ordinary transport."""

    __slots__ = ("origin", "parser", "transport", "waiter", "closed", "last_used", "uses", "deadline", "what",
                 "net")

    def __init__(self, origin: "_Origin"):
        self.origin = origin
        self.parser = H1Parser()
        self.transport = None
        self.net = None
        self.waiter: Optional[asyncio.Future] = None
        self.closed = False
        self.last_used = 0.0
        self.uses = 0
        self.deadline = 0.0
        self.what = ("", "")

    # -- protocol callbacks (asyncio transports: BEHOLDER_NATIVE_IO=0, caller-supplied TLS) ------
    def connection_made(self, transport):
        self.transport = transport

    def data_received(self, data):
        try:
            r = self.parser.feed(data)
        except ValueError as e:
            self._fail(HttpError(f"HPE_INVALID_RESPONSE: {e}"))
            self.abort()
            return
        if r is not None:
            w = self.waiter
            self.waiter = None
            if w is None or w.done():
                self.abort()  # unsolicited response
            else:
                w.resolve(r)  # a handler waiting on it (native Driver) resumes right here

    def eof_received(self):
        return False  # let the transport close; connection_lost completes the response

    def connection_lost(self, exc):
        if self.net is not None:
            return  # the transport was aborted when the socket was handed to the NetConn
        self.closed = True
        w = self.waiter
        self.waiter = None
        self._complete_at_eof(w, exc)

    # -- NetConn callbacks (rare paths) ----------------------------------------
    def _net_lost(self, exc):
        self.closed = True
        self._complete_at_eof(self.net.take_waiter(), exc)

    def _net_error(self, exc):
        if exc is not None:
            self._fail(HttpError(f"HPE_INVALID_RESPONSE: {exc}"))
        self.abort()  # malformed or unsolicited response

    def _complete_at_eof(self, w, exc) -> None:
        if w is None or w.done():
            return
        try:
            r = self.parser.eof()
        except ValueError as e:
            w.set_exception(_Reset(True, f"socket hang up ({e})"))
            return
        if r is not None:
            w.set_result(r)
        else:
            w.set_exception(_Reset(False, f"ECONNRESET: {exc}" if exc else "socket hang up"))

    # -- client side ---------------------------------------------------------
    def _fail(self, exc: BaseException) -> None:
        if self.net is not None:
            w = self.net.take_waiter()
        else:
            w = self.waiter
            self.waiter = None
        if w is not None and not w.done():
            w.set_exception(exc)

    def abort(self) -> None:
        self.closed = True
        if self.net is not None:
            self.net.abort()
        elif self.transport is not None:
            self.transport.abort()

    def timed_out(self) -> None:
        m, url = self.what
        self._fail(HttpError(f"ETIMEDOUT: {m} {redact(url)}"))
        self.abort()


class _Origin:
    __slots__ = ("scheme", "host", "port", "tls", "host_header", "auth", "idle", "open", "waiters", "connecting",
                 "queued_at")

    def __init__(self, scheme: str, host: str, port: int, host_header: str, auth: Optional[str]):
        self.scheme = scheme
        self.host = host
        self.port = port
        self.tls = scheme == "https"
        self.host_header = host_header
        self.auth = auth
        self.idle: Deque[_Conn] = collections.deque()
        self.open = 0
        self.connecting = 0  # connects (and TLS handshakes) in progress
        self.waiters: Deque[asyncio.Future] = collections.deque()
        # monotonic ns at which each waiter queued (the queue-wait histogram); an entry leaves with
        # its waiter, whichever path pops it from ``waiters``
        self.queued_at: Dict[object, int] = {}


def _sockaddr_host(sa) -> str:
    """The address of a getaddrinfo sockaddr; a scoped IPv6 one (link-local, scope id in the 4th
    field) keeps its scope as ``addr%<id>``, which routes it to asyncio's connect."""
    if len(sa) == 4 and sa[3]:
        return f"{sa[0]}%{sa[3]}"
    return sa[0]


def _queued(o: _Origin) -> bool:
    """More requests of ``o`` wait for a connection than connects are in progress for them.
    Finished waiters (timed out, cancelled) are dropped from the front as they are met, so this is
    O(1) amortised: it runs once per queued request, and the first burst queues ~100 at once (a
    count over the whole queue cost ~1.4 ms of loop time there). One finished further back is
    still counted until it reaches the front: at worst a connect starts early, still capped by
    ``max_connecting``."""
    w = o.waiters
    while w and w[0].done():
        o.queued_at.pop(w.popleft(), None)
    return len(w) > o.connecting


_DNS_REUSE_S = 1.0  # a successful name lookup serves the connects of the next second too


def _expire(w) -> None:
    """A queued request's deadline: its waiter fails with TimeoutError unless it was served."""
    if not w.done():
        w.set_exception(asyncio.TimeoutError())


def _split_url(url: str) -> Tuple[str, str]:
    """``(scheme://authority, target)``; target keeps path + query, drops the fragment."""
    i = url.find("://")
    if i <= 0:
        raise HttpError(f"Invalid URI \"{redact(url)}\"")
    k = url.find("/", i + 3)
    if k < 0:
        k = len(url)
    q = url.find("?", i + 3, k)
    if q >= 0:
        k = q
    h = url.find("#", i + 3, k)
    if h >= 0:
        k = h
    target = url[k:]
    if "#" in target:
        target = target[:target.index("#")]
    if not target.startswith("/"):
        target = "/" + target
    return url[:k], target


class H1Client(HttpClient):
    """Pooled keep-alive HTTP/1.1 (+TLS) client. See the module docstring."""

    def __init__(self, timeout_s: float = 30.0, user_agent: str = "beholder/1.0", max_per_host: int = 100,
                 keepalive_s: float = 4.0, ssl_context: Optional[_ssl.SSLContext] = None,
                 max_redirects: int = 10, ssl_cafile: Optional[str] = None, max_connecting: int = 8):
        self.timeout_s = float(timeout_s)
        self.user_agent = user_agent
        self.max_per_host = max(1, int(max_per_host))
        self.max_connecting = max(1, int(max_connecting))
        self.keepalive_s = float(keepalive_s)
        self.max_redirects = int(max_redirects)
        self._own_ssl = ssl_context is None  # our own context: the native TLS path can mirror it
        if ssl_context is None and ssl_cafile:
            ssl_context = _ssl.create_default_context(cafile=ssl_cafile)
        self._ssl = ssl_context
        self.ssl_cafile = ssl_cafile
        self._ntls = None
        self._literal: Dict[str, list] = {}  # hosts that are IP literals: no resolver call
        # name lookups per (host, port), in flight or finished within _DNS_REUSE_S: the connects of
        # a burst share one
        self._resolving: Dict[Tuple[str, int], Tuple[asyncio.Future, float]] = {}
        self._origins: Dict[str, _Origin] = {}
        self._routes: Dict[str, Tuple[_Origin, str, str]] = {}
        self._closed = False
        self._busy: set = set()
        self._dials: set = set()  # background connects for queued requests (_grow)
        self._sweeper = None
        # capability for callers in C (the compiled handlers): the native request path when it is on
        self.native_call = _NATIVE_CALL if netconn.enabled() else None
        self._tail = f"User-Agent: {user_agent}\r\n\r\n".encode("latin-1")
        self._tail_cl0 = f"User-Agent: {user_agent}\r\nContent-Length: 0\r\n\r\n".encode("latin-1")
        self.counts = {"requests": 0, "connections": 0, "reused": 0, "retries": 0, "errors": 0, "timeouts": 0,
                       "connecting_peak": 0, "connect_waits": 0}
        # where a cold pool's time goes (the warm-up tail): each successful connect (+ TLS
        # handshake), and each wait of a queued request until a connection was handed to it
        self.dial_ns = _native.Histogram()
        self.queue_wait_ns = _native.Histogram()

    # -- pool ----------------------------------------------------------------
    def _origin(self, key: str) -> _Origin:
        o = self._origins.get(key)
        if o is not None:
            return o
        scheme, _, authority = key.partition("://")
        if not _is_token_text(authority):  # CR/LF/SP would end up in the Host line
            raise HttpError(f"Invalid URI \"{redact(key)}\"")
        scheme = scheme.lower()
        if scheme not in ("http", "https"):
            raise HttpError(f"Invalid protocol: {scheme}:")
        auth = None
        if "@" in authority:
            userinfo, authority = authority.rsplit("@", 1)
            auth = "Basic " + base64.b64encode(unquote(userinfo).encode("utf-8")).decode("ascii")
        if authority.startswith("["):
            e = authority.find("]")
            if e < 0:
                raise HttpError(f"Invalid URI \"{redact(key)}\"")
            host, rest = authority[1:e], authority[e + 1:]
            port_s = rest[1:] if rest.startswith(":") else ""
        else:
            host, _, port_s = authority.partition(":")
        if not host:
            raise HttpError(f"Invalid URI \"{redact(key)}\"")
        try:
            port = int(port_s) if port_s else (443 if scheme == "https" else 80)
        except ValueError:
            raise HttpError(f"Invalid URI \"{redact(key)}\"") from None
        if not 0 < port < 65536:
            raise HttpError(f"Invalid URI \"{redact(key)}\"")
        o = _Origin(scheme, host, port, authority, auth)
        self._origins[key] = o
        return o

    def _native_tls(self):
        """The native TLS context (ops TlsContext) mirroring this client's own SSL context: the
        default one or the one built from ``ssl_cafile``. None for a caller-supplied
        ``ssl_context`` (its settings cannot be mirrored) or with native connections off."""
        t = self._ntls
        if t is None:
            t = False
            if self._own_ssl and netconn.enabled():
                t = _native.TlsContext(cafile=self.ssl_cafile)
            self._ntls = t
        return t or None

    def prepare_tls(self) -> bool:
        """Make the TLS context now (the service calls this at startup when a sink is HTTPS): the
        native context's one-time OpenSSL warm-up handshake (~6 ms) and the start of its
        handshake threads then happen before the first delivery, not inside the first connect.
        True when the native TLS path will be used."""
        if self._own_ssl and netconn.enabled():
            return self._native_tls() is not None
        self._ssl_context()
        return False

    def _ssl_context(self) -> _ssl.SSLContext:
        if self._ssl is None:
            self._ssl = _ssl.create_default_context()
        return self._ssl

    def _reserve(self, o: _Origin) -> None:
        """Count a connect about to start against the pool (``open``) and admission (``connecting``)."""
        o.open += 1
        o.connecting += 1
        if o.connecting > self.counts["connecting_peak"]:
            self.counts["connecting_peak"] = o.connecting

    async def _connect(self, o: _Origin, deadline: float, infos=None) -> _Conn:
        """A connection for the caller itself (preconnect, the retry of a dead reused connection)."""
        self._reserve(o)
        try:
            return await self._dial(o, deadline, infos)
        except BaseException:
            self._wake(o)
            raise

    async def _dial(self, o: _Origin, deadline: float, infos=None) -> _Conn:
        """Connect (+ TLS) on a slot :meth:`_reserve` counted; frees the slot either way."""
        loop = asyncio.get_running_loop()
        conn = _Conn(o)
        t0 = time.monotonic_ns()
        try:
            remaining = deadline - loop.time()
            if remaining <= 0:
                raise asyncio.TimeoutError
            ntls = self._native_tls() if o.tls else None
            if netconn.enabled() and (ntls is not None or not o.tls):
                await self._connect_native(conn, o, ntls, deadline, loop, infos)
            else:  # asyncio transport: native connections off, or a caller-supplied ssl.SSLContext
                kw = {"ssl": self._ssl_context(), "server_hostname": o.host} if o.tls else {}
                await asyncio.wait_for(loop.create_connection(lambda: conn, o.host, o.port, **kw), remaining)
        except BaseException:
            conn.abort()
            o.open -= 1
            o.connecting -= 1
            raise
        o.connecting -= 1
        self.counts["connections"] += 1
        self.dial_ns.record(time.monotonic_ns() - t0)
        return conn

    def _grow(self, o: _Origin, deadline: float) -> None:
        """Start a background connect for the queued requests of ``o`` if a pool slot and a connect
        slot are free. The new connection goes to whichever request is first in the queue when it is
        ready (or to the idle pool); a request never waits on one particular handshake."""
        if self._closed or o.open >= self.max_per_host or o.connecting >= self.max_connecting:
            return
        self._reserve(o)
        t = asyncio.ensure_future(self._dial_for_queue(o, deadline))
        self._dials.add(t)
        t.add_done_callback(self._dials.discard)

    async def _dial_for_queue(self, o: _Origin, deadline: float) -> None:
        try:
            c = await self._dial(o, deadline)
        except asyncio.CancelledError:  # client closing
            self._wake(o)
            return
        except asyncio.TimeoutError:  # the queued requests time out on their own deadlines
            if _queued(o):
                self._grow(o, asyncio.get_running_loop().time() + self.timeout_s)
            return
        except BaseException as e:  # noqa: BLE001 - the first queued request gets the connect error
            while o.waiters:
                w = o.waiters.popleft()
                o.queued_at.pop(w, None)
                if not w.done():
                    w.set_exception(e)
                    break
            if _queued(o):
                self._grow(o, asyncio.get_running_loop().time() + self.timeout_s)
            return
        self._release(c, True)
        if _queued(o):  # a queue longer than the connects under way: the pool grows (max_connecting at a time)
            self._grow(o, asyncio.get_running_loop().time() + self.timeout_s)

    def _lookup(self, o: _Origin, loop) -> asyncio.Future:
        """``getaddrinfo`` of ``o``, shared by every connect that needs it while it runs and for
        ``_DNS_REUSE_S`` after it succeeded: the first burst after start (or after the keep-alive
        connections expired) opens connections in waves of ``max_connecting``, which would
        otherwise make one identical lookup each (a resolver query on an executor thread). Each
        caller still waits only up to its own deadline (the lookup is shielded from a caller's
        timeout). A failed lookup is not reused."""
        key = (o.host, o.port)
        hit = self._resolving.get(key)
        if hit is not None:
            f, until = hit
            if not f.done() or (loop.time() < until and not f.cancelled() and f.exception() is None):
                return f
        f = asyncio.ensure_future(loop.getaddrinfo(o.host, o.port, type=socket.SOCK_STREAM))
        self._resolving[key] = (f, float("inf"))
        f.add_done_callback(functools.partial(self._lookup_done, key, loop))
        if len(self._resolving) > 256:  # stale entries of many origins: keep the map small
            now = loop.time()
            for k in [k for k, (x, t) in self._resolving.items() if x.done() and t <= now]:
                del self._resolving[k]
        return f

    def _lookup_done(self, key, loop, f) -> None:
        cur = self._resolving.get(key)
        if cur is None or cur[0] is not f:
            return
        if f.cancelled() or f.exception() is not None:  # retrieved: not logged as lost; not reused
            del self._resolving[key]
        else:
            self._resolving[key] = (f, loop.time() + _DNS_REUSE_S)

    async def _connect_native(self, conn: _Conn, o: _Origin, ntls, deadline: float, loop, infos=None) -> None:
        """TCP connect, and TLS for ``ntls``, in C (``ops netconn_connect``): no asyncio transport
        is made and dropped. Addresses are tried in order, as ``loop.create_connection`` does
        (an IP literal as is, a name through ``loop.getaddrinfo`` unless ``infos`` carries the
        addresses already); a TLS failure is final."""
        if infos is None:
            infos = self._literal.get(o.host)
        if infos is None:
            try:
                ipaddress.ip_address(o.host)
                infos = self._literal[o.host] = [o.host]
            except ValueError:  # a name: resolved within the request's deadline, like create_connection
                found = await asyncio.wait_for(asyncio.shield(self._lookup(o, loop)), deadline - loop.time())
                infos = [_sockaddr_host(ai[4]) for ai in found]
        errors = []
        for ip in infos:
            remaining = deadline - loop.time()
            if remaining <= 0:
                raise asyncio.TimeoutError
            if "%" in ip:  # a scoped (link-local) IPv6 address: inet_pton cannot take it, asyncio can
                try:
                    kw = {"ssl": self._ssl_context(), "server_hostname": o.host} if o.tls else {}
                    await asyncio.wait_for(loop.create_connection(lambda: conn, ip, o.port, **kw), remaining)
                    return
                except OSError as e:
                    errors.append(e)
                    continue
            try:
                net = _netconn_connect(ip, o.port, loop, "h1", conn, conn.parser, tls=ntls, server_hostname=o.host,
                                       port=o.port, tls_error=_tls_error)
            except (OSError, ValueError) as e:  # ValueError: an address the native connect cannot parse
                errors.append(e if isinstance(e, OSError) else OSError(str(e)))
                continue
            conn.net = net
            try:
                await asyncio.wait_for(net.handshake, remaining)
                return
            except _ssl.SSLError:
                raise
            except OSError as e:
                net.abort()
                conn.net = None
                errors.append(e)
        if not errors:
            raise OSError(f"getaddrinfo returned no addresses for {o.host}")
        if len(errors) == 1 or all(str(e) == str(errors[0]) for e in errors):
            raise errors[0]
        raise OSError("Multiple exceptions: " + ", ".join(str(e) for e in errors))

    async def _acquire(self, o: _Origin, deadline: float, fresh: bool = False, front: bool = False) -> _Conn:
        """A connection for a request of ``o``: a live idle one, else the first released or newly
        made one (queued; ``front``: at the head of the queue, for a request that had its place
        already)."""
        counts = self.counts
        idle = o.idle
        loop = asyncio.get_running_loop()
        passed_on = False  # a fresh retry passes a healthy connection on to another request only once
        while True:
            now = time.monotonic()
            while idle and not fresh:
                c = idle.pop()
                if not c.closed and now - c.last_used < self.keepalive_s:
                    counts["reused"] += 1
                    return c
                self._drop(c)
            if fresh and o.open < self.max_per_host:
                # the retry of a request whose reused connection died: a connection of its own
                return await self._connect(o, deadline)
            # queue: take the first connection released by another request or made by a background
            # connect (started here when admission allows), whichever is ready first
            w = loop.create_future()
            if front:
                o.waiters.appendleft(w)
            else:
                o.waiters.append(w)
                counts["connect_waits"] += 1
            o.queued_at[w] = time.monotonic_ns()
            if not fresh and _queued(o):
                self._grow(o, deadline)
            th = loop.call_at(deadline, _expire, w)
            try:
                c = await w
            except asyncio.CancelledError:
                o.queued_at.pop(w, None)
                # a connection handed over just before the cancel must go back to the pool
                if w.done() and not w.cancelled() and w.exception() is None and w.result() is not None:
                    self._release(w.result(), True)
                raise
            except BaseException:  # its deadline, a failed background connect
                o.queued_at.pop(w, None)
                raise
            finally:
                th.cancel()
            if c is None:  # a pool slot was freed: look again, keeping this request's place
                front = True
                continue
            if not c.closed and not (fresh and c.uses):
                if c.uses:
                    counts["reused"] += 1
                return c
            if not fresh:
                self._drop(c)  # closed meanwhile: its slot goes to the next waiter; this one queues again
            elif not c.closed and not passed_on and any(not x.done() for x in o.waiters):
                # a healthy keep-alive connection, but this retry needs a fresh one: another queued
                # request takes it (no connect + handshake thrown away); this one keeps its place.
                # Once only: at max_per_host nothing else ever frees a slot while requests queue, so
                # passing every connection on would starve the retry until its deadline
                self._release(c, True)
                passed_on = True
            else:
                # closed meanwhile, nobody else to take it, or one passed on already: the slot is this
                # retry's, for its own connect at the top of the loop (no other waiter is woken for it)
                c.abort()
                o.open -= 1
            front = True

    async def preconnect(self, url: str, n: int) -> Tuple[int, Optional[BaseException]]:
        """Open up to ``n`` connections to ``url``'s origin at once (never past ``max_per_host``)
        and park them idle, so the first burst of requests after start reuses them instead of
        each paying a connect (and TLS handshake) inside its handle latency. Connections left
        unused for ``keepalive_s`` are dropped at the next acquire, as any idle one is."""
        if self._closed or n <= 0:
            return 0, None
        o = self._origin(_split_url(url)[0])
        want = min(int(n), self.max_per_host - o.open)
        if want <= 0:
            return 0, None
        loop = asyncio.get_running_loop()
        deadline = loop.time() + self.timeout_s
        infos = None
        if netconn.enabled() and o.host not in self._literal:
            try:
                ipaddress.ip_address(o.host)
            except ValueError:  # a name: one lookup for the whole batch, not one per connection
                try:
                    found = await asyncio.wait_for(asyncio.shield(self._lookup(o, loop)),
                                                   self.timeout_s)
                except (OSError, asyncio.TimeoutError) as e:
                    return 0, e
                infos = [_sockaddr_host(ai[4]) for ai in found]
        got = await asyncio.gather(*(self._connect(o, deadline, infos) for _ in range(want)), return_exceptions=True)
        opened, err = 0, None
        for c in got:
            if isinstance(c, BaseException):
                err = err or c
            else:
                self._release(c, True)
                opened += 1
        return opened, err

    def touch_idle(self) -> int:
        """Restart the keep-alive clock of every idle connection (the service calls this when it
        starts consuming, so preconnected connections are not dropped for the time startup took).
        Connections still unused ``keepalive_s`` after that are dropped at the next acquire, as
        any idle one is: preconnect pays off when traffic starts within ``keepalive_s``."""
        now = time.monotonic()
        n = 0
        for o in self._origins.values():
            for c in o.idle:
                if not c.closed:
                    c.last_used = now
                    n += 1
        return n

    def _release(self, c: _Conn, keep: bool) -> None:
        o = c.origin
        if not keep or c.closed or self._closed:
            self._drop(c)
            return
        c.last_used = time.monotonic()
        while o.waiters:
            w = o.waiters.popleft()
            t0 = o.queued_at.pop(w, None)
            if not w.done():
                if t0 is not None:
                    self.queue_wait_ns.record(time.monotonic_ns() - t0)
                w.set_result(c)
                return
        o.idle.append(c)

    def _drop(self, c: _Conn) -> None:
        c.abort()
        o = c.origin
        o.open -= 1
        self._wake(o)

    def _wake(self, o: _Origin) -> None:
        while o.waiters:
            w = o.waiters.popleft()
            o.queued_at.pop(w, None)  # it queues again (keeping its place) or connects itself
            if not w.done():
                w.set_result(None)  # a slot is free: the waiter opens its own connection (or queues again)
                return

    # -- deadlines -------------------------------------------------------------
    # One sweep timer per client instead of a TimerHandle per request: busy connections
    # carry their deadline and are checked every `_TICK` seconds while any is busy.
    def _arm(self, loop) -> None:
        self._sweeper = loop.call_later(_TICK, self._sweep, loop)

    def _sweep(self, loop) -> None:
        self._sweeper = None
        now = loop.time()
        for c in [c for c in self._busy if c.deadline <= now]:
            self._busy.discard(c)
            self.counts["timeouts"] += 1
            c.timed_out()
        if self._busy and not self._closed:
            self._arm(loop)

    # -- request -------------------------------------------------------------
    def _resolve(self, url: str) -> Tuple[_Origin, str, str]:
        """``(origin, request target, rest of the request line + Host/Authorization lines)``."""
        key, target = _split_url(url)
        o = self._origin(key)
        if not _is_token_text(target):
            # any byte outside 0x21-0x7E is percent-encoded: a CR/LF in a DB-sourced path
            # segment (Trello's /1/cards/{creatorId}) must not split the request
            target = quote(target, safe=_PATH_SAFE)
        rest = f" HTTP/1.1\r\nHost: {o.host_header}\r\n"
        if o.auth:
            rest += f"Authorization: {o.auth}\r\n"
        return o, target, rest

    def _route(self, url: str) -> Tuple[_Origin, str, str]:
        """:meth:`_resolve` of a URL without query or fragment, cached per client (a sink calls
        a handful of base URLs; the per-event part rides in ``params``)."""
        r = self._routes.get(url)
        if r is None:
            r = self._resolve(url)
            if len(self._routes) >= 4096:
                self._routes.clear()
            self._routes[url] = r
        return r

    def _prepare(self, url: str, params) -> Tuple[str, _Origin, str, str]:
        """``(full URL, *_resolve(full URL))`` for ``url`` + ``params``."""
        if "?" in url or "#" in url:
            # the fragment stays on this side (it is never sent), so the parameters join the query
            # before it, as Node's url.parse + request put them; appended after it, they were
            # dropped with it
            h = url.find("#")
            if h < 0:
                full = with_query(url, params)
                return (full, *self._resolve(full))
            sent = with_query(url[:h], params)
            return (sent + url[h:], *self._resolve(sent))
        # the sinks' shape: a cached route + an encodeURIComponent query (ASCII, no spaces: the
        # quoting of _resolve would leave it as is)
        o, target, rest = self._route(url)
        q = _encode_query(params) if type(params) is dict and params else encode_query(params)
        if q:
            return f"{url}?{q}", o, f"{target}?{q}", rest
        return url, o, target, rest

    def request(self, method, url, *, params=None, timeout=None):
        """Awaitable :class:`HttpResponse`. For a stock client this is a native ``H1Call``
        (``ops/csrc/py_h1call.cpp``): like a coroutine it does nothing until awaited; then, on a
        warm pool, it sends the request and completes a plain reply in C, and in every other
        case it delegates to :meth:`_request`."""
        nc = self.native_call
        if nc is not None:
            call = nc(self, method, url, params, timeout)
            if call is not None:
                return call
        return self._request(method, url, params, timeout)

    async def _request(self, method, url, params, timeout) -> HttpResponse:
        if self._closed:
            raise HttpError("client closed")
        m = method.upper()
        full, o, target, rest = self._prepare(url, params)
        loop = asyncio.get_running_loop()
        deadline = loop.time() + (timeout or self.timeout_s)
        self.counts["requests"] += 1
        return await self._exchange(m, full, o, target, rest, deadline, None, None, False, None)

    async def _resume(self, m, full, deadline, c, w, reused, thrown) -> HttpResponse:
        """The native fast path sent ``m full`` on the pooled connection ``c``. The reply future
        ``w`` holds an error or a redirect, or ``thrown`` was thrown in at the await (a Task
        waking on a failed or cancelled ``w``): the request loop continues from its await."""
        o, target, rest = self._resolve(full)
        return await self._exchange(m, full, o, target, rest, deadline, c, w, reused, thrown)

    def _enqueue(self, o: _Origin, deadline: float, w, front: bool = False):
        """The native fast path (``ops h1_fast``) found no idle connection: queue its waiter ``w``
        as :meth:`_acquire` does (same accounting, background connects, deadline), without the
        request loop's coroutines. Returns the deadline timer (the caller cancels it).

        ``front``: the request continues an event whose earlier sink request has completed (the
        compiled handlers mark an event's second and later requests). It waits at the head of the
        queue: in a burst (the first deliveries after start, or a pool at ``max_per_host``) a
        status event's move / hook requests would otherwise queue behind every newer delivery's
        first request, once per request, and set the tail of the handle latency."""
        if front:
            o.waiters.appendleft(w)
        else:
            o.waiters.append(w)
        o.queued_at.setdefault(w, time.monotonic_ns())
        self.counts["connect_waits"] += 1
        if _queued(o):
            self._grow(o, deadline)
        return asyncio.get_running_loop().call_at(deadline, _expire, w)

    async def _after_queue(self, m, full, deadline, got) -> HttpResponse:
        """A natively queued request (:meth:`_enqueue`) was handed no live connection: a freed pool
        slot (None), a connection that closed meanwhile, the client closing, or an error (its
        deadline, a failed background connect). The request loop continues as :meth:`_acquire`
        and :meth:`_exchange` would have, keeping the request's place in the queue."""
        o, target, rest = self._resolve(full)
        counts = self.counts
        if isinstance(got, BaseException):  # as _exchange maps what its _acquire raised
            if isinstance(got, asyncio.TimeoutError):
                counts["timeouts"] += 1
                counts["errors"] += 1
                raise HttpError(f"ETIMEDOUT: {m} {redact(full)}") from None
            if isinstance(got, OSError):
                counts["errors"] += 1
                raise HttpError(_connect_error(got, o)) from None
            raise got
        if self._closed:
            if got is not None:
                self._release(got, False)
            counts["errors"] += 1
            raise HttpError("client closed")
        if got is not None and got.closed:
            self._drop(got)
            got = None
        return await self._exchange(m, full, o, target, rest, deadline, None, None, False, None, front=True,
                                    conn=got)

    async def _exchange(self, m, full, o, target, rest, deadline, c, w, reused, thrown,
                        front: bool = False, conn: Optional[_Conn] = None) -> HttpResponse:
        """Send on a pooled connection, await the reply; one transparent retry on a fresh
        connection for an idempotent request whose reused connection died before any response
        byte; redirects for GET/HEAD. ``c``/``w``/``reused``: a request already on the wire;
        ``thrown``: what its await raised."""
        counts = self.counts
        loop = asyncio.get_running_loop()
        cur = full
        redirects = 0
        fresh = False
        while True:
            if w is None:
                req = f"{m} {target}{rest}".encode("latin-1") + (self._tail_cl0 if m in _BODY_METHODS else self._tail)
                c = None
                if conn is not None:  # handed to a natively queued request (_after_queue)
                    c, conn = conn, None
                    if c.uses:
                        counts["reused"] += 1
                elif not fresh:  # fast path of _acquire: a live idle keep-alive connection, no await
                    idle = o.idle
                    if idle:
                        now = time.monotonic()
                        while idle:
                            cand = idle.pop()
                            if not cand.closed and now - cand.last_used < self.keepalive_s:
                                counts["reused"] += 1
                                c = cand
                                break
                            self._drop(cand)
                try:
                    if c is None:
                        c = await self._acquire(o, deadline, fresh, front)
                        front = False
                        if self._closed:  # closed while this request connected or waited for a slot
                            self._release(c, False)
                            counts["errors"] += 1
                            raise HttpError("client closed")
                except asyncio.TimeoutError:
                    counts["timeouts"] += 1
                    counts["errors"] += 1
                    raise HttpError(f"ETIMEDOUT: {m} {redact(cur)}") from None
                except OSError as e:
                    counts["errors"] += 1
                    raise HttpError(_connect_error(e, o)) from None
                reused = c.uses > 0
                c.uses += 1
                w = _IOFuture(loop)
                c.deadline = deadline
                c.what = (m, cur)
                net = c.net
                if net is not None:
                    net.request(req, w, m == "HEAD")  # parser started, reply future set, request sent
                else:
                    c.waiter = w
                    c.parser.start(head=m == "HEAD")
                    c.transport.write(req)
                busy = self._busy
                busy.add(c)
                if self._sweeper is None:
                    self._arm(loop)
            busy = self._busy
            try:
                if thrown is not None:
                    e, thrown = thrown, None
                    raise e
                status, _reason, raw, body, keep = await w
            except _Reset as e:
                self._release(c, False)
                if reused and not e.started and m in _IDEMPOTENT and not fresh:
                    counts["retries"] += 1
                    fresh = True
                    w = None
                    continue
                counts["errors"] += 1
                raise HttpError(f"{e}: {m} {redact(cur)}") from None
            except HttpError:
                self._release(c, False)
                counts["errors"] += 1
                raise
            except BaseException:
                self._release(c, False)  # cancelled mid-request: the connection state is unknown
                raise
            finally:
                busy.discard(c)
            w = None
            self._release(c, keep and c.parser.buffered == 0)
            if status in _REDIRECTS and m in ("GET", "HEAD"):
                loc = _header(raw, b"location")
                if loc is not None:
                    redirects += 1
                    if redirects > self.max_redirects:
                        counts["errors"] += 1
                        raise HttpError(f"Exceeded maxRedirects. Probably stuck in a redirect loop {redact(cur)}")
                    cur = urljoin(cur, loc)
                    o, target, rest = self._resolve(cur)
                    fresh = False
                    continue
            return HttpResponse(status, body, None, full, raw)

    def stats(self) -> Dict[str, int]:
        out = dict(self.counts)
        out["open"] = sum(o.open for o in self._origins.values())
        out["idle"] = sum(len(o.idle) for o in self._origins.values())
        for name, h in (("dial", self.dial_ns), ("queue_wait", self.queue_wait_ns)):
            if h.count:
                out[f"{name}_p99_us"] = round(h.percentile(99) / 1e3, 1)
                out[f"{name}_max_us"] = round(h.percentile(100) / 1e3, 1)
        if self._ntls:  # native TLS: full and resumed handshakes (beholder_pool{pool="http"})
            t = self._ntls.stats
            out["tls_handshakes"] = t["handshakes"]
            out["tls_resumed"] = t["resumed"]
        return out

    async def close(self) -> None:
        self._closed = True
        for t in list(self._dials):
            t.cancel()
        if self._sweeper is not None:
            self._sweeper.cancel()
            self._sweeper = None
        # requests waiting for a reply end now (with the sweeper gone nothing would time them out);
        # each request's own path then drops its connection
        for c in list(self._busy):
            self._busy.discard(c)
            c._fail(HttpError("client closed"))
            c.abort()
        for o in self._origins.values():
            while o.idle:
                self._drop(o.idle.pop())
            o.queued_at.clear()
            while o.waiters:
                w = o.waiters.popleft()
                if not w.done():
                    w.set_exception(HttpError("client closed"))


def _header(raw: bytes, name: bytes) -> Optional[str]:
    for line in raw.split(b"\r\n"):
        k, sep, v = line.partition(b":")
        if sep and k.strip().lower() == name:
            return v.strip().decode("latin-1")
    return None


def _connect_error(e: OSError, o: "_Origin") -> str:
    """Node-style messages (what the reference logs via err.message): ``getaddrinfo ENOTFOUND
    host``, ``connect ECONNREFUSED host:port``; TLS failures keep OpenSSL's reason."""
    import errno
    import socket
    if isinstance(e, _ssl.SSLError):
        return e.reason or type(e).__name__
    if isinstance(e, socket.gaierror):
        return f"getaddrinfo ENOTFOUND {o.host}"
    name = errno.errorcode.get(e.errno or 0) if e.errno else None
    return f"connect {name or type(e).__name__} {o.host}:{o.port}"


def _tls_error(reason: str, message: str, verify: bool) -> _ssl.SSLError:
    """A failed native TLS handshake as the ``ssl`` module would raise it (``reason`` is what
    :func:`_connect_error` reports, as for the asyncio TLS path)."""
    e = (_ssl.SSLCertVerificationError if verify else _ssl.SSLError)(1, message)
    e.reason = reason
    e.library = "SSL"
    return e


# Native fast path of H1Client.request (ops/csrc/py_h1call.cpp), handed to each client as its
# `native_call` capability. With BEHOLDER_NATIVE_IO=0 (replies on plain asyncio futures) every
# request takes the Python path.
# (The classes are registered either way: the in-process sink stub builds its responses with the
# same native code, ops/csrc_bench/recorder.cpp.)
_native.h1_setup(H1Client, _Conn, _Origin, HttpResponse)
if _IOFuture is _native.IOFuture:
    _NATIVE_CALL = _native.h1_fast
else:
    _native.h1_disable()
    _NATIVE_CALL = None
