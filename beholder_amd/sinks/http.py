"""Outbound HTTP clients for the sinks.

Two reference semantics matter (SURVEY.md §2.4 "Outbound HTTP"):

* ``request-promise-native`` (Telegram, Emby — index.js:99,112) **rejects on
  non-2xx** (``simple: true``): ``StatusCodeError: 500 - "body"``;
* the ``trello`` npm client (index.js:53,83) resolves with the body on *any*
  HTTP status and only rejects on transport errors.

``HttpClient.request`` returns an :class:`HttpResponse`; callers decide
whether a status is an error (:meth:`HttpResponse.raise_for_status`).

Query strings are encoded the way each reference client does it, so the URLs are byte-identical:

* Trello goes through ``restler`` and ``qs`` 1.2 (``yarn.lock:1665-1673``), which applies
  ``encodeURIComponent`` to every key and value;
* Telegram and Emby go through ``request``'s ``qs`` option, i.e. ``qs`` 6.5
  (``yarn.lock:1545-1548``), which uses RFC 3986 strict encoding: ``!'()*`` are escaped too.
  The sinks ask for it with ``rfc3986=True``;
* in both, a key whose value is ``undefined`` (``None`` here) is left out entirely.
"""
from __future__ import annotations

import abc
import asyncio
import collections
import json as _json
import re
import time
from typing import Any, Callable, Deque, Dict, List, Mapping, Optional, Tuple
from urllib.parse import quote

from .. import ops as _native_ops
from ..ops import encode_query as _native_encode_query

_SAFE = "-_.!~*'()"    # encodeURIComponent
_SAFE_RFC3986 = "-_.~"  # qs 6.x / RFC 3986 unreserved


def js_qs_value(v: Any) -> str:
    """``querystring.stringify`` value rendering (bool→'true', None→'', numbers JS-style)."""
    from ..utils.log import js_number
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return js_number(v)
    return str(v)


def py_encode_query(params: Optional[Mapping[str, Any]], rfc3986: bool = False) -> str:
    """Pure-Python reference for :func:`encode_query` (tests pin the native one to it)."""
    if not params:
        return ""
    safe = _SAFE_RFC3986 if rfc3986 else _SAFE
    return "&".join(f"{quote(str(k), safe=safe)}={quote(js_qs_value(v), safe=safe)}"
                    for k, v in params.items() if v is not None)


def encode_query(params: Optional[Mapping[str, Any]], rfc3986: bool = False) -> str:
    if not params:
        return ""
    if type(params) is not dict:
        params = dict(params)
    return _native_encode_query(params, rfc3986)


def with_query(url: str, params: Optional[Mapping[str, Any]], rfc3986: bool = False) -> str:
    q = encode_query(params, rfc3986)
    if not q:
        return url
    return url + ("&" if "?" in url else "?") + q


_BOT_TOKEN = re.compile(r"/bot[^/?#]+")


_USERINFO = re.compile(r"^([A-Za-z][A-Za-z0-9+.-]*://)[^/?#@]*@")


def redact(url: str) -> str:
    """URL safe for logs: no query string (Trello key/token ride there), no Telegram bot token,
    no ``user:password@``."""
    return _USERINFO.sub(r"\1***@", _BOT_TOKEN.sub("/bot***", url.split("?", 1)[0]))


class HttpError(Exception):
    """Transport failure or (for strict callers) a non-2xx status."""

    def __init__(self, message: str, status: Optional[int] = None, body: bytes = b""):
        super().__init__(message)
        self.status = status
        self.body = body

    @property
    def message(self) -> str:
        return str(self)


class HttpResponse:
    """``status``, ``body`` (bytes), ``headers`` (lower-cased names; parsed on first access
    when built from a raw header block) and the requested ``url``."""

    __slots__ = ("status", "body", "_headers", "_raw", "url")

    def __init__(self, status: int, body: bytes = b"", headers: Optional[Mapping[str, str]] = None, url: str = "",
                 raw_headers: Optional[bytes] = None):
        self.status = status
        self.body = body
        self._headers = {k.lower(): v for k, v in headers.items()} if headers else None
        self._raw = raw_headers
        self.url = url

    @property
    def headers(self) -> Dict[str, str]:
        h = self._headers
        if h is None:
            h = self._headers = parse_raw_headers(self._raw) if self._raw else {}
        return h

    @property
    def ok(self) -> bool:
        return 200 <= self.status < 300

    def text(self) -> str:
        return self.body.decode("utf-8", "replace")

    def json(self) -> Any:
        return _json.loads(self.body or b"null")

    def raise_for_status(self) -> "HttpResponse":
        if not self.ok:
            # request-promise StatusCodeError: `${statusCode} - ${JSON.stringify(body)}`
            # (JSON.stringify leaves non-ASCII characters as they are: ensure_ascii=False)
            raise HttpError(f"{self.status} - {_json.dumps(self.text(), ensure_ascii=False)}", self.status, self.body)
        return self


def parse_raw_headers(raw: bytes) -> Dict[str, str]:
    """``name: value`` lines → dict (lower-cased names; repeated names joined with ', ' like Node)."""
    out: Dict[str, str] = {}
    for line in raw.split(b"\r\n"):
        k, sep, v = line.partition(b":")
        if not sep:
            continue
        name = k.strip().lower().decode("latin-1")
        val = v.strip().decode("latin-1")
        out[name] = f"{out[name]}, {val}" if name in out else val
    return out


class HttpClient(abc.ABC):
    @abc.abstractmethod
    async def request(self, method: str, url: str, *, params: Optional[Mapping[str, Any]] = None,
                      timeout: Optional[float] = None) -> HttpResponse:
        ...

    async def preconnect(self, url: str, n: int) -> Tuple[int, Optional[BaseException]]:
        """Open up to ``n`` keep-alive connections to ``url``'s origin ahead of the first request:
        ``(connections opened, first error or None)``. Clients without a pool open none."""
        return 0, None

    async def close(self) -> None:
        pass


class AiohttpClient(HttpClient):
    """Production client on aiohttp (connection pooling, per-request timeout)."""

    def __init__(self, timeout_s: float = 30.0, user_agent: str = "beholder/1.0"):
        self.timeout_s = timeout_s
        self.user_agent = user_agent
        self._session = None

    async def _sess(self):
        if self._session is None or self._session.closed:
            import aiohttp
            self._session = aiohttp.ClientSession(headers={"User-Agent": self.user_agent})
        return self._session

    async def request(self, method, url, *, params=None, timeout=None) -> HttpResponse:
        # aiohttp's timeout machinery needs asyncio.current_task() to be the request's own task
        # (it cancels that task on timeout). Handlers run eagerly inside the dispatch loop and are
        # resumed by a native Driver, not a Task, so the request gets a Task of its own.
        return await asyncio.ensure_future(self._request(method, url, params, timeout))

    async def _request(self, method, url, params, timeout) -> HttpResponse:
        import aiohttp
        full = with_query(url, params)
        sess = await self._sess()
        try:
            to = aiohttp.ClientTimeout(total=timeout or self.timeout_s)
            # encoded=True: keep our encodeURIComponent-style query untouched
            from yarl import URL
            async with sess.request(method.upper(), URL(full, encoded=True), timeout=to) as r:
                body = await r.read()
                return HttpResponse(r.status, body, dict(r.headers), full)
        except asyncio.TimeoutError as e:
            raise HttpError(f"ETIMEDOUT: {method.upper()} {redact(url)}") from e
        except aiohttp.ClientError as e:
            msg = str(e)
            if full in msg or url in msg:
                msg = msg.replace(full, redact(full)).replace(url, redact(url))
            raise HttpError(f"{type(e).__name__}: {_BOT_TOKEN.sub('/bot***', msg)}") from e

    async def close(self) -> None:
        if self._session is not None and not self._session.closed:
            await self._session.close()


Rule = Tuple[str, str, Callable[[str, str], Any]]


# The canned answer of the in-process stub: what the bench's HTTP fake sends
# (bench/http_sink_server.py), parsed per request like a real reply.
STUB_RESPONSE = b"HTTP/1.1 200 OK\r\nContent-Type: application/json; charset=utf-8\r\nContent-Length: 2\r\n\r\n{}"


class RecordingHttpClient(HttpClient):
    """In-process fake: records every request and answers from rules.

    ``add_rule(method, url_prefix, fn)`` — ``fn(method, url)`` returns an
    ``HttpResponse``, an ``int`` status, or raises (fault injection). Without a
    matching rule the answer is ``200 {}``. ``keep`` bounds the call log (the
    total count is always exact), so benches can use it as a null sink.
    ``delay_s`` simulates network latency (forces a real suspension).

    Its core is native and lives in the bench/test extension (``ops.bench_native.Recorder``,
    ops/csrc_bench/recorder.cpp), not in the service's: per request it builds the request bytes
    with the H1 client's own builder, parses the canned ``200 {}`` with an ``H1Parser`` and
    answers with the H1 client's ``HttpResponse`` (the production client's per-request work,
    minus the socket). While the client has no rules and no delay it exposes that core as
    ``native_record`` (a sink-hook capsule, ops/csrc/native_api.hpp): the compiled handlers then
    call it without entering this class's coroutine, the way they use the H1 client's native
    request path in production (``H1Client.native_call``). ``stub="url"`` is the round-4 stub
    (URL + log only), kept for the A/B of the two (profiles/box_r5_stub_ab/).
    """

    def __init__(self, keep: Optional[int] = None, delay_s: float = 0.0, stub: str = "h1"):
        from ..ops.bench_native import Recorder
        from .h1 import H1Client
        self.calls: Deque[Tuple[str, str]] = collections.deque(maxlen=keep)
        self._rules: Tuple[Rule, ...] = ()
        self._ok = HttpResponse(200, b"{}", None, "")
        shape = H1Client()  # never connects: its origins give Host / Authorization, its tails the User-Agent

        def origin(key: str):
            o = shape._origin(key)
            return o.host_header, o.auth
        self._rec = Recorder(self.calls, self._ok, _native_ops.H1Parser(), STUB_RESPONSE, origin, shape._tail,
                             shape._tail_cl0, mode=stub)
        self._hook = self._rec.hook
        self.delay_s = delay_s  # (sets native_record)

    @property
    def delay_s(self) -> float:
        return self._delay_s

    @delay_s.setter
    def delay_s(self, v: float) -> None:
        self._delay_s = v
        self._sync_fast_path()

    def _sync_fast_path(self) -> None:
        """Expose the native core to the compiled handlers only while every answer is the plain
        ``200 {}`` with no delay, and no subclass overrides request() (jitter, counting)."""
        plain = type(self).request is RecordingHttpClient.request
        self.native_record = self._hook if plain and not self._delay_s and not self._rules else None

    @property
    def count(self) -> int:
        return self._rec.count

    @property
    def rules(self) -> Tuple[Rule, ...]:
        """The rules, read-only: change them with :meth:`add_rule` / :meth:`clear_rules`, which
        keep ``native_record`` in step (a list mutated in place would leave it stale)."""
        return self._rules

    def add_rule(self, method: str, url_prefix: str, fn) -> None:
        self._rules = self._rules + ((method.upper(), url_prefix, fn),)
        self._sync_fast_path()  # answers now depend on the rules: the Python path decides

    def clear_rules(self) -> None:
        self._rules = ()
        self._sync_fast_path()

    def fail(self, method: str, url_prefix: str, status: Optional[int] = None, message: str = "ECONNREFUSED",
             body: bytes = b'"error"'):
        if status is None:
            def boom(m, u):
                raise HttpError(message)
            self.add_rule(method, url_prefix, boom)
        else:
            self.add_rule(method, url_prefix, lambda m, u: HttpResponse(status, body, url=u))

    async def request(self, method, url, *, params=None, timeout=None) -> HttpResponse:
        m = method.upper()
        if type(params) is dict or params is None:  # dict: url + "?" + query, as restler builds it
            full = self._rec.record(m, url, params)
        else:
            full = self._rec.record(m, with_query(url, params), None)
        if self.delay_s:
            await asyncio.sleep(self.delay_s)
        return self.answer(m, full)

    def record(self, method: str, url: str, params=None) -> str:
        """Log one request (method upper-cased by the caller) and return its full URL."""
        if type(params) is dict or params is None:
            return self._rec.record(method, url, params)
        return self._rec.record(method, with_query(url, params), None)

    def answer(self, m: str, full: str) -> HttpResponse:
        """The reply to a recorded request: the first matching rule's, else ``200 {}``."""
        if not self._rules:
            return HttpResponse(200, b"{}", None, full)
        for rm, pref, fn in self._rules:
            if (rm == "*" or rm == m) and full.startswith(pref):
                r = fn(m, full)
                if isinstance(r, int):
                    return HttpResponse(r, b"{}", url=full)
                return r
        return HttpResponse(200, b"{}", url=full)

    def urls(self, method: Optional[str] = None) -> List[str]:
        return [u for m, u in self.calls if method is None or m == method.upper()]


class SinkObserver:
    """Per-sink request accounting: ``beholder_sink_requests_total{sink,code}`` and
    ``beholder_sink_request_seconds{sink}`` (``code`` = HTTP status or ``error``)."""

    def __init__(self, registry):
        self.requests = registry.counter("beholder_sink_requests_total",
                                         "Outbound sink requests by sink and HTTP status (error = transport failure)",
                                         ["sink", "code"])
        self.seconds = registry.histogram("beholder_sink_request_seconds", "Outbound sink request duration",
                                          ["sink"], buckets=(0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10))

    def child(self, sink: str) -> "SinkStats":
        return SinkStats(self.requests, self.seconds.labels(sink), sink)

    def __call__(self, sink: str, status: Optional[int], seconds: float) -> None:
        self.child(sink).record(status, seconds)


# Hot-path handle for one sink (native, ops/csrc/py_metrics.cpp): record(status, seconds) bumps the
# per-status counter child and observes the sink's histogram child in C. The compiled handlers
# (ops/csrc/py_handlers.cpp) record through it without a Python call.
SinkStats = _native_ops.SinkStats


async def observed(stats: Optional["SinkStats"], coro):
    """Await an HTTP request coroutine, recording status and duration into ``stats``."""
    if stats is None:
        return await coro
    t0 = time.perf_counter()
    try:
        r = await coro
    except Exception:
        stats.record(None, time.perf_counter() - t0)
        raise
    stats.record(r.status, time.perf_counter() - t0)
    return r


def parse_query(url: str) -> Dict[str, str]:
    from urllib.parse import parse_qsl, urlsplit
    return dict(parse_qsl(urlsplit(url).query, keep_blank_values=True))
