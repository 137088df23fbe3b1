"""Minimal PostgreSQL v3 wire-protocol client (asyncio).

The reference's ``triton-core/db`` talks to Postgres through ``pg`` 7.12
(yarn.lock:1408-1419). No Postgres driver is installed here, so this
implements the protocol subset a media store needs:

* startup + authentication: trust, cleartext, MD5 and SCRAM-SHA-256
  (the Postgres ≥ 14 default); TLS via ``sslmode`` (disable — node-pg's
  default — prefer, require, verify-ca, verify-full; ``sslrootcert``);
* the extended query protocol (Parse / Bind / Describe / Execute / Sync)
  with server-side prepared statements cached per connection — parameters
  are always sent out-of-band, never interpolated into SQL;
* **pipelining**: queries from concurrent handlers share a connection without
  waiting for each other. Each is its own Sync group, and all the groups queued in
  one event-loop iteration go out in one ``write``. With ``prefetch`` 100
  (index.js:43), up to 100 lookups are in flight on a few connections instead of
  one round trip per connection at a time;
* results assembled natively (``ops/csrc/py_pg.cpp`` ``PgReader``): text-format
  values decoded by type OID (bool, int2/4/8, float4/8, numeric, text/varchar/
  name, json, bytea). :data:`DECODERS` is the Python reference of that mapping;
* ``ErrorResponse`` → :class:`PgError` (with SQLSTATE), connection reuse
  after errors, and a :class:`Pool` that spreads load over up to ``size``
  connections.
"""
from __future__ import annotations

import asyncio
import base64
import collections
import hashlib
import hmac
import os
import struct
import time
from typing import Any, Deque, Dict, List, Optional, Sequence, Tuple
from urllib.parse import parse_qs, unquote, urlsplit

from ..ops import IOFuture as _IOFuture
from ..ops import PgReader
from ..ops import native as _native
from ..utils import netconn


PROTOCOL_V3 = 196608


class PgError(Exception):
    def __init__(self, fields: Dict[str, str]):
        self.fields = fields
        self.sqlstate = fields.get("C", "")
        self.severity = fields.get("S", "ERROR")
        super().__init__(f"{self.severity} {self.sqlstate}: {fields.get('M', 'unknown error')}")


class PgProtocolError(Exception):
    pass


def parse_dsn(dsn: str) -> Dict[str, Any]:
    """``postgres://user:pass@host:port/db?sslmode=disable&application_name=x``."""
    u = urlsplit(dsn)
    if u.scheme not in ("postgres", "postgresql"):
        raise ValueError(f"not a postgres DSN: {dsn!r}")
    q = {k: v[-1] for k, v in parse_qs(u.query).items()}
    return {
        "host": u.hostname or "127.0.0.1", "port": u.port or 5432,
        "user": unquote(u.username) if u.username else os.environ.get("PGUSER", "postgres"),
        "password": unquote(u.password) if u.password else os.environ.get("PGPASSWORD"),
        "database": unquote(u.path[1:]) if u.path and u.path != "/" else "postgres",
        "application_name": q.get("application_name", "beholder"),
        # node-pg's default is a plaintext connection; libpq names for the TLS modes
        "sslmode": q.get("sslmode", os.environ.get("PGSSLMODE", "disable")),
        "sslrootcert": q.get("sslrootcert"),
    }


SSL_MODES = ("disable", "prefer", "require", "verify-ca", "verify-full")


_NATIVE_TLS: Dict[Tuple[str, Optional[str]], Any] = {}


def _native_tls_context(mode: str, rootcert: Optional[str]):
    """The native TLS context (ops TlsContext) for an sslmode, as :func:`_ssl_context` sets
    up the ``ssl`` one; None when native connections or native TLS are off."""
    if not netconn.enabled():
        return None
    key = (mode, rootcert)
    ctx = _NATIVE_TLS.get(key)
    if ctx is None:
        verify = mode not in ("prefer", "require")
        ctx = _NATIVE_TLS[key] = _native.TlsContext(cafile=rootcert, verify=verify,
                                                    check_hostname=mode == "verify-full")
    return ctx


def _tls_error(reason: str, message: str, verify: bool):
    """A failed native TLS handshake as the ``ssl`` module raises it."""
    import ssl
    e = (ssl.SSLCertVerificationError if verify else ssl.SSLError)(1, message)
    e.reason = reason
    e.library = "SSL"
    return e


def _ssl_context(mode: str, rootcert: Optional[str]):
    import ssl
    ctx = ssl.create_default_context(cafile=rootcert) if rootcert else ssl.create_default_context()
    if mode in ("prefer", "require"):  # libpq: encrypt, no certificate checks
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
    elif mode == "verify-ca":
        ctx.check_hostname = False
    return ctx


# ------------------------------------------------------------ type decoding --
def _dec_bool(s: str):
    return s == "t"


def _dec_bytea(s: str):
    if s.startswith("\\x"):
        return bytes.fromhex(s[2:])
    return s.encode()


DECODERS = {16: _dec_bool, 20: int, 21: int, 23: int, 26: int, 700: float, 701: float,
            1700: lambda s: float(s) if "." in s or "e" in s.lower() else int(s),
            25: str, 1043: str, 19: str, 1042: str, 114: str, 3802: str, 17: _dec_bytea}


def encode_param(v: Any) -> Optional[bytes]:
    if v is None:
        return None
    if isinstance(v, bool):
        return b"t" if v else b"f"
    if isinstance(v, (bytes, bytearray)):
        return b"\\x" + bytes(v).hex().encode()
    return str(v).encode()


# --------------------------------------------------------------- SCRAM ------
class _Scram:
    """SCRAM-SHA-256 client (RFC 5802 / RFC 7677), no channel binding."""

    def __init__(self, user: str, password: str, nonce: Optional[str] = None, send_user: bool = False):
        self.password = password
        self.nonce = nonce or base64.b64encode(os.urandom(18)).decode()
        # Postgres ignores the SCRAM user name (the startup message carries it); RFC 7677 sends it
        self.first_bare = f"n={user if send_user else ''},r={self.nonce}"
        self.server_sig = b""

    def client_first(self) -> bytes:
        return ("n,," + self.first_bare).encode()

    def client_final(self, server_first: bytes) -> bytes:
        attrs = dict(kv.split("=", 1) for kv in server_first.decode().split(","))
        rnonce, salt, iters = attrs["r"], base64.b64decode(attrs["s"]), int(attrs["i"])
        if not rnonce.startswith(self.nonce):
            raise PgProtocolError("SCRAM server nonce mismatch")
        salted = hashlib.pbkdf2_hmac("sha256", self.password.encode(), salt, iters)
        client_key = hmac.new(salted, b"Client Key", "sha256").digest()
        stored_key = hashlib.sha256(client_key).digest()
        without_proof = f"c=biws,r={rnonce}"
        auth_msg = f"{self.first_bare},{server_first.decode()},{without_proof}".encode()
        client_sig = hmac.new(stored_key, auth_msg, "sha256").digest()
        proof = bytes(a ^ b for a, b in zip(client_key, client_sig))
        server_key = hmac.new(salted, b"Server Key", "sha256").digest()
        self.server_sig = hmac.new(server_key, auth_msg, "sha256").digest()
        return f"{without_proof},p={base64.b64encode(proof).decode()}".encode()

    def verify(self, server_final: bytes) -> None:
        attrs = dict(kv.split("=", 1) for kv in server_final.decode().split(","))
        if base64.b64decode(attrs.get("v", "")) != self.server_sig:
            raise PgProtocolError("SCRAM server signature mismatch")


# ----------------------------------------------------------- connection -----
_LOST = object()
_pg_bind = _native.pg_bind
_PACK_LEN = struct.Struct("!I").pack


class PgConnection(asyncio.Protocol):
    """One Postgres connection with **pipelined** extended-protocol queries.

    ``execute()`` appends Parse (first use of a statement on this connection) +
    Bind + Describe + Execute + Sync to an output buffer. The buffer is flushed once
    per event-loop iteration, so a batch of handlers costs one ``write``. Each
    Sync group answers exactly one ``execute()``: the native ``PgReader``
    assembles rows / tag / error per ReadyForQuery, and the results are matched to
    callers in FIFO order. An error in one group does not affect the next one
    (Postgres discards until Sync). A parse error evicts the statement from the cache.
    """

    def __init__(self, dsn: str, connect_timeout: float = 10.0):
        self.params = parse_dsn(dsn)
        self.connect_timeout = connect_timeout
        self.server_params: Dict[str, str] = {}
        self.backend_pid = 0
        self.notices: Deque[Dict[str, str]] = collections.deque(maxlen=64)
        self.closed = True
        self._transport = None
        self._reader = PgReader()
        self._startup: Optional[asyncio.Queue] = None
        self._pending: Deque[Tuple[asyncio.Future, Optional[str], bytes]] = collections.deque()
        self._out: List[bytes] = []
        self._flush_handle = None
        self._stmts: Dict[str, bytes] = {}
        self._n_stmts = 0
        self._ssl_answer: Optional[asyncio.Future] = None
        self._lost_in_startup = False
        self.tls = False
        # plain TCP after startup: the socket belongs to a native NetConn (utils/netconn.py),
        # which takes over execute() and the reply matching
        self._net = None

    # -- protocol callbacks --------------------------------------------------
    def connection_made(self, transport):
        self._transport = transport

    def data_received(self, data):
        w = self._ssl_answer
        if w is not None:
            # exactly one byte may precede the TLS handshake; anything more was injected
            # by a man in the middle (CVE-2021-23222)
            if not w.done():
                w.set_result(data if len(data) == 1 else b"?")
            return
        try:
            items = self._reader.feed(data)
        except ValueError as e:
            self._transport.abort()
            self._fail_all(PgProtocolError(f"protocol error: {e}"))
            return
        for it in items:
            if len(it) == 4:
                if not self._pending:
                    self._transport.abort()
                    self._fail_all(PgProtocolError("unexpected ReadyForQuery"))
                    return
                fut, new_sql, name = self._pending.popleft()
                rows, tag, err, parse_ok = it
                if err is not None:
                    if new_sql is not None and not parse_ok and self._stmts.get(new_sql) == name:
                        del self._stmts[new_sql]
                    if not fut.done():
                        fut.reject(PgError(err))
                elif not fut.done():
                    fut.resolve((rows, tag))  # a handler waiting on it resumes right here
            else:
                self._message(it[0], it[1])

    def _message(self, typ: bytes, body: bytes) -> None:
        if self._startup is not None:
            self._startup.put_nowait((typ, body))
        elif typ == b"S":
            k, _, v = body.rstrip(b"\x00").partition(b"\x00")
            self.server_params[k.decode()] = v.decode()
        elif typ == b"N":
            self.notices.append(_fields(body))
        # b"A" NotificationResponse (LISTEN is never used here): ignored

    def connection_lost(self, exc):
        if self._net is not None:
            return  # the transport was aborted when the socket was handed to the NetConn
        self.closed = True
        self._lost_in_startup = self._startup is not None or self._lost_in_startup
        if self._flush_handle is not None:
            self._flush_handle.cancel()
            self._flush_handle = None
        self._out.clear()
        if self._startup is not None:
            self._startup.put_nowait(_LOST)
        if self._ssl_answer is not None and not self._ssl_answer.done():
            self._ssl_answer.set_result(b"")
        self._fail_all(PgProtocolError(f"connection lost: {exc}" if exc else "connection lost"))

    def _fail_all(self, exc: BaseException) -> None:
        self.closed = True
        while self._pending:
            fut = self._pending.popleft()[0]
            if not fut.done():
                fut.set_exception(exc)

    # -- startup -------------------------------------------------------------
    async def _read_msg(self) -> Tuple[bytes, bytes]:
        item = await self._startup.get()
        if item is _LOST:
            raise PgProtocolError("connection lost during startup")
        return item

    def _send(self, typ: bytes, body: bytes) -> None:
        self._write_raw(typ + _PACK_LEN(len(body) + 4) + body)

    def _write_raw(self, data: bytes) -> None:
        if self._net is not None:  # native TLS: startup and authentication over the NetConn
            self._net.write(data)
        else:
            self._transport.write(data)

    async def connect(self) -> "PgConnection":
        p = self.params
        loop = asyncio.get_running_loop()
        if self._net is not None:  # reconnecting this object: back to the asyncio path first
            self._net.abort()
            self._net = None
            self.__dict__.pop("execute", None)
        self._reader = PgReader()
        self._startup = asyncio.Queue()
        self._lost_in_startup = False
        self._stmts.clear()
        mode = p["sslmode"]
        if mode not in SSL_MODES:
            raise PgProtocolError(f"invalid sslmode {mode!r} (one of {', '.join(SSL_MODES)})")
        await asyncio.wait_for(loop.create_connection(lambda: self, p["host"], p["port"]), self.connect_timeout)
        try:
            if mode != "disable":
                await asyncio.wait_for(self._negotiate_tls(mode, p), self.connect_timeout)
            kv = b"".join(k.encode() + b"\x00" + str(v).encode() + b"\x00" for k, v in
                          (("user", p["user"]), ("database", p["database"]),
                           ("application_name", p["application_name"]), ("client_encoding", "UTF8")))
            body = struct.pack("!I", PROTOCOL_V3) + kv + b"\x00"
            self._write_raw(_PACK_LEN(len(body) + 4) + body)
            await asyncio.wait_for(self._auth(), self.connect_timeout)
        except BaseException:
            if self._net is not None:
                self._net.abort()
                self._net = None
            elif self._transport is not None:
                self._transport.abort()
            self._startup = None
            raise
        self._startup = None
        lost = self._net.closed if self._net is not None else (self._transport is None or self._transport.is_closing()
                                                               or self._lost_in_startup)
        if lost:  # the server closed right after ReadyForQuery: connection_lost has already run
            if self._net is not None:
                self._net.abort()
                self._net = None
            raise PgProtocolError("connection lost during startup")
        self._reader.query_mode = True
        self.closed = False
        if self._net is not None:  # native TLS since the SSLRequest
            self.execute = self._net.execute
        elif not self.tls:
            fd = netconn.adopt(self._transport)
            if fd is not None:
                self._net = netconn.NetConn(fd, loop, "pg", self, self._reader, self._stmts, PgError,
                                            PgProtocolError)
                self._transport = None
                self.execute = self._net.execute  # native: Parse/Bind/Execute/Sync + IOFuture
        return self

    def abort(self, reason: Optional[str] = None) -> None:
        """Drop the connection now; outstanding queries fail with PgProtocolError (``reason``:
        its text, default "connection lost")."""
        if self._net is not None:
            self._net.abort()
            self._net_lost(reason)
        elif self._transport is not None:
            if reason:
                self._fail_all(PgProtocolError(reason))
            self._transport.abort()

    # -- NetConn callbacks (rare paths) ----------------------------------------
    def _net_lost(self, exc) -> None:
        self.closed = True
        if self._startup is not None:
            self._startup.put_nowait(_LOST)
        text = exc if isinstance(exc, str) else (f"connection lost: {exc}" if exc else "connection lost")
        self._net.fail_all(PgProtocolError(text))

    def _net_error(self, exc) -> None:
        self.closed = True
        self._net.abort()
        self._net.fail_all(PgProtocolError(f"protocol error: {exc}" if exc is not None
                                           else "unexpected ReadyForQuery"))

    def _net_message(self, typ: bytes, body: bytes) -> None:
        self._message(typ, body)

    async def _negotiate_tls(self, mode: str, p: Dict[str, Any]) -> None:
        """SSLRequest; on 'S' upgrade the transport in place (``loop.start_tls``)."""
        self._ssl_answer = asyncio.get_running_loop().create_future()
        self._transport.write(_PACK_LEN(8) + struct.pack("!I", 80877103))
        ans = await self._ssl_answer
        self._ssl_answer = None
        if ans == b"S":
            loop = asyncio.get_running_loop()
            nctx = _native_tls_context(mode, p.get("sslrootcert"))
            fd = netconn.adopt(self._transport) if nctx is not None else None
            if fd is not None:  # TLS in C on the socket (ops/csrc/py_tls.cpp): handshake, then startup
                try:
                    self._net = netconn.NetConn(fd, loop, "pg", self, self._reader, self._stmts, PgError,
                                                PgProtocolError, tls=nctx, server_hostname=p["host"],
                                                port=int(p["port"]), tls_error=_tls_error)
                except BaseException:
                    os.close(fd)
                    raise
                self._transport = None
                await self._net.handshake
            else:
                ctx = _ssl_context(mode, p.get("sslrootcert"))
                self._transport = await loop.start_tls(self._transport, self, ctx, server_hostname=p["host"])
            self.tls = True
        elif ans == b"N":
            if mode != "prefer":
                raise PgProtocolError(f"server does not support SSL, but sslmode={mode}")
        else:
            raise PgProtocolError(f"unexpected answer to SSLRequest: {ans!r}")

    async def _auth(self) -> None:
        p = self.params
        scram: Optional[_Scram] = None
        while True:
            typ, body = await self._read_msg()
            if typ == b"R":
                code = struct.unpack("!I", body[:4])[0]
                if code == 0:
                    continue
                pw = p["password"]
                if code in (3, 5, 10) and pw is None:
                    raise PgProtocolError("server requested a password but none was given")
                if code == 3:
                    self._send(b"p", pw.encode() + b"\x00")
                elif code == 5:
                    salt = body[4:8]
                    inner = hashlib.md5(pw.encode() + p["user"].encode()).hexdigest()
                    outer = hashlib.md5(inner.encode() + salt).hexdigest()
                    self._send(b"p", b"md5" + outer.encode() + b"\x00")
                elif code == 10:
                    mechs = [m for m in body[4:].split(b"\x00") if m]
                    if b"SCRAM-SHA-256" not in mechs:
                        raise PgProtocolError(f"unsupported SASL mechanisms {mechs}")
                    scram = _Scram(p["user"], pw)
                    first = scram.client_first()
                    self._send(b"p", b"SCRAM-SHA-256\x00" + struct.pack("!i", len(first)) + first)
                elif code in (11, 12) and scram is None:
                    raise PgProtocolError(f"SASL message {code} before SASL negotiation")
                elif code == 11:
                    self._send(b"p", scram.client_final(body[4:]))
                elif code == 12:
                    scram.verify(body[4:])
                else:
                    raise PgProtocolError(f"unsupported authentication method {code}")
            elif typ == b"S":
                k, v = body.rstrip(b"\x00").split(b"\x00", 1)
                self.server_params[k.decode()] = v.decode()
            elif typ == b"K":
                self.backend_pid = struct.unpack("!I", body[:4])[0]
            elif typ == b"Z":
                return
            elif typ == b"E":
                raise PgError(_fields(body))
            elif typ == b"N":
                continue
            else:
                raise PgProtocolError(f"unexpected message {typ!r} during startup")

    # -- queries -------------------------------------------------------------
    @property
    def pending(self) -> int:
        """Queries sent (or buffered) and not yet answered."""
        net = self._net
        return net.pending if net is not None else len(self._pending)

    def execute(self, sql: str, params: Sequence[Any] = ()) -> "asyncio.Future[Tuple[List[Tuple], str]]":
        """Queue one statement with ``$n`` parameters; the returned future resolves to
        ``(rows, command_tag)`` or raises :class:`PgError`. It is an ``ops.IOFuture``: a
        handler awaiting it through the native Driver resumes inside ``data_received``, with no
        event-loop round trip per reply."""
        if self.closed:
            raise PgProtocolError("connection is closed")
        out = self._out
        name = self._stmts.get(sql)
        new_sql = None
        if name is None:
            self._n_stmts += 1
            name = b"b%d" % self._n_stmts
            self._stmts[sql] = name
            new_sql = sql
            pbody = name + b"\x00" + sql.encode() + b"\x00\x00\x00"
            out.append(b"P" + _PACK_LEN(len(pbody) + 4) + pbody)
        out.append(_pg_bind(name, params))  # Bind + Describe + Execute + Sync (ops/csrc/py_pg.cpp)
        loop = asyncio.get_running_loop()
        fut = _IOFuture(loop)
        self._pending.append((fut, new_sql, name))
        if self._flush_handle is None:
            self._flush_handle = loop.call_soon(self._flush)
        return fut

    def _flush(self) -> None:
        self._flush_handle = None
        if self._out and not self.closed:
            data = b"".join(self._out)
            self._out.clear()
            self._transport.write(data)

    async def close(self) -> None:
        net = self._net
        if net is not None:
            if not self.closed:
                deadline = time.monotonic() + self.connect_timeout
                while net.pending and not net.closed and time.monotonic() < deadline:
                    await asyncio.sleep(0.001)  # in-flight queries finish; a dead server cannot hang shutdown
                if not net.closed:
                    net.flush()
                    net.write(b"X" + _PACK_LEN(4))  # Terminate
                    net.close()
                net.fail_all(PgProtocolError("connection closed"))
            self.closed = True
            return
        if self._transport is None or self.closed:
            self.closed = True
            return
        pending = [f for f, _, _ in self._pending]
        if pending:  # let in-flight queries finish, but never hang shutdown on a dead server
            try:
                await asyncio.wait_for(asyncio.gather(*pending, return_exceptions=True), self.connect_timeout)
            except asyncio.TimeoutError:
                self._transport.abort()
        if not self.closed:
            self._flush()
            try:
                self._send(b"X", b"")
            except (ConnectionError, OSError):
                pass
            self._transport.close()
        self.closed = True


def _msg(typ: bytes, body: bytes) -> bytes:
    return typ + struct.pack("!I", len(body) + 4) + body


def _fields(body: bytes) -> Dict[str, str]:
    out = {}
    for part in body.split(b"\x00"):
        if part:
            out[chr(part[0])] = part[1:].decode("utf-8", "replace")
    return out


class Pool:
    """Up to ``size`` pipelined :class:`PgConnection` s.

    A query goes to the open connection with the fewest queries in flight. A new
    connection is opened (up to ``size``) only when every open one already has
    ``spread_at`` or more in flight, so light load stays on one connection and one
    ``write`` per loop iteration. The pool grows in the background: the query that finds
    every connection busy is still sent at once on the least-loaded one, and the new
    connection takes queries once its startup and authentication are done (a query never
    waits for a connect while a connection is open; the warm-up tail of ``tcp_e2e``). A
    failed grow is retried after ``GROW_RETRY_S``. Broken connections are dropped and
    replaced on demand.
    """

    GROW_RETRY_S = 1.0

    def __init__(self, dsn: str, size: int = 4, spread_at: int = 8, stall_timeout_s: Optional[float] = 30.0,
                 min_open: int = 1):
        self.dsn = dsn
        self.size = max(1, int(size))
        # connections opened by open(): the first burst of queries (prefetch 100 deliveries at
        # startup) is spread at once instead of queueing on one connection while the pool grows
        self.min_open = max(1, min(self.size, int(min_open)))
        self.spread_at = spread_at
        # a connection with queries in flight and no reply for this long is dropped (its queries
        # fail): a half-open TCP connection (peer gone without a FIN or RST) would otherwise hold
        # every query sent on it, and their handlers, forever. None = off.
        self.stall_timeout_s = stall_timeout_s
        self._watchdog: Optional[asyncio.Task] = None
        self.stalls = 0
        self._conns: List[PgConnection] = []
        # the native pick's view of `_conns` (_sync_nets): their NetConns, whose own closed flags
        # it reads (a PgConnection and its NetConn close together), or None while any connection
        # is on the asyncio path
        self._nets: Optional[List[Any]] = []
        self._lock = asyncio.Lock()
        self._growing: Optional[asyncio.Future] = None
        self._grow_after = 0.0
        self._closed = False
        self.grows = 0  # connections added by the background grow
        self.grow_errors = 0
        # capability (also for the compiled handlers): the native least-loaded pick + send over a
        # pool of native connections (ops/csrc/py_netconn.cpp), None with native I/O off
        self.native_pick = _native.pg_pool_execute if netconn.enabled() else None

    async def open(self) -> "Pool":
        self._conns.append(await PgConnection(self.dsn).connect())  # fail fast on bad DSN/credentials
        if self.min_open > 1:  # the rest together; one that fails is left to the background grow
            more = await asyncio.gather(*(PgConnection(self.dsn).connect() for _ in range(self.min_open - 1)),
                                        return_exceptions=True)
            fatal = None
            for c in more:
                if not isinstance(c, BaseException):
                    self._conns.append(c)
                elif isinstance(c, (OSError, asyncio.TimeoutError, PgError, PgProtocolError)):
                    self.grow_errors += 1
                elif fatal is None:
                    fatal = c
            if fatal is not None:  # nothing is handed out: close what opened, then fail
                for c in self._conns:
                    await c.close()
                self._conns = []
                self._sync_nets()
                raise fatal
        self._sync_nets()
        if self.stall_timeout_s:
            self._watchdog = asyncio.get_running_loop().create_task(self._watch_stalls())
        return self

    async def _watch_stalls(self) -> None:
        """Drops a connection whose replies stopped while queries are in flight: progress is the
        reader's count of answered Sync groups, checked every quarter timeout."""
        timeout = float(self.stall_timeout_s)
        seen: Dict[int, Tuple[int, float]] = {}  # id(conn) -> (answered, since)
        loop = asyncio.get_running_loop()
        while not self._closed:
            await asyncio.sleep(min(1.0, timeout / 4))
            now = loop.time()
            live = {}
            for c in list(self._conns):
                if c.closed or not c.pending:
                    continue
                answered = c._reader.results
                prev = seen.get(id(c))
                since = prev[1] if prev is not None and prev[0] == answered else now
                live[id(c)] = (answered, since)
                if now - since >= timeout:
                    self.stalls += 1
                    c.abort(f"no reply from Postgres for {timeout:g} s with {c.pending} queries in flight")
                    live.pop(id(c))
            seen = live

    def execute(self, sql: str, params: Sequence[Any] = ()):
        """Awaitable ``(rows, command_tag)`` (a future on the fast path)."""
        pick = self.native_pick
        if pick is not None:
            f = pick(self._nets, sql, params, self.spread_at, self.size)  # None unless all connections native
            if f is not None:
                return f
        best = None
        bp = 0
        live = 0
        for c in self._conns:
            if not c.closed:
                live += 1
                n = c.pending
                if best is None or n < bp:
                    best, bp = c, n
        if best is None:
            return self._execute_slow(sql, params)
        if bp >= self.spread_at and live < self.size:
            self._grow()
        return best.execute(sql, params)

    def _grow(self) -> None:
        if self._growing is not None or self._closed:
            return
        loop = asyncio.get_running_loop()
        if loop.time() < self._grow_after:
            return
        self._growing = loop.create_task(self._grow_one())

    async def _grow_one(self) -> None:
        try:
            c = await PgConnection(self.dsn).connect()
        except (OSError, asyncio.TimeoutError, PgError, PgProtocolError):
            self.grow_errors += 1
            self._grow_after = asyncio.get_running_loop().time() + self.GROW_RETRY_S
            return
        finally:
            self._growing = None
        if self._closed:
            await c.close()
            return
        self._conns[:] = [x for x in self._conns if not x.closed]
        self._conns.append(c)  # in place: a connect in _execute_slow appends to the same list
        self._sync_nets()
        self.grows += 1

    async def _execute_slow(self, sql: str, params: Sequence[Any]):
        """No open connection: connect under the lock, so a burst makes one connection, then send."""
        async with self._lock:
            self._conns[:] = [c for c in self._conns if not c.closed]
            self._sync_nets()
            live = self._conns
            if len(live) < self.size and (not live or min(c.pending for c in live) >= self.spread_at):
                try:
                    live.append(await PgConnection(self.dsn).connect())
                except (OSError, asyncio.TimeoutError, PgError, PgProtocolError):
                    if not live:
                        raise
                self._sync_nets()
            c = min(live, key=lambda c: c.pending)
        return await c.execute(sql, params)

    @property
    def connections(self) -> int:
        return sum(1 for c in self._conns if not c.closed)

    async def close(self) -> None:
        self._closed = True
        if self._watchdog is not None:
            self._watchdog.cancel()
            self._watchdog = None
        g = self._growing
        if g is not None:
            g.cancel()
            try:
                await g
            except (asyncio.CancelledError, Exception):  # noqa: BLE001 -- closing anyway
                pass
        for c in list(self._conns):
            await c.close()
        self._conns = []
        self._sync_nets()

    def _sync_nets(self) -> None:
        """Rebuilds ``_nets`` after ``_conns`` changed (closing needs no rebuild: the pick skips a
        closed NetConn, as Pool.execute skips a closed connection)."""
        nets = [c._net for c in self._conns]
        self._nets = nets if all(n is not None for n in nets) else None
