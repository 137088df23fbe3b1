"""Minimal PostgreSQL v3 wire-protocol client (asyncio).

The reference's ``triton-core/db`` talks to Postgres through ``pg`` 7.12
(yarn.lock:1408-1419). No Postgres driver is installed here, so this
implements the protocol subset a media store needs:

* startup + authentication: trust, cleartext, MD5 and SCRAM-SHA-256
  (the Postgres ≥ 14 default);
* the extended query protocol (Parse / Bind / Describe / Execute / Sync)
  with server-side prepared statements cached per connection — parameters
  are always sent out-of-band, never interpolated into SQL;
* text-format results decoded by type OID (bool, int2/4/8, float4/8,
  numeric, text/varchar/name, json, bytea);
* ``ErrorResponse`` → :class:`PgError` (with SQLSTATE), connection reuse
  after errors, and a small connection :class:`Pool`.
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import hmac
import os
import struct
from typing import Any, Dict, List, Optional, Sequence, Tuple
from urllib.parse import parse_qs, unquote, urlsplit

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
    }


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

    def __init__(self, user: str, password: str):
        self.password = password
        self.nonce = base64.b64encode(os.urandom(18)).decode()
        self.first_bare = f"n=,r={self.nonce}"  # Postgres ignores the SCRAM user name
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
class PgConnection:
    def __init__(self, dsn: str, connect_timeout: float = 10.0):
        self.params = parse_dsn(dsn)
        self.connect_timeout = connect_timeout
        self.reader: Optional[asyncio.StreamReader] = None
        self.writer: Optional[asyncio.StreamWriter] = None
        self.server_params: Dict[str, str] = {}
        self.backend_pid = 0
        self._stmts: Dict[str, str] = {}
        self._lock = asyncio.Lock()
        self.closed = True

    async def _read_msg(self) -> Tuple[bytes, bytes]:
        hdr = await self.reader.readexactly(5)
        typ, ln = hdr[:1], struct.unpack("!I", hdr[1:])[0]
        body = await self.reader.readexactly(ln - 4) if ln > 4 else b""
        return typ, body

    def _send(self, typ: bytes, body: bytes) -> None:
        self.writer.write(typ + struct.pack("!I", len(body) + 4) + body)

    async def connect(self) -> "PgConnection":
        p = self.params
        self.reader, self.writer = await asyncio.wait_for(asyncio.open_connection(p["host"], p["port"]),
                                                          self.connect_timeout)
        kv = b"".join(k.encode() + b"\x00" + str(v).encode() + b"\x00" for k, v in
                      (("user", p["user"]), ("database", p["database"]),
                       ("application_name", p["application_name"]), ("client_encoding", "UTF8")))
        body = struct.pack("!I", PROTOCOL_V3) + kv + b"\x00"
        self.writer.write(struct.pack("!I", len(body) + 4) + body)
        await asyncio.wait_for(self._auth(), self.connect_timeout)
        self.closed = False
        return self

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

    async def execute(self, sql: str, params: Sequence[Any] = ()) -> Tuple[List[Tuple], str]:
        """Run one statement with ``$n`` parameters. Returns ``(rows, command_tag)``."""
        async with self._lock:
            if self.closed:
                raise PgProtocolError("connection is closed")
            name = self._stmts.get(sql)
            parts = []
            if name is None:
                name = f"b{len(self._stmts) + 1}"
                parts.append(_msg(b"P", name.encode() + b"\x00" + sql.encode() + b"\x00" + struct.pack("!H", 0)))
            enc = [encode_param(v) for v in params]
            bind = name.encode()
            bind = b"\x00" + bind + b"\x00" + struct.pack("!H", 0) + struct.pack("!H", len(enc))
            for e in enc:
                bind += struct.pack("!i", -1) if e is None else struct.pack("!i", len(e)) + e
            bind += struct.pack("!H", 0)
            parts.append(_msg(b"B", bind))
            parts.append(_msg(b"D", b"P\x00"))
            parts.append(_msg(b"E", b"\x00" + struct.pack("!I", 0)))
            parts.append(_msg(b"S", b""))
            self.writer.write(b"".join(parts))
            rows: List[Tuple] = []
            cols: List[int] = []
            tag = ""
            err: Optional[PgError] = None
            parsed_ok = False
            try:
                while True:
                    typ, body = await self._read_msg()
                    if typ == b"1":
                        parsed_ok = True
                    elif typ == b"T":
                        cols = _row_description(body)
                    elif typ == b"D":
                        rows.append(_data_row(body, cols))
                    elif typ == b"C":
                        tag = body.rstrip(b"\x00").decode()
                    elif typ == b"E":
                        err = PgError(_fields(body))
                    elif typ == b"Z":
                        break
                    # 2 BindComplete, n NoData, s PortalSuspended, I EmptyQuery, N Notice, S ParamStatus: ignore
            except (asyncio.IncompleteReadError, ConnectionError) as e:
                self.closed = True
                raise PgProtocolError(f"connection lost: {e}") from e
            if parsed_ok or sql in self._stmts:
                self._stmts[sql] = name
            if err is not None:
                raise err
            return rows, tag

    async def close(self) -> None:
        if self.writer is not None and not self.closed:
            try:
                self._send(b"X", b"")
                await self.writer.drain()
            except (ConnectionError, OSError):
                pass
            self.writer.close()
        self.closed = True


def _msg(typ: bytes, body: bytes) -> bytes:
    return typ + struct.pack("!I", len(body) + 4) + body


def _fields(body: bytes) -> Dict[str, str]:
    out = {}
    for part in body.split(b"\x00"):
        if part:
            out[chr(part[0])] = part[1:].decode("utf-8", "replace")
    return out


def _row_description(body: bytes) -> List[int]:
    n = struct.unpack_from("!H", body)[0]
    i = 2
    oids = []
    for _ in range(n):
        j = body.index(b"\x00", i)
        i = j + 1
        _table, _col, oid, _size, _mod, _fmt = struct.unpack_from("!IhIhih", body, i)
        oids.append(oid)
        i += 18
    return oids


def _data_row(body: bytes, oids: List[int]) -> Tuple:
    n = struct.unpack_from("!H", body)[0]
    i = 2
    out = []
    for k in range(n):
        ln = struct.unpack_from("!i", body, i)[0]
        i += 4
        if ln < 0:
            out.append(None)
            continue
        s = body[i:i + ln].decode("utf-8")
        i += ln
        dec = DECODERS.get(oids[k] if k < len(oids) else 25, str)
        out.append(dec(s))
    return tuple(out)


class Pool:
    """Fixed-size pool of :class:`PgConnection` (lazy connect, replaces broken connections)."""

    def __init__(self, dsn: str, size: int = 4):
        self.dsn = dsn
        self.size = size
        self._free: "asyncio.Queue[PgConnection]" = asyncio.Queue()
        self._all: List[PgConnection] = []

    async def open(self) -> "Pool":
        first = await PgConnection(self.dsn).connect()  # fail fast on bad DSN/credentials
        self._all.append(first)
        self._free.put_nowait(first)
        for _ in range(self.size - 1):
            c = PgConnection(self.dsn)
            self._all.append(c)
            self._free.put_nowait(c)
        return self

    async def execute(self, sql: str, params: Sequence[Any] = ()) -> Tuple[List[Tuple], str]:
        c = await self._free.get()
        try:
            if c.closed:
                await c.connect()
            return await c.execute(sql, params)
        except PgProtocolError:
            c.closed = True
            raise
        finally:
            self._free.put_nowait(c)

    async def close(self) -> None:
        for c in self._all:
            await c.close()
