"""A fake PostgreSQL server speaking the v3 wire protocol, backed by sqlite3.

Enough of the protocol to exercise beholder's pgwire client for real over TCP:
startup (SSLRequest refused), trust / cleartext / md5 / SCRAM-SHA-256 auth,
extended query (Parse/Bind/Describe/Execute/Sync), simple Query, errors with
SQLSTATE and error-recovery until Sync.
"""
import asyncio
import base64
import hashlib
import hmac
import os
import re
import sqlite3
import struct


def _msg(t: bytes, body: bytes) -> bytes:
    return t + struct.pack("!I", len(body) + 4) + body


class FakePg:
    def __init__(self, auth="scram", user="beholder", password="s3cret", ssl_context=None):
        self.auth = auth
        self.ssl_context = ssl_context  # answer SSLRequest with 'S' and upgrade
        self.tls_sessions = 0
        self.user = user
        self.password = password
        self.db = sqlite3.connect(":memory:", check_same_thread=False, isolation_level=None)
        self.port = 0
        self._server = None
        self.statements_parsed = 0
        self.queries = []
        self._writers = set()
        self.connections = 0

    def drop_connections(self) -> int:
        """Abort every open client connection (a Postgres restart / failover)."""
        n = len(self._writers)
        for w in list(self._writers):
            t = w.transport
            if t is not None:  # None: mid-upgrade to TLS (SSLRequest answered, start_tls running)
                t.abort()
        return n

    @property
    def dsn(self):
        return f"postgres://{self.user}:{self.password}@127.0.0.1:{self.port}/media"

    async def start(self):
        self._server = await asyncio.start_server(self._serve, "127.0.0.1", 0)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        self._server.close()
        await self._server.wait_closed()

    async def _read(self, r):
        hdr = await r.readexactly(5)
        n = struct.unpack("!I", hdr[1:])[0]
        return hdr[:1], (await r.readexactly(n - 4) if n > 4 else b"")

    async def _serve(self, r, w):
        self._writers.add(w)
        self.connections += 1
        try:
            n = struct.unpack("!I", await r.readexactly(4))[0]
            body = await r.readexactly(n - 4)
            if struct.unpack("!I", body[:4])[0] == 80877103:  # SSLRequest
                if self.ssl_context is None:
                    w.write(b"N")
                else:
                    w.write(b"S")
                    await w.drain()
                    # asyncio 3.10 streams have no server-side start_tls: upgrade the transport and
                    # point the stream objects at the TLS one
                    proto = w.transport.get_protocol()
                    tls = await asyncio.get_running_loop().start_tls(w.transport, proto, self.ssl_context,
                                                                     server_side=True)
                    w._transport = tls
                    proto._transport = tls
                    r._transport = tls
                    self.tls_sessions += 1
                n = struct.unpack("!I", await r.readexactly(4))[0]
                body = await r.readexactly(n - 4)
            kv = body[4:].split(b"\x00")
            params = dict(zip(kv[0::2], kv[1::2]))
            if params.get(b"user", b"").decode() != self.user:
                w.write(_msg(b"E", b"SFATAL\x00C28000\x00Mrole does not exist\x00\x00"))
                return
            if not await self._authenticate(r, w):
                return
            w.write(_msg(b"R", struct.pack("!I", 0)))
            w.write(_msg(b"S", b"server_version\x0016.0-fake\x00"))
            w.write(_msg(b"K", struct.pack("!II", 42, 7)))
            w.write(_msg(b"Z", b"I"))
            await self._loop(r, w)
        except (asyncio.IncompleteReadError, ConnectionError, OSError):
            pass
        finally:
            self._writers.discard(w)
            if w.transport is not None:  # None: dropped while start_tls was upgrading it
                w.close()

    async def _authenticate(self, r, w) -> bool:
        if self.auth == "trust":
            return True
        if self.auth == "cleartext":
            w.write(_msg(b"R", struct.pack("!I", 3)))
            _, body = await self._read(r)
            ok = body.rstrip(b"\x00").decode() == self.password
        elif self.auth == "md5":
            salt = os.urandom(4)
            w.write(_msg(b"R", struct.pack("!I", 5) + salt))
            _, body = await self._read(r)
            inner = hashlib.md5((self.password + self.user).encode()).hexdigest()
            ok = body.rstrip(b"\x00").decode() == "md5" + hashlib.md5(inner.encode() + salt).hexdigest()
        else:  # scram
            w.write(_msg(b"R", struct.pack("!I", 10) + b"SCRAM-SHA-256\x00\x00"))
            _, body = await self._read(r)
            mech_end = body.index(b"\x00")
            first = body[mech_end + 5:].decode()
            bare = first.split(",", 2)[2]
            cnonce = dict(kv.split("=", 1) for kv in bare.split(","))["r"]
            salt, iters = os.urandom(16), 4096
            snonce = cnonce + base64.b64encode(os.urandom(12)).decode()
            server_first = f"r={snonce},s={base64.b64encode(salt).decode()},i={iters}"
            w.write(_msg(b"R", struct.pack("!I", 11) + server_first.encode()))
            _, final = await self._read(r)
            final = final.decode()
            without_proof, proof = final.rsplit(",p=", 1)
            salted = hashlib.pbkdf2_hmac("sha256", self.password.encode(), salt, iters)
            client_key = hmac.new(salted, b"Client Key", "sha256").digest()
            stored = hashlib.sha256(client_key).digest()
            auth_msg = f"{bare},{server_first},{without_proof}".encode()
            sig = hmac.new(stored, auth_msg, "sha256").digest()
            got_key = bytes(a ^ b for a, b in zip(base64.b64decode(proof), sig))
            ok = hashlib.sha256(got_key).digest() == stored
            if ok:
                skey = hmac.new(salted, b"Server Key", "sha256").digest()
                ssig = hmac.new(skey, auth_msg, "sha256").digest()
                w.write(_msg(b"R", struct.pack("!I", 12) + f"v={base64.b64encode(ssig).decode()}".encode()))
        if not ok:
            w.write(_msg(b"E", b"SFATAL\x00C28P01\x00Mpassword authentication failed\x00\x00"))
        return ok

    def _run(self, sql, params):
        self.queries.append(sql)
        lite = re.sub(r"\$(\d+)", r"?\1", sql)
        cur = self.db.execute(lite, params)
        rows = cur.fetchall()
        verb = sql.strip().split()[0].upper()
        tag = {"SELECT": f"SELECT {len(rows)}", "UPDATE": f"UPDATE {cur.rowcount}",
               "INSERT": f"INSERT 0 {cur.rowcount}", "DELETE": f"DELETE {cur.rowcount}"}.get(verb, verb)
        return rows, (cur.description or []), tag

    def _rowdesc(self, rows, desc):
        body = struct.pack("!H", len(desc))
        for i, d in enumerate(desc):
            v = rows[0][i] if rows else None
            oid = 20 if isinstance(v, int) else 25
            body += d[0].encode() + b"\x00" + struct.pack("!IhIhih", 0, 0, oid, -1, -1, 0)
        return _msg(b"T", body)

    def _datarow(self, row):
        body = struct.pack("!H", len(row))
        for v in row:
            if v is None:
                body += struct.pack("!i", -1)
            else:
                s = str(v).encode()
                body += struct.pack("!i", len(s)) + s
        return _msg(b"D", body)

    async def _loop(self, r, w):
        stmts, portal, failed = {}, None, False
        while True:
            t, body = await self._read(r)
            if t == b"X":
                return
            if t == b"S":
                failed = False
                w.write(_msg(b"Z", b"I"))
                await w.drain()
                continue
            if failed:
                continue
            try:
                if t == b"P":
                    name, rest = body.split(b"\x00", 1)
                    sql = rest.split(b"\x00", 1)[0].decode()
                    if "syntax error" in sql:
                        raise sqlite3.OperationalError('syntax error at or near "syntax"')
                    stmts[name] = sql
                    self.statements_parsed += 1
                    w.write(_msg(b"1", b""))
                elif t == b"B":
                    i = body.index(b"\x00") + 1
                    j = body.index(b"\x00", i)
                    stmt = body[i:j]
                    i = j + 1
                    nfmt = struct.unpack_from("!H", body, i)[0]
                    i += 2 + 2 * nfmt
                    nparam = struct.unpack_from("!H", body, i)[0]
                    i += 2
                    params = []
                    for _ in range(nparam):
                        ln = struct.unpack_from("!i", body, i)[0]
                        i += 4
                        if ln < 0:
                            params.append(None)
                        else:
                            s = body[i:i + ln].decode()
                            i += ln
                            params.append(int(s) if re.fullmatch(r"-?\d+", s) else s)
                    if stmt not in stmts:
                        raise sqlite3.OperationalError(f'prepared statement "{stmt.decode()}" does not exist')
                    portal = (stmts[stmt], params, None)
                    w.write(_msg(b"2", b""))
                elif t == b"D":
                    rows, desc, tag = self._run(portal[0], portal[1])
                    portal = (portal[0], portal[1], (rows, desc, tag))
                    w.write(self._rowdesc(rows, desc) if desc else _msg(b"n", b""))
                elif t == b"E":
                    rows, desc, tag = portal[2] or self._run(portal[0], portal[1])
                    for row in rows:
                        w.write(self._datarow(row))
                    w.write(_msg(b"C", tag.encode() + b"\x00"))
                elif t == b"Q":
                    sql = body.rstrip(b"\x00").decode()
                    rows, desc, tag = self._run(sql, [])
                    if desc:
                        w.write(self._rowdesc(rows, desc))
                        for row in rows:
                            w.write(self._datarow(row))
                    w.write(_msg(b"C", tag.encode() + b"\x00"))
                    w.write(_msg(b"Z", b"I"))
            except (sqlite3.Error, ValueError) as e:
                failed = t != b"Q"
                code = b"42601" if "syntax" in str(e) else (b"23505" if "UNIQUE" in str(e) else b"XX000")
                w.write(_msg(b"E", b"SERROR\x00C" + code + b"\x00M" + str(e).encode() + b"\x00\x00"))
                if t == b"Q":
                    w.write(_msg(b"Z", b"I"))
