"""Fake Postgres for the ``tcp_e2e`` bench config.

It speaks enough of the v3 protocol for the media store's two hot statements,
``SELECT <cols> FROM media WHERE id = $1`` and
``UPDATE media SET status = $1 WHERE id = $2``. It supports trust auth, the
extended protocol (including pipelined Sync groups) and an in-memory table. The
table is the synthetic media population of :class:`~.generator.Workload`
(``--media N --seed S``), so a replayed event stream finds its rows. Several
copies can share one port (``SO_REUSEPORT``). It prints ``READY <port>`` once it
is listening. On SIGTERM it prints ``DONE queries=<n>`` and its ``STALLS`` line.

It stands in for the database so the bench measures the consumer. It is not a
database. By default the protocol is served by the native ``PgFake``
(ops/csrc_bench/pg_fake.cpp) on its own thread: this asyncio server costs ~5 us of CPU
per query, and with the consumer's pool spread unevenly over two copies by
SO_REUSEPORT one copy saturated and capped the run (profiles/box_r5_util/).
``--python`` serves it from the asyncio protocol below instead.
"""
from __future__ import annotations

import argparse
import asyncio
import signal
import socket
import struct
import sys

from .stallmon import fake_monitor

_U32 = struct.Struct("!I")


def _msg(t: bytes, body: bytes) -> bytes:
    return t + _U32.pack(len(body) + 4) + body


_COLS = ("id", "name", "creator", "creator_id", "type", "source", "source_uri", "metadata", "metadata_id", "status")
_INT = {2, 4, 5, 7, 9}
_ROWDESC = _msg(b"T", struct.pack("!H", len(_COLS)) + b"".join(
    c.encode() + b"\x00" + struct.pack("!IhIhih", 0, 0, 23 if i in _INT else 25, -1, -1, 0)
    for i, c in enumerate(_COLS)))
_AUTH_OK = (_msg(b"R", _U32.pack(0)) + _msg(b"S", b"server_version\x0016.0-bench\x00") +
            _msg(b"K", struct.pack("!II", 1, 1)) + _msg(b"Z", b"I"))
_PARSE_OK, _BIND_OK, _NODATA, _READY = _msg(b"1", b""), _msg(b"2", b""), _msg(b"n", b""), _msg(b"Z", b"I")


def _row(values) -> bytes:
    parts = [struct.pack("!H", len(values))]
    for v in values:
        b = str(v).encode()
        parts.append(_U32.pack(len(b)) + b)
    return _msg(b"D", b"".join(parts))


class _Proto(asyncio.Protocol):
    table: dict = {}
    queries = 0

    def connection_made(self, transport):
        self.t = transport
        self.buf = b""
        self.started = False
        self.stmts = {}
        self.kind = None
        self.params = []
        self.failed = False

    def data_received(self, data):
        buf = self.buf + data if self.buf else data
        i = 0
        out = []
        n = len(buf)
        if not self.started:
            if n < 4:
                self.buf = buf
                return
            ln = _U32.unpack_from(buf)[0]
            if n < ln:
                self.buf = buf
                return
            if _U32.unpack_from(buf, 4)[0] == 80877103:  # SSLRequest: refuse, expect a plain startup
                self.t.write(b"N")
                self.buf = buf[ln:]
                return
            i = ln
            self.started = True
            out.append(_AUTH_OK)
        while n - i >= 5:
            t = buf[i:i + 1]
            ln = _U32.unpack_from(buf, i + 1)[0]
            if n - i - 1 < ln:
                break
            body = buf[i + 5:i + 1 + ln]
            i += 1 + ln
            if t == b"S":
                self.failed = False
                out.append(_READY)
            elif self.failed:
                continue
            elif t == b"P":
                name, rest = body.split(b"\x00", 1)
                sql = rest.split(b"\x00", 1)[0].decode().strip().upper().replace('"', "")
                if sql.startswith("SELECT") and "WHERE ID = $1" in sql:
                    self.stmts[name] = "select"
                elif sql.startswith("UPDATE") and "SET STATUS = $1" in sql:
                    self.stmts[name] = "update"
                else:
                    self.stmts[name] = "other"
                out.append(_PARSE_OK)
            elif t == b"B":
                j = body.index(b"\x00") + 1
                k = body.index(b"\x00", j)
                self.kind = self.stmts.get(body[j:k])
                j = k + 1
                nf = struct.unpack_from("!H", body, j)[0]
                j += 2 + 2 * nf
                npar = struct.unpack_from("!H", body, j)[0]
                j += 2
                params = []
                for _ in range(npar):
                    pl = struct.unpack_from("!i", body, j)[0]
                    j += 4
                    params.append(None if pl < 0 else body[j:j + pl].decode())
                    j += max(pl, 0)
                self.params = params
                out.append(_BIND_OK)
            elif t == b"D":
                out.append(_ROWDESC if self.kind == "select" else _NODATA)
            elif t == b"E":
                _Proto.queries += 1
                if self.kind == "select":
                    r = self.table.get(self.params[0])
                    if r is not None:
                        out.append(_row(r))
                    out.append(_msg(b"C", b"SELECT %d\x00" % (r is not None)))
                elif self.kind == "update":
                    r = self.table.get(self.params[1])
                    if r is not None:
                        r[9] = int(self.params[0])
                    out.append(_msg(b"C", b"UPDATE %d\x00" % (r is not None)))
                else:
                    out.append(_msg(b"E", b"SERROR\x00C0A000\x00Mbench endpoint: unsupported statement\x00\x00"))
                    self.failed = True
            elif t == b"X":
                self.t.close()
                return
        self.buf = buf[i:]
        if out:
            self.t.write(b"".join(out))


async def main(port: int, media: int, seed: int) -> int:
    from .generator import make_media
    _Proto.table = {m.id: list(m) for m in make_media(media, seed)}
    loop = asyncio.get_running_loop()
    # proto=IPPROTO_TCP: asyncio sets TCP_NODELAY only on sockets whose proto says TCP (accepted
    # sockets inherit it). With proto 0 a small reply written behind an unacknowledged segment
    # (TLS 1.3 session tickets, then the first response) waits ~40 ms for the client's delayed
    # ACK (Nagle) -- a stall no production server (nginx: tcp_nodelay on) has.
    sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM, socket.IPPROTO_TCP)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sock.bind(("127.0.0.1", port))
    srv = await loop.create_server(_Proto, sock=sock, backlog=1024)
    mon = fake_monitor()
    print(f"READY {sock.getsockname()[1]}", flush=True)
    stop = loop.create_future()
    loop.add_signal_handler(signal.SIGTERM, lambda: stop.done() or stop.set_result(None))
    await stop
    srv.close()
    mon.stop()
    print(f"DONE queries={_Proto.queries}", flush=True)
    print(mon.dump_line("pg"), flush=True)
    return 0


def main_native(port: int, media: int, seed: int) -> int:
    """The same endpoint on the native PgFake: its loop runs on a thread without the GIL; this
    thread waits for SIGTERM (blocked, so it reaches no other thread), then stops it and reports
    the queries and the loop's busy spells in the asyncio server's DONE / STALLS format."""
    import json
    import threading

    from ..ops.bench_native import PgFake
    from .generator import make_media
    signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGTERM})  # before the loop thread starts
    f = PgFake([list(m) for m in make_media(media, seed)])
    bound = f.listen(port)
    t = threading.Thread(target=f.run, name="pg-fake", daemon=True)
    t.start()
    print(f"READY {bound}", flush=True)
    signal.sigwait({signal.SIGTERM})
    f.stop()
    t.join(5)
    st = f.stats()
    print(f"DONE queries={st['queries']}", flush=True)
    ivs = st["stall_intervals"]
    print("STALLS " + json.dumps({
        "name": "pg", "loop_lag_max_us": round(st["max_busy_us"], 1), "loop_stalls": len(ivs),
        "loop_stalled_ms": round(sum(b - a for a, b in ivs) / 1e6, 2), "gc_pauses": 0,
        "gc_max_pause_us": None, "gc_stalls": 0, "stall_intervals": ivs}, separators=(",", ":")), flush=True)
    return 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--media", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--python", action="store_true", help="serve from the asyncio protocol, not the native PgFake")
    a = ap.parse_args()
    if a.python:
        sys.exit(asyncio.run(main(a.port, a.media, a.seed)))
    sys.exit(main_native(a.port, a.media, a.seed))
