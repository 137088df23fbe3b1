"""Fake Trello / Telegram / Emby endpoint for the ``http_tcp`` bench config.

A minimal HTTP/1.1 keep-alive server: it answers every request with ``200 {}``.
Several copies can share one port (``SO_REUSEPORT``), so the server side is
never the bottleneck of the consumer being measured. It prints ``READY <port>``
once it is listening. On SIGTERM it prints ``DONE requests=<n>`` and exits.

    python -m beholder_amd.bench.http_sink_server --port 0 [--tls]

``--tls`` serves HTTPS with the bench's self-signed ``localhost`` / ``127.0.0.1`` certificate
(``bench/tls/``; a throwaway test key, never a deployment secret).
"""
from __future__ import annotations

import argparse
import asyncio
import signal
import os
import socket
import ssl
import sys

from .stallmon import fake_monitor

_RESP = b"HTTP/1.1 200 OK\r\nContent-Type: application/json; charset=utf-8\r\nContent-Length: 2\r\n\r\n{}"


class _Proto(asyncio.Protocol):
    count = 0

    def connection_made(self, transport):
        self.t = transport
        self.buf = b""

    def data_received(self, data):
        buf = self.buf + data if self.buf else data
        n = buf.count(b"\r\n\r\n")  # requests carry no body (query-string parameters only)
        if n:
            _Proto.count += n
            self.t.write(_RESP * n)
            buf = buf[buf.rfind(b"\r\n\r\n") + 4:]
        self.buf = buf


TLS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tls")
TLS_CERT = os.path.join(TLS_DIR, "cert.pem")


def server_ssl_context() -> ssl.SSLContext:
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(TLS_CERT, os.path.join(TLS_DIR, "key.pem"))
    return ctx


def warm_up(server_ctx: ssl.SSLContext) -> None:
    """One full handshake with ``server_ctx`` over memory BIOs, before READY. OpenSSL 3 fetches
    and caches its algorithm implementations (key exchange, signature, HKDF, AEAD) on first
    use, so a fresh process's first handshakes cost a few ms more than later ones. The
    endpoints this fake stands in for (api.trello.com, api.telegram.org) are long-running
    servers; without this, each run's fresh fake servers would bill their own cold start to
    the consumer's warm-up latency."""
    client_ctx = ssl.create_default_context(cafile=TLS_CERT)
    c_in, c_out, s_in, s_out = ssl.MemoryBIO(), ssl.MemoryBIO(), ssl.MemoryBIO(), ssl.MemoryBIO()
    cli = client_ctx.wrap_bio(c_in, c_out, server_hostname="127.0.0.1")
    srv = server_ctx.wrap_bio(s_in, s_out, server_side=True)
    done = [False, False]
    for _ in range(10):
        for i, (end, out, peer_in) in enumerate(((cli, c_out, s_in), (srv, s_out, c_in))):
            if not done[i]:
                try:
                    end.do_handshake()
                    done[i] = True
                except ssl.SSLWantReadError:
                    pass
            data = out.read()
            if data:
                peer_in.write(data)
        if all(done):
            return
    raise RuntimeError("TLS warm-up handshake did not finish")


async def main(port: int, tls: bool = False) -> int:
    loop = asyncio.get_running_loop()
    # proto=IPPROTO_TCP: asyncio sets TCP_NODELAY only on sockets whose proto says TCP (accepted
    # sockets inherit it). With proto 0 a small reply written behind an unacknowledged segment
    # (TLS 1.3 session tickets, then the first response) waits ~40 ms for the client's delayed
    # ACK (Nagle) -- a stall no production server (nginx: tcp_nodelay on) has.
    sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM, socket.IPPROTO_TCP)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sock.bind(("127.0.0.1", port))
    ctx = server_ssl_context() if tls else None
    if ctx is not None:
        warm_up(ctx)
    srv = await loop.create_server(_Proto, sock=sock, backlog=1024, ssl=ctx)
    mon = fake_monitor()
    print(f"READY {sock.getsockname()[1]}", flush=True)
    stop = loop.create_future()
    loop.add_signal_handler(signal.SIGTERM, lambda: stop.done() or stop.set_result(None))
    await stop
    srv.close()
    mon.stop()
    print(f"DONE requests={_Proto.count}", flush=True)
    print(mon.dump_line("https" if tls else "http"), flush=True)
    return 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--tls", action="store_true")
    a = ap.parse_args()
    sys.exit(asyncio.run(main(a.port, a.tls)))
