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
    srv = await loop.create_server(_Proto, sock=sock, backlog=1024, ssl=server_ssl_context() if tls else None)
    print(f"READY {sock.getsockname()[1]}", flush=True)
    stop = loop.create_future()
    loop.add_signal_handler(signal.SIGTERM, lambda: stop.done() or stop.set_result(None))
    await stop
    srv.close()
    print(f"DONE requests={_Proto.count}", flush=True)
    return 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--tls", action="store_true")
    a = ap.parse_args()
    sys.exit(asyncio.run(main(a.port, a.tls)))
