"""Fake Trello / Telegram / Emby endpoint for the ``http_tcp`` bench config.

A minimal HTTP/1.1 keep-alive server: it answers every request with ``200 {}``.
Several copies can share one port (``SO_REUSEPORT``), so the server side is
never the bottleneck of the consumer being measured. It prints ``READY <port>``
once it is listening. On SIGTERM it prints ``DONE requests=<n>`` and exits.

    python -m beholder_amd.bench.http_sink_server --port 0
"""
from __future__ import annotations

import argparse
import asyncio
import signal
import socket
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


async def main(port: int) -> int:
    loop = asyncio.get_running_loop()
    sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sock.bind(("127.0.0.1", port))
    srv = await loop.create_server(_Proto, sock=sock, backlog=1024)
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
    sys.exit(asyncio.run(main(ap.parse_args().port)))
