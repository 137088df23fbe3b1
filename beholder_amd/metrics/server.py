"""HTTP exposer for the registry — ``Prom.expose()`` (index.js:28).

A tiny asyncio HTTP/1.1 server (no framework: it only serves a handful of
GETs) with:

* ``GET /metrics`` — Prometheus text exposition (the reference's scrape path);
* ``GET /healthz`` — ``200 ok`` once the service is consuming, else ``503``
  (liveness/readiness for the k8s deployment the reference runs in);
* ``GET /stats`` — JSON snapshot of ingest/ack statistics.
"""
from __future__ import annotations

import asyncio
import json
from typing import Callable, Optional

from .registry import Registry

_REASONS = {200: "OK", 404: "Not Found", 405: "Method Not Allowed", 500: "Internal Server Error",
            503: "Service Unavailable", 400: "Bad Request"}


class MetricsServer:
    def __init__(self, registry: Registry, host: str = "0.0.0.0", port: int = 3000,
                 health: Optional[Callable[[], bool]] = None,
                 stats: Optional[Callable[[], dict]] = None, logger=None):
        self.registry = registry
        self.host = host
        self.port = port
        self._health = health
        self._stats = stats
        self._server: Optional[asyncio.AbstractServer] = None
        self.log = logger

    @property
    def bound_port(self) -> int:
        if self._server and self._server.sockets:
            return self._server.sockets[0].getsockname()[1]
        return self.port

    async def start(self) -> "MetricsServer":
        self._server = await asyncio.start_server(self._handle, self.host, self.port)
        return self

    async def stop(self) -> None:
        if self._server:
            self._server.close()
            await self._server.wait_closed()
            self._server = None

    def _respond(self, status: int, body: bytes, ctype: str, head_only: bool = False) -> bytes:
        hdr = (f"HTTP/1.1 {status} {_REASONS.get(status, 'OK')}\r\n"
               f"Content-Type: {ctype}\r\nContent-Length: {len(body)}\r\nConnection: close\r\n\r\n").encode()
        return hdr if head_only else hdr + body

    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            try:
                head = await asyncio.wait_for(reader.readuntil(b"\r\n\r\n"), timeout=10)
            except (asyncio.IncompleteReadError, asyncio.LimitOverrunError, asyncio.TimeoutError):
                return
            line = head.split(b"\r\n", 1)[0].decode("latin-1")
            parts = line.split()
            if len(parts) < 2:
                writer.write(self._respond(400, b"bad request\n", "text/plain"))
                return
            method, target = parts[0], parts[1].split("?", 1)[0]
            if method not in ("GET", "HEAD"):
                writer.write(self._respond(405, b"method not allowed\n", "text/plain"))
                return
            head_only = method == "HEAD"
            if target == "/metrics":
                try:
                    body = self.registry.render().encode()
                except Exception as e:  # never crash the scrape loop
                    writer.write(self._respond(500, f"{e}\n".encode(), "text/plain"))
                    return
                writer.write(self._respond(200, body, Registry.CONTENT_TYPE, head_only))
            elif target in ("/healthz", "/health", "/ready"):
                ok = self._health() if self._health else True
                writer.write(self._respond(200 if ok else 503, b"ok\n" if ok else b"not ready\n",
                                           "text/plain", head_only))
            elif target == "/stats":
                data = self._stats() if self._stats else {}
                writer.write(self._respond(200, json.dumps(data, default=str).encode(), "application/json",
                                           head_only))
            else:
                writer.write(self._respond(404, b"not found\n", "text/plain", head_only))
        finally:
            try:
                await writer.drain()
                writer.close()
                await writer.wait_closed()
            except (ConnectionError, OSError):
                pass
