"""Local fake HTTP endpoint for Trello / Telegram / Emby (integration tests, plumbing bench).

A real TCP HTTP/1.1 server on 127.0.0.1 running in its own thread + event
loop. It answers every request with ``200 {}`` (or a configured status per
path prefix) and records ``(method, path, query)``.
"""
from __future__ import annotations

import asyncio
import threading
from typing import Dict, List, Tuple
from urllib.parse import parse_qsl, urlsplit


class FakeHttpServer:
    def __init__(self, host: str = "127.0.0.1"):
        self.host = host
        self.port = 0
        self.requests: List[Tuple[str, str, Dict[str, str]]] = []
        self.status_for: Dict[str, int] = {}
        self._loop = None
        self._server = None
        self._thread = None
        self._ready = threading.Event()
        self._lock = threading.Lock()

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    async def _handle(self, reader, writer):
        try:
            while True:
                try:
                    head = await reader.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, ConnectionError):
                    return
                lines = head.decode("latin-1").split("\r\n")
                method, target, _ = lines[0].split(" ", 2)
                hdrs = {}
                for ln in lines[1:]:
                    if ":" in ln:
                        k, v = ln.split(":", 1)
                        hdrs[k.strip().lower()] = v.strip()
                n = int(hdrs.get("content-length", "0") or 0)
                if n:
                    await reader.readexactly(n)
                u = urlsplit(target)
                with self._lock:
                    self.requests.append((method, u.path, dict(parse_qsl(u.query, keep_blank_values=True))))
                status = 200
                for pref, st in self.status_for.items():
                    if u.path.startswith(pref):
                        status = st
                body = b"{}"
                writer.write(f"HTTP/1.1 {status} X\r\nContent-Type: application/json\r\n"
                             f"Content-Length: {len(body)}\r\n\r\n".encode() + body)
                await writer.drain()
                if hdrs.get("connection", "").lower() == "close":
                    return
        finally:
            try:
                writer.close()
            except Exception:  # noqa: BLE001
                pass

    def _run(self):
        self._loop = asyncio.new_event_loop()
        asyncio.set_event_loop(self._loop)

        async def start():
            self._server = await asyncio.start_server(self._handle, self.host, 0)
            self.port = self._server.sockets[0].getsockname()[1]
            self._ready.set()

        self._loop.run_until_complete(start())
        self._loop.run_forever()
        self._server.close()
        self._loop.run_until_complete(self._server.wait_closed())
        self._loop.close()

    def start(self) -> "FakeHttpServer":
        self._thread = threading.Thread(target=self._run, daemon=True, name="fake-http")
        self._thread.start()
        self._ready.wait(10)
        return self

    def stop(self) -> None:
        if self._loop is not None:
            self._loop.call_soon_threadsafe(self._loop.stop)
        if self._thread is not None:
            self._thread.join(5)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
