"""SQLite media store.

SQLite calls are synchronous; they run on a dedicated single worker thread so
the event loop never blocks on disk I/O, and statements are serialised (one
connection, ``check_same_thread=False`` owned by that thread).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import sqlite3
from typing import Optional

from .base import Media, MediaNotFound, MediaStore
from .schema import MediaSchema, sqlite_ph

class SqliteStore(MediaStore):
    name = "sqlite"

    def __init__(self, path: str = ":memory:", table: str = "media", columns=None):
        self.path = path
        self.schema = sc = MediaSchema(table, columns)
        self._select = sc.select_by_id(sqlite_ph)
        self._update = sc.update_status(sqlite_ph)
        self._upsert = sc.upsert(sqlite_ph, excluded="excluded")
        self._replace = self._upsert.split(" ON CONFLICT", 1)[0].replace("INSERT INTO", "INSERT OR REPLACE INTO", 1)
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="sqlite")
        self._conn: Optional[sqlite3.Connection] = None

    def _open(self) -> None:
        conn = sqlite3.connect(self.path, check_same_thread=False, isolation_level=None)
        conn.execute("PRAGMA journal_mode=WAL") if self.path != ":memory:" else None
        conn.execute(self.schema.create_table())
        self._conn = conn

    def describe(self) -> str:
        return f"sqlite {self.path} {self.schema.describe()}"

    async def _run(self, fn, *args):
        loop = asyncio.get_running_loop()
        return await loop.run_in_executor(self._pool, fn, *args)

    async def connect(self) -> None:
        if self._conn is None:
            await self._run(self._open)

    async def close(self) -> None:
        if self._conn is not None:
            await self._run(self._conn.close)
            self._conn = None
        self._pool.shutdown(wait=True)

    def _need(self) -> sqlite3.Connection:
        if self._conn is None:
            self._open()
        return self._conn  # type: ignore[return-value]

    async def update_status(self, media_id: str, status: int) -> None:
        def q():
            self._need().execute(self._update, (int(status), media_id))
        await self._run(q)

    async def get_by_id(self, media_id: str) -> Media:
        def q():
            return self._need().execute(self._select, (media_id,)).fetchone()
        row = await self._run(q)
        if row is None:
            raise MediaNotFound(media_id)
        return Media(*row)

    async def upsert(self, media: Media) -> None:
        def q():
            self._need().execute(self._upsert, tuple(media))
        await self._run(q)

    async def upsert_many(self, medias) -> None:
        rows = [tuple(getattr(m, f) for f in Media._fields) for m in medias]

        def q():
            c = self._need()
            c.execute("BEGIN")
            c.executemany(self._replace, rows)
            c.execute("COMMIT")
        await self._run(q)

    async def count(self) -> int:
        def q():
            return self._need().execute(self.schema.count()).fetchone()[0]
        return await self._run(q)
