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

SCHEMA = """
CREATE TABLE IF NOT EXISTS media (
    id          TEXT PRIMARY KEY,
    name        TEXT NOT NULL DEFAULT '',
    creator     INTEGER NOT NULL DEFAULT 0,
    creator_id  TEXT NOT NULL DEFAULT '',
    type        INTEGER NOT NULL DEFAULT 0,
    source      INTEGER NOT NULL DEFAULT 0,
    source_uri  TEXT NOT NULL DEFAULT '',
    metadata    INTEGER NOT NULL DEFAULT 0,
    metadata_id TEXT NOT NULL DEFAULT '',
    status      INTEGER NOT NULL DEFAULT 0
)
"""
_COLS = "id, name, creator, creator_id, type, source, source_uri, metadata, metadata_id, status"


class SqliteStore(MediaStore):
    name = "sqlite"

    def __init__(self, path: str = ":memory:"):
        self.path = path
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="sqlite")
        self._conn: Optional[sqlite3.Connection] = None

    def _open(self) -> None:
        conn = sqlite3.connect(self.path, check_same_thread=False, isolation_level=None)
        conn.execute("PRAGMA journal_mode=WAL") if self.path != ":memory:" else None
        conn.execute(SCHEMA)
        self._conn = conn

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
            self._need().execute("UPDATE media SET status = ? WHERE id = ?", (int(status), media_id))
        await self._run(q)

    async def get_by_id(self, media_id: str) -> Media:
        def q():
            return self._need().execute(f"SELECT {_COLS} FROM media WHERE id = ?", (media_id,)).fetchone()
        row = await self._run(q)
        if row is None:
            raise MediaNotFound(media_id)
        return Media(*row)

    async def upsert(self, media: Media) -> None:
        def q():
            self._need().execute(
                f"INSERT INTO media ({_COLS}) VALUES (?,?,?,?,?,?,?,?,?,?) "
                "ON CONFLICT(id) DO UPDATE SET name=excluded.name, creator=excluded.creator, "
                "creator_id=excluded.creator_id, type=excluded.type, source=excluded.source, "
                "source_uri=excluded.source_uri, metadata=excluded.metadata, "
                "metadata_id=excluded.metadata_id, status=excluded.status",
                tuple(getattr(media, f) for f in Media._fields))
        await self._run(q)

    async def upsert_many(self, medias) -> None:
        rows = [tuple(getattr(m, f) for f in Media._fields) for m in medias]

        def q():
            c = self._need()
            c.execute("BEGIN")
            c.executemany(f"INSERT OR REPLACE INTO media ({_COLS}) VALUES (?,?,?,?,?,?,?,?,?,?)", rows)
            c.execute("COMMIT")
        await self._run(q)

    async def count(self) -> int:
        def q():
            return self._need().execute("SELECT COUNT(*) FROM media").fetchone()[0]
        return await self._run(q)
