"""Postgres media store — ``triton-core/db`` (index.js:42,68,76,140) over :mod:`.pgwire`.

Table layout (our documented assumption; triton-core's migrations are not
vendored)::

    CREATE TABLE media (
        id TEXT PRIMARY KEY, name TEXT, creator INT, creator_id TEXT, type INT, source INT,
        source_uri TEXT, metadata INT, metadata_id TEXT, status INT)

``service.store.dsn`` is a ``postgres://`` URL (default ``dyn('postgres')``);
``service.store.table`` overrides the table name; ``create_schema: true``
creates it if missing.
"""
from __future__ import annotations

import re
from typing import Iterable, Optional

from .base import Media, MediaNotFound, MediaStore
from .pgwire import Pool

_COLS = "id, name, creator, creator_id, type, source, source_uri, metadata, metadata_id, status"
_IDENT = re.compile(r"^[A-Za-z_][A-Za-z0-9_]*(\.[A-Za-z_][A-Za-z0-9_]*)?$")


def row_to_media(r) -> Media:
    """One ``SELECT {_COLS}`` row as a Media (NULL text -> "", NULL/str numbers -> int). The
    compiled handlers (ops/csrc/py_handlers.cpp) take the all-int, no-NULL case themselves."""
    if None not in r and type(r[2]) is type(r[4]) is type(r[5]) is type(r[7]) is type(r[9]) is int:
        return Media._make(r)  # int columns arrived as int4/int8: no per-field conversion
    return Media(*(("" if v is None else v) if i in (0, 1, 3, 6, 8) else (0 if v is None else int(v))
                   for i, v in enumerate(r)))


class PostgresStore(MediaStore):
    name = "postgres"

    def __init__(self, dsn: Optional[str] = None, table: str = "media", pool_size: int = 4,
                 create_schema: bool = False):
        if dsn is None:
            from ..dynamics import dyn
            dsn = dyn("postgres")
        if not _IDENT.match(table):
            raise ValueError(f"invalid table name {table!r}")
        self.dsn = dsn
        self.table = table
        self.pool_size = pool_size
        self.create_schema = create_schema
        self._pool: Optional[Pool] = None
        self._select = f"SELECT {_COLS} FROM {table} WHERE id = $1"
        self._update = f"UPDATE {table} SET status = $1 WHERE id = $2"

    async def connect(self) -> None:
        if self._pool is None:
            self._pool = await Pool(self.dsn, self.pool_size).open()
            if self.create_schema:
                await self._pool.execute(
                    f"CREATE TABLE IF NOT EXISTS {self.table} (id TEXT PRIMARY KEY, name TEXT NOT NULL DEFAULT '', "
                    "creator INTEGER NOT NULL DEFAULT 0, creator_id TEXT NOT NULL DEFAULT '', "
                    "type INTEGER NOT NULL DEFAULT 0, source INTEGER NOT NULL DEFAULT 0, "
                    "source_uri TEXT NOT NULL DEFAULT '', metadata INTEGER NOT NULL DEFAULT 0, "
                    "metadata_id TEXT NOT NULL DEFAULT '', status INTEGER NOT NULL DEFAULT 0)")

    async def close(self) -> None:
        if self._pool is not None:
            await self._pool.close()
            self._pool = None

    async def _exec(self, sql: str, params=()):
        if self._pool is None:
            await self.connect()
        return await self._pool.execute(sql, params)

    async def update_status(self, media_id: str, status: int) -> None:
        await self._exec(self._update, (int(status), media_id))

    async def get_by_id(self, media_id: str) -> Media:
        pool = self._pool
        if pool is None:
            await self.connect()
            pool = self._pool
        rows, _ = await pool.execute(self._select, (media_id,))
        if not rows:
            raise MediaNotFound(media_id)
        return row_to_media(rows[0])

    async def upsert(self, media: Media) -> None:
        await self._exec(
            f"INSERT INTO {self.table} ({_COLS}) VALUES ($1,$2,$3,$4,$5,$6,$7,$8,$9,$10) "
            "ON CONFLICT (id) DO UPDATE SET name = EXCLUDED.name, creator = EXCLUDED.creator, "
            "creator_id = EXCLUDED.creator_id, type = EXCLUDED.type, source = EXCLUDED.source, "
            "source_uri = EXCLUDED.source_uri, metadata = EXCLUDED.metadata, "
            "metadata_id = EXCLUDED.metadata_id, status = EXCLUDED.status", tuple(media))

    async def upsert_many(self, medias: Iterable[Media]) -> None:
        for m in medias:
            await self.upsert(m)

    async def count(self) -> int:
        rows, _ = await self._exec(f"SELECT COUNT(*) FROM {self.table}")
        return int(rows[0][0])
