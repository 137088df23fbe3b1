"""Postgres media store — ``triton-core/db`` (index.js:42,68,76,140) over :mod:`.pgwire`.

Table layout: :mod:`.schema` (our documented default guess, triton-core's migrations are not
vendored)::

    CREATE TABLE media (
        id TEXT PRIMARY KEY, name TEXT, creator INT, creator_id TEXT, type INT, source INT,
        source_uri TEXT, metadata INT, metadata_id TEXT, status INT)

``service.store.dsn`` is a ``postgres://`` URL (default ``dyn('postgres')``);
``service.store.table`` and ``service.store.columns`` override the table and column names;
``create_schema: true`` creates the table if missing.
"""
from __future__ import annotations

from typing import Iterable, Mapping, Optional

from .base import untrack_row, Media, MediaNotFound, MediaStore
from .pgwire import Pool
from .schema import MediaSchema, pg_ph


def row_to_media(r) -> Media:
    """One ``SELECT`` row (Media field order) as a Media (NULL text -> "", NULL/str numbers ->
    int). The compiled handlers (ops/csrc/py_handlers.cpp) take the all-int, no-NULL case
    themselves."""
    if None not in r and type(r[2]) is type(r[4]) is type(r[5]) is type(r[7]) is type(r[9]) is int:
        return untrack_row(Media._make(r))  # int columns arrived as int4/int8: no per-field conversion
    return untrack_row(Media(*(("" if v is None else v) if i in (0, 1, 3, 6, 8) else (0 if v is None else int(v))
                               for i, v in enumerate(r))))


class PostgresStore(MediaStore):
    name = "postgres"

    def __init__(self, dsn: Optional[str] = None, table: str = "media", pool_size: int = 4,
                 create_schema: bool = False, columns: Optional[Mapping[str, str]] = None, spread_at: int = 8,
                 stall_timeout_s: Optional[float] = 30.0, min_connections: Optional[int] = None):
        if dsn is None:
            from ..dynamics import dyn
            dsn = dyn("postgres")
        self.schema = MediaSchema(table, columns)
        self.dsn = dsn
        self.table = table
        self.pool_size = pool_size
        self.spread_at = spread_at  # queries in flight on every connection before the pool grows
        self.stall_timeout_s = stall_timeout_s  # Pool: drop a connection whose replies stopped
        # opened at connect(); None = pool_size (the startup burst spreads over the whole pool)
        self.min_connections = pool_size if min_connections is None else min_connections
        self.create_schema = create_schema
        self._pool: Optional[Pool] = None
        # the compiled handlers issue these two texts themselves (py_handlers.cpp pg_execute)
        self._select = self.schema.select_by_id(pg_ph)
        self._update = self.schema.update_status(pg_ph)
        self._upsert = self.schema.upsert(pg_ph)

    def describe(self) -> str:
        return f"postgres {self.schema.describe()}"

    async def connect(self) -> None:
        if self._pool is None:
            self._pool = await Pool(self.dsn, self.pool_size, self.spread_at, self.stall_timeout_s,
                                    min_open=self.min_connections).open()
            if self.create_schema:
                await self._pool.execute(self.schema.create_table())

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
        await self._exec(self._upsert, tuple(media))

    async def upsert_many(self, medias: Iterable[Media]) -> None:
        for m in medias:
            await self.upsert(m)

    async def count(self) -> int:
        rows, _ = await self._exec(self.schema.count())
        return int(rows[0][0])
