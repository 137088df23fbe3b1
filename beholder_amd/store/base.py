"""Media storage interface — parity with ``triton-core/db`` as beholder uses it.

The reference uses exactly two methods of ``new Storage()`` (index.js:42):

* ``updateStatus(mediaId, status)`` — index.js:68 (status handler, before the
  ``NO_TRELLO`` short-circuit);
* ``getByID(mediaId)`` → ``{creator, creatorId, status, name, metadataId}`` —
  index.js:76 and :140.

Semantics we pin down (triton-core is not vendored, so these are documented
choices): ``update_status`` of an unknown id is a no-op (an SQL ``UPDATE``
matching zero rows); ``get_by_id`` of an unknown id raises
:class:`MediaNotFound` — in the reference ``media.creator`` on a missing row
throws a ``TypeError`` either way, so the handler-level outcome is identical
(status: un-acked, Q1; progress: warn + ack, Q7).
"""
from __future__ import annotations

import abc
from typing import Iterable, NamedTuple, Optional
from ..ops import native as _native


class MediaNotFound(LookupError):
    def __init__(self, media_id: str):
        super().__init__(f"media {media_id} not found")  # the stand-in db.js text (tests/reference_oracle.py)
        self.media_id = media_id


class StoreError(RuntimeError):
    pass


# untrack_row(row) -> row: a row of atoms leaves the cyclic collector at once. NamedTuple rows are
# otherwise tracked for life, and a store that replaces or reads many of them keeps the young
# generation full of them (the compiled handlers do the same for the rows they make).
untrack_row = _native.untrack_row


class Media(NamedTuple):
    """One media row (fields of ``api.Media``, see models/proto/api.proto).

    Rows are immutable values: a read returns the stored tuple itself (no
    per-read copy), an update stores a new tuple (``_replace``).
    """

    id: str
    name: str = ""
    creator: int = 0          # CreatorType; TRELLO == 1 (index.js:79)
    creatorId: str = ""       # Trello card id (index.js:82-83,147)
    type: int = 0
    source: int = 0
    sourceURI: str = ""
    metadata: int = 0
    metadataId: str = ""      # Kitsu id (index.js:103)
    status: int = 0           # TelemetryStatusEntry (index.js:94)


FIELDS = Media._fields


class MediaStore(abc.ABC):
    """Async media-store interface. Implementations: memory, sqlite, postgres."""

    name = "abstract"

    async def connect(self) -> None:
        """Open connections (called once by the service at startup)."""

    async def close(self) -> None:
        """Release resources."""

    def describe(self) -> str:
        """What the store reads and writes, for the startup log line (``service.py``)."""
        return self.name

    @abc.abstractmethod
    async def update_status(self, media_id: str, status: int) -> None:
        """``db.updateStatus`` (index.js:68)."""

    @abc.abstractmethod
    async def get_by_id(self, media_id: str) -> Media:
        """``db.getByID`` (index.js:76,140); raises :class:`MediaNotFound`."""

    #: Optional synchronous accessors for stores that answer without I/O (memory).
    #: Handlers call these when not None and skip one coroutine per message; the
    #: semantics (return value / MediaNotFound) are identical to the async methods.
    get_by_id_nowait = None
    update_status_nowait = None

    # -- administration (used by tools/tests; not on the reference hot path) --
    @abc.abstractmethod
    async def upsert(self, media: Media) -> None:
        ...

    async def upsert_many(self, medias: Iterable[Media]) -> None:
        for m in medias:
            await self.upsert(m)

    @abc.abstractmethod
    async def count(self) -> int:
        ...

    # camelCase aliases (triton-core API names)
    async def updateStatus(self, media_id: str, status: int) -> None:  # noqa: N802
        await self.update_status(media_id, status)

    async def getByID(self, media_id: str) -> Media:  # noqa: N802
        return await self.get_by_id(media_id)


def open_store(backend: str, dsn: Optional[str] = None, **kw) -> MediaStore:
    """Factory used by the service from ``service.store`` config."""
    backend = (backend or "memory").lower()
    if backend == "memory":
        from .memory import MemoryStore
        kw.pop("table", None), kw.pop("columns", None)  # no table: nothing to map
        return MemoryStore(**kw)
    if backend == "sqlite":
        from .sqlite import SqliteStore
        return SqliteStore(dsn or ":memory:", **kw)
    if backend in ("postgres", "postgresql", "pg"):
        from .postgres import PostgresStore
        return PostgresStore(dsn, **kw)
    raise ValueError(f"unknown store backend {backend!r} (memory|sqlite|postgres)")
