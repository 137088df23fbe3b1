"""In-memory media store (tests, benches, single-process deployments)."""
from __future__ import annotations

from typing import Dict, Iterable, Optional

from .base import Media, MediaNotFound, MediaStore, untrack_row


class MemoryStore(MediaStore):
    name = "memory"

    def __init_subclass__(cls, **kw):
        # a subclass that overrides an async accessor must not be bypassed by the sync fast path
        super().__init_subclass__(**kw)
        if cls.get_by_id is not MemoryStore.get_by_id and cls.get_by_id_nowait is MemoryStore.get_by_id_nowait:
            cls.get_by_id_nowait = None
        if (cls.update_status is not MemoryStore.update_status
                and cls.update_status_nowait is MemoryStore.update_status_nowait):
            cls.update_status_nowait = None

    def __init__(self, medias: Optional[Iterable[Media]] = None):
        self._rows: Dict[str, Media] = {}
        self.update_calls = 0
        self.get_calls = 0
        for m in medias or ():
            self._rows[m.id] = m

    def describe(self) -> str:
        return f"memory ({len(self._rows)} rows)"

    def update_status_nowait(self, media_id: str, status: int) -> None:
        self.update_calls += 1
        m = self._rows.get(media_id)
        if m is not None:
            self._rows[media_id] = untrack_row(m._replace(status=int(status)))

    def get_by_id_nowait(self, media_id: str) -> Media:
        self.get_calls += 1
        m = self._rows.get(media_id)
        if m is None:
            raise MediaNotFound(media_id)
        return m  # immutable row: safe to share

    async def update_status(self, media_id: str, status: int) -> None:
        self.update_status_nowait(media_id, status)

    async def get_by_id(self, media_id: str) -> Media:
        return self.get_by_id_nowait(media_id)

    async def upsert(self, media: Media) -> None:
        self._rows[media.id] = media

    async def count(self) -> int:
        return len(self._rows)

    def snapshot(self) -> Dict[str, Media]:
        return dict(self._rows)
