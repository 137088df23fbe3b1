"""In-memory media store (tests, benches, single-process deployments)."""
from __future__ import annotations

from typing import Dict, Iterable, Optional

from .base import Media, MediaNotFound, MediaStore


class MemoryStore(MediaStore):
    name = "memory"

    def __init__(self, medias: Optional[Iterable[Media]] = None):
        self._rows: Dict[str, Media] = {}
        self.update_calls = 0
        self.get_calls = 0
        for m in medias or ():
            self._rows[m.id] = m

    async def update_status(self, media_id: str, status: int) -> None:
        self.update_calls += 1
        m = self._rows.get(media_id)
        if m is not None:
            self._rows[media_id] = m._replace(status=int(status))

    async def get_by_id(self, media_id: str) -> Media:
        self.get_calls += 1
        m = self._rows.get(media_id)
        if m is None:
            raise MediaNotFound(media_id)
        return m  # immutable row: safe to share

    async def upsert(self, media: Media) -> None:
        self._rows[media.id] = media

    async def count(self) -> int:
        return len(self._rows)

    def snapshot(self) -> Dict[str, Media]:
        return dict(self._rows)
