"""Synthetic telemetry workload (BASELINE.json configs use synthetic events).

Produces a media table and a stream of ``TelemetryStatus`` /
``TelemetryProgress`` protobuf messages shaped like the triton stack's:
36-char UUID media ids, 24-hex Trello card ids, a handful of worker hosts,
progress 0-100. Every branch of both handlers is exercised: Trello-created
and API-created media, DEPLOYED transitions (Telegram + Emby), status values
with and without a flow-list mapping.
"""
from __future__ import annotations

import random
import uuid
from typing import List, Sequence, Tuple

from ..models import proto
from ..ops import codec_for, frames
from ..store import Media
from ..topics import PROGRESS_ID, STATUS_ID

STATUS_NAMES = ("QUEUED", "DOWNLOADING", "CONVERTING", "UPLOADING", "DEPLOYED", "ERRORED")


def bench_config(flow_statuses: Sequence[str] = ("queued", "downloading", "converting", "uploading", "deployed"),
                 telegram: bool = True, emby: bool = True) -> dict:
    """A complete config (reference key layout, §2.4) with all sinks enabled."""
    return {
        "keys": {
            "trello": {"key": "bench-key", "token": "bench-token"},
            "telegram": {"token": "123:bench"},
            "emby": {"token": "emby-bench"},
        },
        "instance": {
            "flow_ids": {s: f"list-{s}" for s in flow_statuses},
            "telegram": {"enabled": telegram, "channel": "-100123"},
            "emby": {"enabled": emby, "host": "http://emby.local:8096"},
        },
        "service": {"metrics": {"enabled": False}, "log": {"level": "info"}},
    }


def make_media(n: int, seed: int = 0, trello_fraction: float = 0.5) -> List[Media]:
    rng = random.Random(seed)
    out = []
    for i in range(n):
        mid = str(uuid.UUID(int=rng.getrandbits(128), version=4))
        trello = rng.random() < trello_fraction
        out.append(Media(
            id=mid, name=f"Show {i}", creator=1 if trello else 0,
            creatorId="%024x" % rng.getrandbits(96) if trello else "",
            metadataId=str(rng.randint(1, 50000)), status=rng.randint(0, 4)))
    return out


class Workload:
    """Deterministic event stream over a media population."""

    def __init__(self, n_media: int = 10000, seed: int = 0, progress_fraction: float = 0.9,
                 trello_fraction: float = 0.5, unknown_media_fraction: float = 0.0,
                 hosts: Sequence[str] = ("worker-0", "worker-1", "worker-2", "")):
        self.rng = random.Random(seed + 1)
        self.media = make_media(n_media, seed, trello_fraction)
        self.progress_fraction = progress_fraction
        self.unknown_media_fraction = unknown_media_fraction
        self.hosts = list(hosts)
        self._sc = codec_for(proto.load("api.TelemetryStatus"))
        self._pc = codec_for(proto.load("api.TelemetryProgress"))

    def events(self, n: int) -> List[Tuple[int, bytes]]:
        """``n`` (topic_id, payload) pairs."""
        rng = self.rng
        media = self.media
        nm = len(media)
        out = []
        sc, pc = self._sc.encode, self._pc.encode
        hosts = self.hosts
        for _ in range(n):
            if self.unknown_media_fraction and rng.random() < self.unknown_media_fraction:
                mid = "missing-" + str(rng.getrandbits(32))
            else:
                mid = media[rng.randrange(nm)].id
            st = rng.randrange(len(STATUS_NAMES))
            if rng.random() < self.progress_fraction:
                out.append((PROGRESS_ID, pc((mid, st, rng.randint(0, 100), hosts[rng.randrange(len(hosts))]))))
            else:
                out.append((STATUS_ID, sc((mid, st))))
        return out

    def framed(self, n: int) -> bytes:
        return frames(self.events(n))
