"""Shared fakes for handler / service tests."""
from __future__ import annotations

import asyncio
import copy
from typing import Optional

from beholder_amd.config import Config
from beholder_amd.handlers import TelemetryHandlers, native_handlers
from beholder_amd.metrics import Registry
from beholder_amd.models import proto
from beholder_amd.ops import Delivery, Settler
from beholder_amd.sinks import EmbyClient, RecordingHttpClient, TelegramClient, TrelloClient, parse_query
from beholder_amd.store import Media, MemoryStore
from beholder_amd.topics import PROGRESS_ID, STATUS_ID
from beholder_amd.utils.log import Logger, MemoryStream

BASE_CFG = {
    "keys": {
        "trello": {"key": "TK", "token": "TT"},
        "telegram": {"token": "123:TG"},
        "emby": {"token": "EMBYKEY"},
    },
    "instance": {
        "flow_ids": {"queued": "L-queued", "downloading": "L-dl", "converting": "L-conv", "deployed": "L-dep"},
        "telegram": {"enabled": True, "channel": "-1001"},
        "emby": {"enabled": True, "host": "http://emby:8096"},
    },
}

STATUS = proto.load("api.TelemetryStatus")
PROGRESS = proto.load("api.TelemetryProgress")
ENUM = {n: v for v, n in STATUS.enum("TelemetryStatusEntry")[0].items()}  # name -> number


def cfg(overrides: Optional[dict] = None, env: Optional[dict] = None) -> Config:
    d = copy.deepcopy(BASE_CFG)
    if overrides:
        from beholder_amd.config import deep_merge
        deep_merge(d, overrides)
    return Config.from_dict(d, env=env or {})


def status_msg(media_id: str, status) -> bytes:
    s = ENUM[status] if isinstance(status, str) else status
    return proto.encode(STATUS, {"mediaId": media_id, "status": s})


def progress_msg(media_id: str, status, progress=0, host: str = "") -> bytes:
    s = ENUM[status] if isinstance(status, str) else status
    return proto.encode(PROGRESS, {"mediaId": media_id, "status": s, "progress": progress, "host": host})


# which handler implementation Rig drives: "python" (handlers.py) or "native" (py_handlers.cpp);
# tests/test_handlers.py runs every case under both
HANDLER_IMPL = "python"
# whether Rig's default store and HTTP client suspend at every call, as production's socket
# clients always do (tests/test_handlers.py runs every case both ways): the compiled handlers
# then leave C at each await and resume in their state machine (py_handlers.cpp, states 1-6)
SUSPEND = False


def suspending(base):
    """``base`` (a MemoryStore class) whose every access yields to the loop once before it runs
    (a network store's shape). Its synchronous accessors are hidden from the handlers, so
    they await the coroutines."""
    class Suspending(base):
        async def update_status(self, media_id, status):
            await asyncio.sleep(0)
            base.update_status_nowait(self, media_id, status)

        async def get_by_id(self, media_id):
            await asyncio.sleep(0)
            return base.get_by_id_nowait(self, media_id)
    Suspending.__name__ = Suspending.__qualname__ = "Suspending" + base.__name__
    return Suspending


SuspendingStore = suspending(MemoryStore)


class SuspendingHttpClient(RecordingHttpClient):
    """Records a request, yields to the loop once, then answers it (rules and faults included),
    so every answer, a failure too, reaches the handler through a resumed await (a socket
    client's shape; the plain recorder answers within the call)."""

    async def request(self, method, url, *, params=None, timeout=None):
        m = method.upper()
        full = self.record(m, url, params)
        await asyncio.sleep(0)
        return self.answer(m, full)


async def _await(aw):
    return await aw


class Rig:
    """Handlers wired to an in-memory store, a recording HTTP client and a captured log."""

    def __init__(self, config: Optional[Config] = None, medias=(), no_trello: Optional[bool] = None,
                 http: Optional[RecordingHttpClient] = None, positional_args: str = "append", store=None):
        self.config = config or cfg()
        self.http = http or (SuspendingHttpClient() if SUSPEND else RecordingHttpClient())
        self.store = store if store is not None else (SuspendingStore if SUSPEND else MemoryStore)(list(medias))
        self.stream = MemoryStream()
        self.log = Logger(stream=self.stream, positional_args=positional_args)
        self.registry = Registry()
        self.progress = self.registry.counter("beholder_progress_updates_total",
                                              "Total number of messages processed in this processes lifetime",
                                              ["status"])
        self.comments = self.registry.counter("beholder_trello_comments",
                                              "Total trello comments crreated in this processes lifetime")
        keys = self.config.root.require("keys.trello")
        self.h = TelemetryHandlers(
            config=self.config, store=self.store,
            trello=TrelloClient(keys.get("key"), keys.get("token"), self.http),
            telegram=TelegramClient(None, self.http), emby=EmbyClient(None, None, self.http),
            progress_counter=self.progress, comments_counter=self.comments, logger=self.log,
            no_trello=no_trello)
        self.settler = Settler()
        self.impl = self.h if HANDLER_IMPL == "python" else native_handlers(self.h)

    def delivery(self, topic_id: int, body: bytes) -> Delivery:
        return Delivery(body, topic_id, 1, self.settler)

    def status(self, body: bytes):
        d = self.delivery(STATUS_ID, body)
        exc = None
        try:
            asyncio.run(_await(self.impl.on_status(d)))
        except Exception as e:  # noqa: BLE001
            exc = e
        return d, exc

    def progress_(self, body: bytes):
        d = self.delivery(PROGRESS_ID, body)
        asyncio.run(_await(self.impl.on_progress(d)))
        return d

    def calls(self):
        return [(m, u.split("?")[0], parse_query(u)) for m, u in self.http.calls]

    def msgs(self, level: Optional[int] = None):
        self.log.flush()
        return [r.get("msg") for r in self.stream.records() if level is None or r["level"] == level]


def trello_media(mid="m1", status="QUEUED", **kw) -> Media:
    return Media(id=mid, name=kw.pop("name", "Cowboy Bebop"), creator=1, creatorId=kw.pop("card", "card1"),
                 metadataId=kw.pop("metadataId", "1"), status=ENUM[status], **kw)


def api_media(mid="m2", status="QUEUED", **kw) -> Media:
    return Media(id=mid, name=kw.pop("name", "Trigun"), creator=0, creatorId="", metadataId="2",
                 status=ENUM[status], **kw)
