"""Reference-executed parity gate: the reference's own ``index.js`` against both handler implementations.

``scripts/reference_node/oracle.js`` runs ``/root/reference/index.js`` (loaded in place, never
copied) on the image's Node under the stand-ins in ``scripts/reference_node/stubs`` and records,
per delivered event, acks, the listener's rejection, whether decode threw, every sink request
(method + full URL) and every log line; at the end it records the counters and the media
table's statuses. :func:`run_python` replays the same scenario through this repo's handlers
(``handlers.py`` or the compiled ``ops/csrc/py_handlers.cpp``) and records the same things;
:func:`diff` compares them field by field. :func:`run_service` replays it through the whole consumer
instead (an in-process AMQP broker, ``AmqpSource``, the service's dispatch and its acks), as
production receives events.

A scenario (:func:`make_scenario`) is a seeded random config, media table, sink-fault list and
event stream. The streams are built to reach every branch of index.js:50-155, malformed bodies
included (truncated fields, wrong wire types, unknown fields and groups, invalid UTF-8, field
number 0). Modes: ``base``, ``no_trello`` (NO_TRELLO set, index.js:70), ``faults`` (transport
errors and non-2xx answers from Trello, Telegram and Emby, index.js:92-122), ``drop``
(``positional_args: drop``, pino@5's exact message text, quirk Q11) and ``reread`` (another writer
updates chosen rows between the listener's ``updateStatus`` and its ``getByID``, index.js:68,76:
the re-read status differs from the message's, so a handler that keys the hooks off the message's
status instead of the row's, quirk Q3 at index.js:94, or the list off the row's instead of the
message's, index.js:74-80, diverges from the reference).

What the stand-ins assume is listed in their headers. The ones that touch this comparison:
``triton-core/db`` (not vendored) rejects ``getByID`` of an unknown id with the text in
``NOT_FOUND`` and ignores ``updateStatus`` of one; ``trello@0.9.1`` resolves on any HTTP status;
``request-promise`` rejects non-2xx with ``StatusCodeError``.

Run by ``tests/test_reference_oracle.py``; by hand:
``python tests/reference_oracle.py --seeds 10 --events 600``.
"""
from __future__ import annotations

import asyncio
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile
from typing import Dict, List, Optional

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
if HERE not in sys.path:
    sys.path.insert(0, HERE)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from beholder_amd.config import Config  # noqa: E402
from beholder_amd.models import proto  # noqa: E402
from beholder_amd.ops import codec_for  # noqa: E402
from beholder_amd.sinks import RecordingHttpClient  # noqa: E402
from beholder_amd.store import Media, MemoryStore  # noqa: E402

REFERENCE_INDEX = os.environ.get("BEHOLDER_REFERENCE_INDEX", "/root/reference/index.js")
ORACLE_JS = os.path.join(ROOT, "scripts", "reference_node", "oracle.js")
STUBS = os.path.join(ROOT, "scripts", "reference_node", "stubs")
NODE = shutil.which("node")
NOT_FOUND = "media {id} not found"  # beholder_amd.store.base.MediaNotFound's text
# sendMessage for a row named "Cowboy Bebop" (query order chat_id, text, parse_mode; RFC 3986)
TELEGRAM_FAULT_PREFIX = ("https://api.telegram.org/bot123:TG/sendMessage?chat_id=-1001&text="
                         "%2ANew%20Anime%3A%2A%20Cowboy%20Bebop")
MODES = ("base", "no_trello", "faults", "drop", "reread", "concurrent")
CONCURRENT_CAP = 4  # deliveries in flight at once in mode "concurrent"

_S = codec_for(proto.load("api.TelemetryStatus"))
_P = codec_for(proto.load("api.TelemetryProgress"))


def available() -> bool:
    return NODE is not None and os.path.exists(REFERENCE_INDEX)


# ---------------------------------------------------------------------------------- scenarios ---
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _malformed(rng: random.Random, ids: List[str]) -> bytes:
    """Bodies that reach protobufjs's reader edge cases (ops/csrc/pbjs.hpp lists them)."""
    mid = rng.choice(ids).encode()
    st = rng.randrange(-1, 8)
    valid = _P.encode((mid.decode(), st, rng.randrange(0, 101), "w")) if rng.random() < 0.5 else \
        _S.encode((mid.decode(), st))
    kind = rng.randrange(14)
    if kind == 0:  # random bytes
        return bytes(rng.randrange(256) for _ in range(rng.randrange(1, 14)))
    if kind == 1:  # truncated valid message
        return valid[:rng.randrange(1, max(2, len(valid)))]
    if kind == 2:  # mediaId with a varint wire type (read as a string anyway)
        return b"\x08" + _varint(rng.randrange(0, 6)) + mid + b"\x10\x04"
    if kind == 3:  # status with a length-delimited wire type
        return b"\x0a" + _varint(len(mid)) + mid + b"\x12\x02\x04\x05"
    if kind == 4:  # unknown fields of every wire type, then the real fields
        return (b"\x48\x96\x01" + b"\x51" + bytes(8) + b"\x5a\x02hi" + b"\x65" + bytes(4) + valid)
    if kind == 5:  # a group (start/end of different field numbers), nested
        return b"\x6b\x73\x08\x01\x74\x6c" + valid
    if kind == 6:  # stray end-group / wire types 6 and 7
        return valid + bytes([rng.choice([0x4c, 0x4e, 0x4f, 0x0e])])
    if kind == 7:  # invalid UTF-8 in the media id and host
        bad = bytes([0xFF, 0xC3, 0x28, 0xED, 0xA0, 0x80, 0xF0, 0x9F, 0x98])
        return b"\x0a" + _varint(len(bad)) + bad + b"\x10\x02\x18\x07\x22\x03\xe2\x82\x28"
    if kind == 8:  # string length past the end (clamped by protobufjs's BufferReader)
        return b"\x0a" + _varint(len(mid) + rng.randrange(1, 50)) + mid
    if kind == 9:  # 10-byte varints (negative int32 status / progress), then more fields
        return b"\x0a" + _varint(len(mid)) + mid + b"\x10" + _varint(-rng.randrange(1, 3)) + b"\x18" + \
            _varint(-5) + b"\x22\x01h"
    if kind == 10:  # field number 0 and a tag with a 5-byte varint
        return b"\x00\x00" + b"\x80\x80\x80\x80\x00" + valid
    if kind == 11:  # two messages concatenated: the last value of each field wins
        return valid + _S.encode(("m1", 4))
    if kind == 12:  # uint32 overrun: 5 continuation bytes, then fewer than 5 left
        return b"\x10\xff\xff\xff\xff\xff\x01\x02"
    return b"\x1d\x01\x02\x03\x04" + valid  # progress field with a fixed32 wire type


def make_scenario(seed: int, n_events: int = 520, mode: str = "base") -> dict:
    """A seeded random config, media table, fault list and event stream."""
    rng = random.Random(seed * 7919 + MODES.index(mode))
    names = ["Cowboy Bebop", "Ü & ?", "", "50% *off* [x](y)", "new\nline", "🎬 Trigun"]
    card_ids = ["card1", "c/2", "", "ü", "a&b=c?d#e", "5f1a0b2c3d4e5f6a7b8c9d0e", "%20 +"]
    ids = ["m%d" % i for i in range(10)] + ["ü-7", "x y", "%s", ""]
    media = []
    for mid in ids:
        if rng.random() < 0.85:
            media.append({"id": mid, "name": rng.choice(names), "creator": rng.choice([0, 1, 1, 1, 2]),
                          "creatorId": rng.choice(card_ids), "metadataId": rng.choice(["1", "42", "", "ä"]),
                          "status": rng.randrange(0, 7)})
    statuses = ["queued", "downloading", "converting", "uploading", "deployed", "errored"]
    flow = {}
    keys = statuses + ["1", "10", "02"]  # integer-like keys come first in Object.keys
    rng.shuffle(keys)
    for k in keys:
        if rng.random() < 0.6:
            flow[k] = rng.choice(["L1", "L2", "", 0, 7, "list-ü", "a b"])
    config: dict = {
        "keys": {"trello": {"key": "TK", "token": rng.choice(["TT", "t/k=1"])}},
        "instance": {"flow_ids": flow},
    }
    if rng.random() < 0.85:
        config["keys"]["telegram"] = {"token": rng.choice(["123:TG", "9:a/b"])}
    if rng.random() < 0.8:
        config["keys"]["emby"] = {"token": rng.choice(["EMBYKEY", "", "k&y"])}
    if rng.random() < 0.85:
        config["instance"]["telegram"] = {"enabled": rng.choice([True, True, False, "yes", 0]),
                                          "channel": rng.choice(["-1001", 5, "@chan nel"])}
    if rng.random() < 0.85:
        config["instance"]["emby"] = {"enabled": rng.choice([True, True, False]),
                                      "host": rng.choice(["http://emby:8096", "https://e.example/x"])}
    faults: List[dict] = []
    if mode == "faults":  # both hooks on, so a Telegram failure visibly skips Emby (Q4)
        config["keys"]["telegram"] = {"token": "123:TG"}
        config["keys"]["emby"] = {"token": "EMBYKEY"}
        config["instance"]["telegram"] = {"enabled": True, "channel": "-1001"}
        config["instance"]["emby"] = {"enabled": True, "host": rng.choice(["http://emby:8096", "https://e.example/x"])}
        pool = [("POST", "https://api.trello.com"), ("PUT", "https://api.trello.com"),
                ("GET", "http://emby"), ("GET", "https://e.example"),
                ("*", "https://api.trello.com/1/cards/card1")]
        # always: a Telegram failure for the rows named "Cowboy Bebop" (Emby still runs for the
        # others, so a handler that runs Emby after a failed Telegram call diverges, Q4,
        # index.js:92-122) and a failing comment POST on card "card1" (its counter must not count,
        # index.js:53-57, and the progress handler still acks, Q7)
        rows = {m["id"]: m for m in media}
        for mid, over in (("m1", {"creator": 1, "creatorId": "card1"}), ("m2", {"name": "Cowboy Bebop"})):
            if mid not in rows:
                rows[mid] = {"id": mid, "name": "Trigun", "creator": 0, "creatorId": "", "metadataId": "1",
                             "status": 0}
                media.append(rows[mid])
            rows[mid].update(over)
        faults.append({"method": "GET", "prefix": TELEGRAM_FAULT_PREFIX, "status": rng.choice([None, 400, 500, 502]),
                       "message": rng.choice(["ECONNREFUSED", "socket hang up"]),
                       "body": '{"ok":false,"description":"Bad Request: chat not found é"}'})
        faults.append({"method": "POST", "prefix": "https://api.trello.com/1/cards/card1/actions/comments",
                       "status": None, "message": "ETIMEDOUT", "body": '"error"'})
        for method, prefix in rng.sample(pool, rng.randrange(0, 4)):
            f = {"method": method, "prefix": prefix, "status": rng.choice([None, 404, 500, 502, 204]),
                 "message": rng.choice(["ECONNREFUSED", "socket hang up"]),
                 "body": rng.choice(['"error"', '{"ok":false,"description":"Bad Request: chat not found é"}'])}
            faults.append(f)
    races: Dict[str, int] = {}
    if mode == "reread":
        # both hooks on; half the rows end DEPLOYED whatever the message said, the other half end
        # in another status even after a DEPLOYED message
        config["keys"]["telegram"] = {"token": "123:TG"}
        config["keys"]["emby"] = {"token": "EMBYKEY"}
        config["instance"]["telegram"] = {"enabled": True, "channel": "-1001"}
        config["instance"]["emby"] = {"enabled": True, "host": "http://emby:8096"}
        for m in media:
            if rng.random() < 0.7:
                races[m["id"]] = 4 if rng.random() < 0.5 else rng.choice([0, 1, 2, 3, 5])
    concurrent = None
    if mode == "concurrent":
        # few media, both hooks on: many deliveries of one media in flight together (Q9)
        config["keys"]["telegram"] = {"token": "123:TG"}
        config["keys"]["emby"] = {"token": "EMBYKEY"}
        config["instance"]["telegram"] = {"enabled": True, "channel": "-1001"}
        config["instance"]["emby"] = {"enabled": True, "host": "http://emby:8096"}
        for m in media:
            if m["id"] in ("m1", "m2", "m3"):
                m["creator"] = 1 if m["id"] != "m3" else 0
        concurrent = {"cap": CONCURRENT_CAP, "script": [rng.randrange(2 ** 31) for _ in range(4096)]}
    msg_ids = (["m1", "m2", "m3", "m1", "m2", "missing"] if mode == "concurrent"
               else ids + ["missing", "m1", "m1", "m2"])
    events = []
    for _ in range(n_events):
        r = rng.random()
        mid = rng.choice(msg_ids)
        st = rng.choice([4, 4, 4, 2]) if rng.random() < 0.3 else rng.choice([-1, 0, 1, 2, 3, 5, 6, 7, 2 ** 31 - 1])
        if r < 0.12:
            events.append(["status" if rng.random() < 0.5 else "progress", _malformed(rng, ids).hex()])
        elif r < 0.5:
            events.append(["status", _S.encode((mid, st)).hex()])
        else:
            prog = rng.choice([0, 5, 45, 100, -5, 150, 2 ** 31 - 1, -2 ** 31])
            host = rng.choice(["", "", "worker-1", "ünï", "a b&c", "%s %d"])
            events.append(["progress", _P.encode((mid, st, prog, host)).hex()])
    return {"seed": seed, "mode": mode, "config": config, "media": media, "events": events, "faults": faults,
            "positionalArgs": "drop" if mode == "drop" else "append", "notFound": NOT_FOUND, "logLevel": "info",
            "noTrello": mode == "no_trello", "races": races, "concurrent": concurrent}


def bench_scenario(n_events: int, seed: int = 0) -> dict:
    """The bench's own workload (``beholder_amd.bench.generator``: bench config, 10k-media table,
    90% progress / 10% status stream) as a scenario, so the gate also covers the exact events the
    throughput numbers are measured on (and the Node A/B, ``scripts/bench_reference_node.py``)."""
    from beholder_amd.bench.generator import Workload, bench_config
    w = Workload(n_media=10000, seed=seed)
    cfg = bench_config()
    framed = w.framed(n_events)
    topics = {1: "status", 2: "progress"}
    events, i = [], 0
    while i < len(framed):
        n = int.from_bytes(framed[i:i + 4], "little")
        events.append([topics[framed[i + 4]], framed[i + 5:i + 4 + n].hex()])
        i += 4 + n
    media = [{"id": m.id, "name": m.name, "creator": m.creator, "creatorId": m.creatorId,
              "metadataId": m.metadataId, "status": m.status} for m in w.media]
    return {"seed": seed, "mode": "bench", "config": {"keys": cfg["keys"], "instance": cfg["instance"]},
            "media": media, "events": events, "faults": [], "positionalArgs": "append", "notFound": NOT_FOUND,
            "logLevel": "info", "noTrello": False}


# ------------------------------------------------------------------------------------- runners ---
def run_node(sc: dict, timeout: float = 120.0) -> dict:
    """The reference's own index.js on Node, under the stand-ins (oracle.js)."""
    env = dict(os.environ, NODE_PATH=STUBS)
    env.pop("NO_TRELLO", None)
    if sc.get("noTrello"):
        env["NO_TRELLO"] = "1"
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(sc, f)
        path = f.name
    try:
        r = subprocess.run([NODE, ORACLE_JS, "--index", REFERENCE_INDEX, "--scenario", path], env=env,
                           capture_output=True, text=True, timeout=timeout)
    finally:
        os.unlink(path)
    if r.returncode != 0:
        raise RuntimeError(f"oracle.js failed ({r.returncode}): {r.stderr[-2000:]}")
    return json.loads(r.stdout)


def _counter_hashes(counter, label_names) -> list:
    """prom-client's hashMap keys ("k:v" joined by ",", keys sorted) -> value; zero entries dropped."""
    out = []
    for key, value in counter.values().items():
        if not value:
            continue
        h = ",".join(f"{n}:{v}" for n, v in sorted(zip(label_names, key)))
        out.append([h, value])
    return sorted(out)


class RacingStore(MemoryStore):
    """The ``reread`` scenarios' media table: after each ``update_status`` of a row in ``races``,
    another writer's UPDATE leaves ``races[id]`` in it before the handler's ``get_by_id``
    (the Node stand-in, stubs/triton-core/db.js, does the same)."""

    def __init__(self, medias, races: Dict[str, int]):
        super().__init__(medias)
        self.races = dict(races)

    def update_status_nowait(self, media_id: str, status: int) -> None:
        super().update_status_nowait(media_id, status)
        row = self._rows.get(media_id)
        if row is not None and media_id in self.races:
            self._rows[media_id] = row._replace(status=self.races[media_id])


class _Gates:
    """Mode ``concurrent``: the gate each in-flight event's store call / sink request waits on,
    opened by :func:`_run_concurrent` in the scenario's scripted order (oracle.js ``concurrent``)."""

    def __init__(self):
        self.current: Optional[int] = None  # the event whose code runs in this step
        self.waiting: Dict[int, tuple] = {}  # event index -> (kind, future)

    def wait(self, kind: str):
        i = self.current
        if i in self.waiting:
            raise RuntimeError(f"event {i} waits on two gates")
        f = asyncio.get_running_loop().create_future()
        self.waiting[i] = (kind, f)
        return f


def _gated_store(base, gates: _Gates):
    """``base`` whose UPDATE lands, and whose row is read, when the event's gate opens."""
    class Gated(base):
        async def update_status(self, media_id, status):
            await gates.wait("update")
            base.update_status_nowait(self, media_id, status)

        async def get_by_id(self, media_id):
            await gates.wait("get")
            return base.get_by_id_nowait(self, media_id)
    return Gated


class _GatedHttpClient(RecordingHttpClient):
    """Records a request when it is issued and answers it when the event's gate opens."""

    def __init__(self, gates: _Gates):
        super().__init__()
        self.gates = gates

    async def request(self, method, url, *, params=None, timeout=None):
        m = method.upper()
        full = self.record(m, url, params)
        await self.gates.wait("http")
        return self.answer(m, full)


def run_python(sc: dict, impl: str = "python", mutate=None, suspend: bool = False) -> dict:
    """This repo's handlers (``impl`` = python | native) over the same scenario.

    ``suspend``: the store and the sink client yield to the loop at every call before they answer
    (production's shape: its socket clients always wait), so the compiled handlers finish each
    event in their resume states. Mode ``concurrent`` always suspends (at its gates)."""
    import helpers
    from beholder_amd.handlers import native_handlers
    from beholder_amd.models.proto import DecodeError

    config = Config.from_dict(sc["config"], env={})
    conc = sc.get("concurrent")
    gates = _Gates() if conc else None
    if gates is not None:
        http = _GatedHttpClient(gates)
    else:
        http = helpers.SuspendingHttpClient() if suspend else RecordingHttpClient()
    for f in sc["faults"]:
        http.fail(f["method"], f["prefix"], status=f["status"], message=f["message"],
                  body=f["body"].encode())
    rows = [Media(id=m["id"], name=m["name"], creator=m["creator"], creatorId=m["creatorId"],
                  metadataId=m["metadataId"], status=m["status"]) for m in sc["media"]]
    base = RacingStore if sc.get("races") else MemoryStore
    if gates is not None:
        cls = _gated_store(base, gates)
    else:
        cls = helpers.suspending(base) if suspend else base
    store = cls(rows, sc["races"]) if base is RacingStore else cls(rows)
    rig = helpers.Rig(config=config, medias=rows, no_trello=bool(sc.get("noTrello")), http=http,
                      positional_args=sc["positionalArgs"], store=store)
    if mutate is not None:
        mutate(rig.h)
    target = rig.h if impl == "python" else native_handlers(rig.h)
    assert target is not None
    dec = {"status": rig.h.decode_status, "progress": rig.h.decode_progress}

    def decode_error(topic, body) -> bool:
        try:
            dec[topic](body)
            return False
        except DecodeError:
            return True

    events = []
    order = None

    async def go():
        for topic, hexbody in sc["events"]:
            body = bytes.fromhex(hexbody)
            n_http = len(http.calls)
            n_log = len(rig.stream.lines)
            d = rig.delivery(1 if topic == "status" else 2, body)
            threw = None
            try:
                await (target.on_status(d) if topic == "status" else target.on_progress(d))
            except Exception as e:  # noqa: BLE001 - Q1: status errors escape
                threw = str(e)
            rig.log.flush()
            logs = [[x["level"], x["msg"]] for x in map(json.loads, rig.stream.lines[n_log:])]
            events.append({"acks": 1 if d.state == "acked" else 0, "threw": threw,
                           "decodeError": decode_error(topic, body),
                           "requests": [list(c) for c in list(http.calls)[n_http:]], "logs": logs})

    if conc:
        events, order = asyncio.run(_run_concurrent(sc, rig, target, gates, decode_error))
    else:
        asyncio.run(go())
    counters = {
        "beholder_progress_updates_total": _counter_hashes(rig.progress, ["status"]),
        "beholder_trello_comments": _counter_hashes(rig.comments, []),
    }
    snap = rig.h.store.snapshot()
    out = {"events": events, "counters": counters, "media": {k: v.status for k, v in snap.items()}}
    if order is not None:
        out["order"] = order
    return out


# card ids the scenarios use that a socket cannot carry as the Node stand-in records them (a raw
# '#', '?', space or non-ASCII byte in the request path): replaced for the socket runs, on both sides
_WIRE_CARD_IDS = {"ü": "card-u", "a&b=c?d#e": "card-amp", "%20 +": "card-pct"}


def for_sockets(sc: dict) -> dict:
    """The scenario as :func:`run_service` replays it over real sockets (``sockets=True``), for
    Node and this service alike: card ids a request line cannot hold as written are replaced, and
    the sink faults that are transport errors (their text, e.g. ``ECONNREFUSED``, is the stand-in
    client's, not one a real socket would give) become ``503`` answers."""
    import copy
    sc = copy.deepcopy(sc)
    for m in sc["media"]:
        m["creatorId"] = _WIRE_CARD_IDS.get(m["creatorId"], m["creatorId"])
    for f in sc["faults"]:
        if f["status"] is None:
            f["status"] = 503
    sc["sockets"] = True
    return sc


class _SinkServer:
    """One sink origin (Trello, Telegram or Emby) on 127.0.0.1, HTTP/1.1 keep-alive: records each
    request as the reference's URL (its origin + the request target) and answers from the
    scenario's faults, first match first, as RecordingHttpClient does; else ``200 {}``."""

    def __init__(self, origin: str, faults: List[dict], calls: list, tls: bool = False):
        self.origin, self.faults, self.calls, self.tls = origin, faults, calls, tls
        self.port = 0
        self._server = None

    async def start(self) -> "_SinkServer":
        ctx = None
        if self.tls:  # the bench's own CA and certificate for 127.0.0.1
            from beholder_amd.bench.http_sink_server import server_ssl_context
            ctx = server_ssl_context()
        self._server = await asyncio.start_server(self._serve, "127.0.0.1", 0, ssl=ctx)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    @property
    def local(self) -> str:
        return f"{'https' if self.tls else 'http'}://127.0.0.1:{self.port}"

    async def stop(self) -> None:
        self._server.close()
        await self._server.wait_closed()

    def _answer(self, method: str, url: str):
        for f in self.faults:
            if (f["method"] == "*" or f["method"] == method) and url.startswith(f["prefix"]):
                return f["status"], f["body"].encode()
        return 200, b"{}"

    async def _serve(self, r, w) -> None:
        try:
            while True:
                line = await r.readline()
                if not line:
                    return
                method, target, _ = line.decode("latin-1").split(" ", 2)
                n = 0
                while True:
                    h = await r.readline()
                    if h in (b"\r\n", b"\n", b""):
                        break
                    k, _, v = h.decode("latin-1").partition(":")
                    if k.strip().lower() == "content-length":
                        n = int(v)
                if n:
                    await r.readexactly(n)
                url = self.origin + target
                self.calls.append([method, url])
                status, body = self._answer(method, url)
                if status == 204:
                    body = b""
                w.write(b"HTTP/1.1 %d X\r\nContent-Length: %d\r\n\r\n%s" % (status, len(body), body))
                await w.drain()
        except (ConnectionError, asyncio.IncompleteReadError):
            pass
        finally:
            w.close()


def _racing_pg(races: Dict[str, int]):
    """tests/pg_fake.py's server with the ``reread`` scenarios' other writer: after each UPDATE of
    a row in ``races``, a second UPDATE leaves ``races[id]`` in it (as RacingStore does)."""
    from pg_fake import FakePg

    class RacingPg(FakePg):
        def _run(self, sql, params):
            out = super()._run(sql, params)
            if races and sql.lstrip()[:6].upper() == "UPDATE" and params and str(params[-1]) in races:
                super()._run(sql, (races[str(params[-1])], params[-1]))
            return out
    return RacingPg(auth="trust")


def run_service(sc: dict, impl: str = "native", suspend: bool = False, sockets: bool = False,
                tls: bool = False) -> dict:
    """The same scenario through the whole consumer, as production runs it: each event is
    published to an in-process AMQP broker, delivered to :class:`AmqpSource` and
    handed to the service's dispatch (from the read callback when the service waits: the direct
    hand-over), handled, and acked over AMQP. One event at a time, as ``oracle.js`` delivers them;
    the next is published once this one is settled (acked, or left un-acked under Q1) and no
    handler is in flight.

    Recorded as :func:`run_python` records: ``acks`` as the broker counted them, ``threw`` from
    the service's ``unhandled error in <topic> handler: <message>`` line (Node's unhandled
    rejection, index.js:62; the line itself is not one of the reference's), the sink requests and
    the other log lines. Mode ``concurrent`` follows ``oracle.js``'s script step for step: a step
    publishes the next event or opens one waiting event's gate, then waits until that event is at
    its next gate or settled, and records what the step did (as :func:`_run_concurrent`).

    ``sockets``: the store and the sinks are production's clients over TCP too, not in-process
    fakes: ``PostgresStore`` against tests/pg_fake.py's server holding the scenario's table, and
    ``H1Client`` against one local HTTP server per sink origin, which records each request under
    the reference's origin (the scenario must come from :func:`for_sockets`). Every store call and
    sink request then waits on a socket, through the NetPoller, as in production. ``tls`` (with
    ``sockets``): the sink servers speak HTTPS, as Trello's and Telegram's do, and the H1 client's
    native TLS connections verify them against the bench's CA."""
    import copy
    import gc

    import helpers
    from beholder_amd import topics as T
    from beholder_amd.bench.harness import _settled
    from beholder_amd.models.proto import DecodeError
    from beholder_amd.service import Service
    from beholder_amd.transport.amqp import AmqpBroker, AmqpSource
    from beholder_amd.utils.log import Logger, MemoryStream

    conc = sc.get("concurrent")
    assert not (conc and sockets), "the concurrent mode's gates are in-process fakes"
    gates = _Gates() if conc else None
    data = copy.deepcopy(sc["config"])
    data["service"] = {"native_handlers": impl == "native", "gc_freeze": False,
                       "metrics": {"default_metrics": False},
                       "log": {"positional_args": sc["positionalArgs"]}}
    config = Config.from_dict(data, env={"NO_TRELLO": "1"} if sc.get("noTrello") else {})
    rows = [Media(id=m["id"], name=m["name"], creator=m["creator"], creatorId=m["creatorId"],
                  metadataId=m["metadataId"], status=m["status"]) for m in sc["media"]]
    if sockets:
        assert sc.get("sockets"), "a socket run replays a for_sockets() scenario"
        http = store = None  # made on the run's loop
    else:
        if gates is not None:
            http = _GatedHttpClient(gates)
        else:
            http = helpers.SuspendingHttpClient() if suspend else RecordingHttpClient()
        for f in sc["faults"]:
            http.fail(f["method"], f["prefix"], status=f["status"], message=f["message"], body=f["body"].encode())
        base = RacingStore if sc.get("races") else MemoryStore
        if gates is not None:
            cls = _gated_store(base, gates)
        else:
            cls = helpers.suspending(base) if suspend else base
        store = cls(rows, sc["races"]) if base is RacingStore else cls(rows)
    stream = MemoryStream()
    unhandled = ("unhandled error in %s handler: " % T.STATUS, "unhandled error in %s handler: " % T.PROGRESS)

    host_back: Dict[str, str] = {}

    async def go():
        nonlocal http, store, config
        loop = asyncio.get_running_loop()
        broker = await AmqpBroker().start()
        servers, pg = [], None
        try:
            if sockets:
                from beholder_amd.sinks import H1Client
                from beholder_amd.store.postgres import PostgresStore
                calls: list = []
                emby = data.get("instance", {}).get("emby", {}).get("host") or "http://emby:8096"
                ep = emby.split("/", 3)  # scheme:, '', host[:port], base path
                origins = {"trello": "https://api.trello.com", "telegram": "https://api.telegram.org",
                           "emby": "/".join(ep[:3])}
                for name, origin in origins.items():
                    servers.append(await _SinkServer(origin, sc["faults"], calls, tls=tls).start())
                local = {n: srv.local for n, srv in zip(origins, servers)}
                d2 = copy.deepcopy(data)
                d2["service"]["endpoints"] = {"trello": local["trello"], "telegram": local["telegram"]}
                if "emby" in d2.get("instance", {}):
                    d2["instance"]["emby"]["host"] = local["emby"] + ("/" + ep[3] if len(ep) > 3 else "")
                    # the Emby log line names the configured host: ours, read back as the scenario's
                    host_back[d2["instance"]["emby"]["host"]] = emby
                config = Config.from_dict(d2, env=config.env)
                pg = await _racing_pg(sc.get("races") or {}).start()
                setup = PostgresStore(pg.dsn, create_schema=True)
                await setup.connect()
                for m in rows:
                    await setup.upsert(m)
                await setup.close()
                store = PostgresStore(pg.dsn)
                if tls:
                    from beholder_amd.bench.http_sink_server import TLS_CERT
                    http = H1Client(timeout_s=10, ssl_cafile=TLS_CERT)
                else:
                    http = H1Client(timeout_s=10)
                http.calls = calls  # what the servers recorded, read as RecordingHttpClient's
            # the broker's window holds every event: the deliveries Q1 leaves un-acked keep their
            # slots (as on a real broker, where 100 of them stall a consumer for good), and the Node
            # stand-in has no window to fill
            src = AmqpSource(broker.url, prefetch=max(100, len(sc["events"]) + 1))
            svc = Service(config, source=src, store=store, http=http, serve_metrics=False,
                          logger=Logger(stream=stream, positional_args=sc["positionalArgs"]))
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            h = svc.handlers
            dec = {"status": h.decode_status, "progress": h.decode_progress}
            settler = src.settler
            queues = [broker.queues[q] for q in (T.STATUS, T.PROGRESS) if q in broker.queues]

            def broker_acked() -> int:
                return sum(q.acked for q in queues)
            acks_arrive = True  # until one event's acks failed to reach the broker in a second

            def logs_since(n_log: int):
                """The log lines written since ``n_log``: Node's rejection (the service's line for
                an unhandled handler error) apart from the reference's own lines."""
                svc.log.flush()
                threw, logs = None, []
                for x in map(json.loads, stream.lines[n_log:]):
                    msg = x["msg"]
                    if x["level"] == 50 and msg.startswith(unhandled):
                        threw = msg[len(unhandled[0 if msg.startswith(unhandled[0]) else 1]):]
                        continue
                    for ours, theirs in host_back.items():
                        msg = msg.replace(ours, theirs)
                    logs.append([x["level"], msg])
                return threw, logs

            def decode_error(topic: str, body: bytes) -> bool:
                try:
                    dec[topic](body)
                    return False
                except DecodeError:
                    return True

            async def until(cond, what: str) -> None:
                t_end = loop.time() + 10.0
                collected = False
                while not cond():
                    if task.done():
                        task.result()  # the service failed: raise it here
                    if loop.time() > t_end:
                        raise TimeoutError(f"{what}: not within 10 s")
                    if not collected and loop.time() > t_end - 9.8:
                        gc.collect()  # an un-acked delivery is counted once it is freed (Q1)
                        collected = True
                    await asyncio.sleep(0.0002)

            async def acks_flushed() -> None:
                """The acks the handlers settled, as the broker counts them (flushed over AMQP)."""
                nonlocal acks_arrive
                t_ack = loop.time() + (1.0 if acks_arrive else 0.005)
                while broker_acked() < settler.acked and loop.time() < t_ack:
                    await asyncio.sleep(0.0002)
                acks_arrive = broker_acked() >= settler.acked

            order = None
            events = []
            if conc:  # oracle.js concurrent(), step for step, with each delivery over AMQP
                cap, script = conc["cap"], conc["script"]
                topics = [t for t, _ in sc["events"]]
                bodies = [bytes.fromhex(hx) for _, hx in sc["events"]]
                n = len(bodies)
                events = [{"acks": 0, "threw": None, "decodeError": decode_error(t, b), "requests": [], "logs": []}
                          for t, b in zip(topics, bodies)]
                settled = [False] * n
                order = []
                nxt = step = 0
                while True:
                    ready = sorted(gates.waiting)
                    r = script[step % len(script)]
                    step += 1
                    active = nxt - sum(settled[:nxt])
                    if nxt < n and (not ready or (active < cap and r % 2 == 0)):
                        i, action, kind = nxt, "deliver", None
                        nxt += 1
                    elif ready:
                        i = ready[(r >> 1) % len(ready)]
                        action = "resolve"
                    else:
                        if active:
                            raise RuntimeError(f"{active} deliveries in flight, none at a gate")
                        break
                    gates.current = i
                    svc.log.flush()
                    n_http, n_log = len(http.calls), len(stream.lines)
                    s0, a0 = _settled(settler), broker_acked()
                    if action == "deliver":
                        broker.publish(T.STATUS if topics[i] == "status" else T.PROGRESS, bodies[i])
                    else:
                        kind, fut = gates.waiting.pop(i)
                        fut.set_result(None)
                    # the event reaches its next gate, or ends (settled); then whatever else that
                    # made runnable runs (oracle.js: one setImmediate)
                    await until(lambda: i in gates.waiting or _settled(settler) > s0, f"step {step} event {i}")
                    for _ in range(10000):
                        await asyncio.sleep(0)
                        if not loop._ready:  # noqa: SLF001 - the loop's runnable queue
                            break
                    await acks_flushed()
                    if _settled(settler) > s0:
                        settled[i] = True
                    threw, logs = logs_since(n_log)
                    reqs = [list(c) for c in list(http.calls)[n_http:]]
                    ev = events[i]
                    ev["logs"] += logs
                    ev["requests"] += reqs
                    if threw is not None:
                        ev["threw"] = threw
                    got = broker_acked() - a0
                    ev["acks"] += got
                    order.append([action, i, kind, len(logs), len(reqs), int(got > 0), settled[i]])
            for topic, hexbody in ([] if conc else sc["events"]):
                body = bytes.fromhex(hexbody)
                svc.log.flush()
                n_http, n_log = len(http.calls), len(stream.lines)
                settled0, acked0 = _settled(settler), broker_acked()
                broker.publish(T.STATUS if topic == "status" else T.PROGRESS, body)
                await until(lambda: _settled(settler) > settled0 and not len(svc._inflight),
                            f"event {len(events)} settled")
                await acks_flushed()
                threw, logs = logs_since(n_log)
                events.append({"acks": broker_acked() - acked0, "threw": threw, "decodeError": decode_error(topic, body),
                               "requests": [list(c) for c in list(http.calls)[n_http:]], "logs": logs})
            svc.request_stop()
            await task
            counters = {
                "beholder_progress_updates_total": _counter_hashes(svc.progress_updates_total, ["status"]),
                "beholder_trello_comments": _counter_hashes(svc.trello_comments_total, []),
            }
            path = {"direct_batches": src.direct_batches, "idle_wakeups": src.idle_wakeups,
                    "netpoller": getattr(loop, "_beholder_netpoller", None) is not None}
            stats = getattr(svc.handler_impl, "stats", None)
            if callable(stats):  # the compiled handlers: how many events left C to wait on I/O
                path["suspended"] = stats().get("suspended")
            await svc.close()
            if sockets:  # the table as the server holds it (the service closed its own store)
                check = PostgresStore(pg.dsn)
                await check.connect()
                media = {m.id: (await check.get_by_id(m.id)).status for m in rows}
                await check.close()
            else:
                media = {k: v.status for k, v in store.snapshot().items()}
            return events, counters, path, media, order
        finally:
            for srv in servers:
                await srv.stop()
            if pg is not None:
                await pg.stop()
            await broker.stop()

    events, counters, path, media, order = asyncio.run(go())
    # ``path``: how the deliveries reached the handlers (AmqpSource.direct hand-overs, and the
    # batches the service's task woke up for); diff() does not compare it
    out = {"events": events, "counters": counters, "media": media, "path": path}
    if order is not None:
        out["order"] = order
    return out


async def _run_concurrent(sc: dict, rig, target, gates: _Gates, decode_error):
    """oracle.js ``concurrent()``, step for step: deliver the next event or open one waiting
    event's gate (the scenario's script decides), then run the loop until nothing is runnable.
    Deliveries go through the service's ordering layer when ``service.ordering`` is ``per_media``
    (parallel/ordering.py, as service.py wires it); the default, ``none``, is the reference's."""
    from beholder_amd.parallel.ordering import KeyedSerializer
    loop = asyncio.get_running_loop()
    cap, script = sc["concurrent"]["cap"], sc["concurrent"]["script"]
    n = len(sc["events"])
    bodies = [bytes.fromhex(h) for _, h in sc["events"]]
    topics = [t for t, _ in sc["events"]]
    events = [{"acks": 0, "threw": None, "decodeError": decode_error(t, b), "requests": [], "logs": []}
              for t, b in zip(topics, bodies)]
    deliveries = [rig.delivery(1 if t == "status" else 2, b) for t, b in zip(topics, bodies)]
    tasks: Dict[int, asyncio.Task] = {}
    settled = [False] * n
    http = rig.http

    def start(i: int, on_finish=None) -> bool:
        d = deliveries[i]
        coro = target.on_status(d) if topics[i] == "status" else target.on_progress(d)

        async def run():
            try:
                await coro
            except Exception as e:  # noqa: BLE001 - Q1: status errors escape
                events[i]["threw"] = str(e)
            finally:
                settled[i] = True
                if on_finish is not None:
                    on_finish()
        tasks[i] = loop.create_task(run())
        return False

    def media_key(i: int):
        h = rig.h
        return (h.decode_status if topics[i] == "status" else h.decode_progress)(bodies[i]).mediaId

    ordering = rig.config.data.get("service", {}).get("ordering", "none")
    submit = KeyedSerializer(start, media_key).submit if ordering == "per_media" else start

    order = []
    nxt = 0
    step = 0
    while True:
        ready = sorted(gates.waiting)
        r = script[step % len(script)]
        step += 1
        active = nxt - sum(settled[:nxt])
        if nxt < n and (not ready or (active < cap and r % 2 == 0)):
            i, action, kind = nxt, "deliver", None
            nxt += 1
        elif ready:
            i = ready[(r >> 1) % len(ready)]
            action = "resolve"
        else:
            if active:
                raise RuntimeError(f"{active} deliveries in flight, none at a gate")
            break
        gates.current = i
        n_http, n_log = len(http.calls), len(rig.stream.lines)
        acked = deliveries[i].state == "acked"
        if action == "deliver":
            submit(i)
        else:
            kind, fut = gates.waiting.pop(i)
            fut.set_result(None)
        for _ in range(10000):  # until nothing is runnable (oracle.js: one setImmediate)
            await asyncio.sleep(0)
            if not loop._ready:  # noqa: SLF001 - the loop's runnable queue
                break
        rig.log.flush()
        ev = events[i]
        logs = [[x["level"], x["msg"]] for x in map(json.loads, rig.stream.lines[n_log:])]
        reqs = [list(c) for c in list(http.calls)[n_http:]]
        ev["logs"] += logs
        ev["requests"] += reqs
        now_acked = deliveries[i].state == "acked"
        ev["acks"] = 1 if now_acked else 0
        order.append([action, i, kind, len(logs), len(reqs), int(now_acked and not acked), settled[i]])
    for t in tasks.values():
        await t
    return events, order


def diff(ref: dict, got: dict, limit: int = 8) -> List[str]:
    """Human-readable differences (empty = identical)."""
    out: List[str] = []
    if len(ref["events"]) != len(got["events"]):
        return [f"event count {len(ref['events'])} != {len(got['events'])}"]
    for i, (a, b) in enumerate(zip(ref["events"], got["events"])):
        for k in ("acks", "threw", "decodeError", "requests", "logs"):
            if a[k] != b[k]:
                out.append(f"event {i} {k}: reference={a[k]!r} ours={b[k]!r}")
                if len(out) >= limit:
                    return out
    if "order" in ref or "order" in got:
        for j, (a, b) in enumerate(zip(ref.get("order") or [], got.get("order") or [])):
            if a != b:
                out.append(f"step {j}: reference={a!r} ours={b!r}")
                break
        else:
            if len(ref.get("order") or []) != len(got.get("order") or []):
                out.append(f"steps {len(ref.get('order') or [])} != {len(got.get('order') or [])}")
    ref_counters = {k: [e for e in v if e[1]] for k, v in ref["counters"].items()}
    if ref_counters != got["counters"]:
        out.append(f"counters: reference={ref_counters} ours={got['counters']}")
    if ref["media"] != got["media"]:
        out.append(f"media: reference={ref['media']} ours={got['media']}")
    return out


def check(seed: int, mode: str, n_events: int = 520, impls=("python", "native"),
          suspend: bool = False) -> Dict[str, List[str]]:
    sc = make_scenario(seed, n_events, mode)
    ref = run_node(sc)
    return {impl: diff(ref, run_python(sc, impl, suspend=suspend)) for impl in impls}


def coverage(ref: dict) -> dict:
    """Which reference branches a run reached (from its own trace)."""
    msgs = [m for e in ref["events"] for _, m in e["logs"]]
    reqs = [r for e in ref["events"] for r in e["requests"]]
    return {
        "threw": sum(1 for e in ref["events"] if e["threw"] is not None),
        "decode_errors": sum(1 for e in ref["events"] if e["decodeError"]),
        "unacked": sum(1 for e in ref["events"] if e["acks"] == 0),
        "card_moves": sum(1 for m, _ in reqs if m == "PUT"),
        "comments": sum(1 for m, _ in reqs if m == "POST"),
        "telegram": sum(1 for _, u in reqs if "api.telegram.org" in u),
        "emby": sum(1 for _, u in reqs if "/emby/library/refresh" in u),
        "missing_list_warns": sum(1 for m in msgs if m.startswith("unable to find list")),
        "hook_warns": sum(1 for m in msgs if m.startswith("failed to run deployed hooks")),
        "progress_warns": sum(1 for m in msgs if m.startswith("failed to update media progress")),
    }


def reread_coverage(sc: dict, ref: dict) -> dict:
    """For a ``reread`` scenario: status events whose re-read row status differs from the message's
    in the direction that decides the hooks (index.js:94), as the reference ran them."""
    races = sc.get("races") or {}
    known = {m["id"] for m in sc["media"]}
    hooks_without_deployed_msg = hooks_skipped_on_deployed_msg = 0
    for (topic, hexbody), ev in zip(sc["events"], ref["events"]):
        if topic != "status" or ev["decodeError"]:
            continue
        try:
            mid, st = _S.decode(bytes.fromhex(hexbody))[:2]
        except Exception:  # noqa: BLE001
            continue
        if mid not in known or mid not in races:
            continue
        hooked = any("api.telegram.org" in u for _, u in ev["requests"])
        if races[mid] == 4 and st != 4 and hooked:
            hooks_without_deployed_msg += 1
        if races[mid] != 4 and st == 4 and not hooked:
            hooks_skipped_on_deployed_msg += 1
    return {"hooks_without_deployed_msg": hooks_without_deployed_msg,
            "hooks_skipped_on_deployed_msg": hooks_skipped_on_deployed_msg}


def _media_ids(sc: dict) -> List[Optional[str]]:
    out: List[Optional[str]] = []
    for topic, hexbody in sc["events"]:
        try:
            out.append((_S if topic == "status" else _P).decode(bytes.fromhex(hexbody))[0])
        except Exception:  # noqa: BLE001 - undecodable: no media
            out.append(None)
    return out


def concurrent_coverage(sc: dict, ref: dict) -> dict:
    """For a ``concurrent`` scenario, as the reference ran it: steps with two deliveries of one
    media in flight, status events whose hooks decision (index.js:94, the re-read row) disagrees
    with the message's status because another delivery's UPDATE landed in between, and steps
    that resumed a delivery other than the oldest one waiting."""
    ids = _media_ids(sc)
    known = {m["id"] for m in sc["media"]}
    inflight: set = set()
    overlap = out_of_order = 0
    waiting: set = set()
    for action, i, kind, _logs, _reqs, _acks, settled in ref["order"]:
        if action == "deliver":
            inflight.add(i)
        else:
            if waiting and i != min(waiting):
                out_of_order += 1
            waiting.discard(i)
        if settled:
            inflight.discard(i)
        else:
            waiting.add(i)
        live = [ids[j] for j in inflight if ids[j] is not None]
        overlap += len(live) != len(set(live))
    flipped = 0
    for (topic, hexbody), ev, mid in zip(sc["events"], ref["events"], ids):
        if topic != "status" or ev["decodeError"] or mid not in known or ev["threw"] is not None:
            continue
        st = _S.decode(bytes.fromhex(hexbody))[1]
        hooked = any("api.telegram.org" in u for _, u in ev["requests"])
        flipped += hooked != (st == 4)
    return {"same_media_overlap_steps": overlap, "hooks_flipped_by_interleaving": flipped,
            "resumed_out_of_arrival_order": out_of_order}


def main(argv: Optional[List[str]] = None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description="reference-executed parity gate")
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--events", type=int, default=520)
    ap.add_argument("--modes", default=",".join(MODES))
    ap.add_argument("--impls", default="python,native")
    ap.add_argument("--suspend", action="store_true",
                    help="store and sink client yield at every call (the compiled handlers' resume states)")
    ap.add_argument("--service", action="store_true",
                    help="through the whole consumer: AMQP broker, AmqpSource, Service dispatch, acks "
                         "(run_service)")
    ap.add_argument("--sockets", action="store_true",
                    help="with --service: Postgres and the sinks over TCP too (for_sockets scenarios)")
    ap.add_argument("--tls", action="store_true", help="with --sockets: the sinks over HTTPS")
    a = ap.parse_args(argv)
    bad = 0
    for seed in range(a.seeds):
        for mode in a.modes.split(","):
            sc = make_scenario(seed, a.events, mode)
            sockets = a.sockets and mode != "concurrent"  # the concurrent gates are in-process
            if a.service and sockets:
                sc = for_sockets(sc)
            ref = run_node(sc)
            for impl in a.impls.split(","):
                if a.service:
                    d = diff(ref, run_service(sc, impl, suspend=a.suspend, sockets=sockets, tls=a.tls))
                else:
                    d = diff(ref, run_python(sc, impl, suspend=a.suspend))
                bad += bool(d)
                print(f"seed {seed} {mode:10s} {impl:6s} {'OK' if not d else 'DIFF'} {coverage(ref) if not d else ''}")
                for line in d:
                    print("   ", line)
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
