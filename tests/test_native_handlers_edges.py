"""The compiled handlers (ops/csrc/py_handlers.cpp) with dependencies off their fast paths.

tests/test_handlers.py and test_native_handlers.py drive the stock clients, stores, counters and
deliveries, which the compiled handlers recognise and call in C. Everything else must behave as
the Python handlers (handlers.py) do through the generic Python protocol: a delivery that is not a
native Delivery, counters and per-sink stats in Python, Telegram / Emby / Trello clients with a
rate limit or retry policy (their own methods), a flow-list map that is not a dict, list ids of
every JS truthiness, media rows of another tuple type, a store that returns something not
awaitable. Each case runs the same events through both implementations and compares the observable
trace (native_coverage's gap list). The last cases pin the HandlerCall's
coroutine protocol edges (iteration, throw / close on odd delegates, misuse).
"""
from __future__ import annotations

import asyncio
import collections
import types

import pytest

import helpers
from beholder_amd.handlers import native_handlers
from beholder_amd.sinks.ratelimit import RetryPolicy, TokenBucket
from beholder_amd.store import MemoryStore
from helpers import Rig, api_media, cfg, progress_msg, status_msg, trello_media

DEPLOYED_ROWS = [trello_media("m1", "UPLOADING", card="C1"), api_media("m2", "QUEUED"),
                 trello_media("m3", "DEPLOYED", card="C3", name="Ü & ?")]
EVENTS = [("status", "m1", "DEPLOYED"), ("progress", "m1", "CONVERTING", 40, "w1"), ("status", "m2", "DEPLOYED"),
          ("progress", "m2", "QUEUED", 5, ""), ("status", "missing", "QUEUED"), ("progress", "missing", "QUEUED", 1, ""),
          ("status", "m3", 7), ("status", "m1", "QUEUED"), ("progress", "m3", "DEPLOYED", 100, "h"),
          ("status", "garbage", b"\xff"), ("progress", "garbage", b"\x0a\x05ab")]


def _body(ev):
    if ev[1] == "garbage":
        return ev[2]
    if ev[0] == "status":
        return status_msg(ev[1], ev[2])
    return progress_msg(*ev[1:])


class PyDelivery:
    """An envelope that is not a native Delivery: ``rmsg.message.content`` and ``rmsg.ack()``
    through the Python protocol (index.js:63,129; 71,124,151,154)."""

    def __init__(self, body):
        self.message = types.SimpleNamespace(content=body)
        self.acks = 0

    def ack(self):
        self.acks += 1

    @property
    def state(self):
        return "acked" if self.acks else "pending"


class PyStats:
    """Per-sink stats in Python (``record(status, seconds)``): the sink clients' observer protocol."""

    def __init__(self, log, sink):
        self.log, self.sink = log, sink

    def record(self, status, seconds):
        assert seconds >= 0
        self.log.append((self.sink, status))


def trace(impl, rows=DEPLOYED_ROWS, events=EVENTS, config=None, setup=None, store=None, py_delivery=False,
          fail=()):
    """Both implementations over the same rig changes: deliveries, logs, requests, counters, rows."""
    helpers.HANDLER_IMPL = "python"
    r = Rig(config=config or cfg(), medias=list(rows), store=store)
    for method, prefix, status in fail:
        r.http.fail(method, prefix, status=status)
    extra: dict = {}
    if setup is not None:
        setup(r, extra)
    target = native_handlers(r.h) if impl == "native" else r.h
    assert target is not None
    ds = [(ev[0], PyDelivery(_body(ev)) if py_delivery else r.delivery(1 if ev[0] == "status" else 2, _body(ev)))
          for ev in events]

    async def go():
        out = []
        for kind, d in ds:
            try:
                await (target.on_status(d) if kind == "status" else target.on_progress(d))
                out.append(None)
            except Exception as e:  # noqa: BLE001 - Q1: status errors escape
                out.append(f"{type(e).__name__}: {e}")
        return out
    errors = asyncio.run(go())
    r.log.flush()
    return {"deliveries": [(d.state, e) for (_, d), e in zip(ds, errors)],
            "logs": [(x["level"], x["msg"]) for x in r.stream.records()], "http": list(r.http.calls),
            "progress": sorted(r.progress.values().items()), "comments": r.comments.get(),
            "store": sorted((k, tuple(v)) for k, v in r.h.store.snapshot().items()),
            **{k: list(v) for k, v in extra.items()}}


def same(**kw):
    got, want = trace("native", **kw), trace("python", **kw)
    assert got == want
    return got


@pytest.mark.parametrize("io", ["sync", "suspend"])
def test_envelope_that_is_not_a_native_delivery(io, monkeypatch):
    """content and ack() through the Python protocol, not the Delivery fast path."""
    monkeypatch.setattr(helpers, "SUSPEND", io == "suspend")
    got = same(py_delivery=True)
    assert [s for s, _ in got["deliveries"]].count("acked") >= 8


def test_counters_and_sink_stats_in_python():
    """A comment counter, progress counter children and per-sink stats that are plain Python
    objects (the compiled handlers otherwise bump native counters and stats in C)."""
    def setup(r, extra):
        extra["stats"] = log = []
        extra["incs"] = incs = []
        for sink in ("trello", "telegram", "emby"):
            getattr(r.h, sink).stats = PyStats(log, sink)
        r.h._comment_inc = lambda: incs.append("comment")

        class Child:
            def __init__(self, label):
                self.label = label

            def inc(self):
                incs.append(self.label)

        class PyCounter:
            def child_for(self, label):
                return Child(label)
        r.h.progress_counter = PyCounter()
    got = same(setup=setup, fail=[("GET", "http://emby", 500)])
    assert ("telegram", 200) in got["stats"] and ("emby", 500) in got["stats"] and ("trello", 200) in got["stats"]
    assert "comment" in got["incs"] and "converting" in got["incs"]


@pytest.mark.parametrize("fault", [None, 500, "raise"])
def test_clients_with_a_rate_limit_or_retry_use_their_own_methods(fault):
    """Telegram / Emby / Trello clients with a limiter or a retry policy: the handlers call the
    client's own send_message / refresh_library / make_request (sinks/ratelimit.py guarded)."""
    def setup(r, extra):
        r.h.telegram.limiter = TokenBucket(1000, 1.0)
        r.h.emby.retry = RetryPolicy(0)
        r.h.trello.limiter = TokenBucket(1000, 1.0)
    fail = [] if fault is None else [("GET", "https://api.telegram.org", None if fault == "raise" else fault)]
    got = same(setup=setup, fail=fail)
    urls = [u for _, u in got["http"]]
    assert any("sendMessage" in u for u in urls)
    assert any("/emby/library/refresh" in u for u in urls) == (fault is None)


@pytest.mark.parametrize("value", [0.0, 1.5, float("nan"), {}, [], {"a": 1}, "", "L9", 0, 7, None, True, False])
def test_list_ids_of_every_js_truthiness(value):
    """index.js:81 `if (listPointer)`: floats (NaN and 0.0 falsy), objects and arrays (truthy, even
    empty) as flow-list ids; a truthy one moves the card with it (String() of the id)."""
    c = cfg()
    c.data["instance"]["flow_ids"] = {"deployed": value, "queued": value}
    same(config=c, events=[("status", "m1", "DEPLOYED"), ("status", "m1", "QUEUED")])


def test_flow_list_map_that_is_not_a_dict():
    """`lists[statusText.toLowerCase()]` on a mapping that is not a dict (handlers._get)."""
    def setup(r, extra):
        r.h.lists = types.MappingProxyType({"deployed": "L-dep", "converting": ""})
    got = same(setup=setup)
    assert any("idList=L-dep" in u for _, u in got["http"])


def test_rows_of_another_tuple_type():
    """A media table whose rows are not store.base.Media: fields read by attribute, the status
    update made with the row's own ``_replace`` (store/memory.py update_status_nowait)."""
    Row = collections.namedtuple("Row", ["id", "name", "creator", "creatorId", "metadataId", "status"])
    rows = [Row(m.id, m.name, m.creator, m.creatorId, m.metadataId, m.status) for m in DEPLOYED_ROWS]
    got = same(rows=rows)
    assert {type(v).__name__ for _, v in [(k, v) for k, v in got["store"]]} == {"tuple"}
    assert all(len(v) == 6 for _, v in got["store"])


class NotAwaitableStore(MemoryStore):
    """get_by_id returns a plain value: ``await`` on it raises TypeError in both implementations."""

    def get_by_id(self, media_id):  # noqa: D102 - not a coroutine on purpose
        return 42

    async def update_status(self, media_id, status):
        MemoryStore.update_status_nowait(self, media_id, status)


def test_store_returning_something_not_awaitable():
    """Q1 for the status handler (the TypeError escapes, un-acked), Q7 for the progress one."""
    got = same(store=NotAwaitableStore(list(DEPLOYED_ROWS)))
    assert any(e and "can't be used in 'await' expression" in e for _, e in got["deliveries"])
    assert any(m.startswith("failed to update media progress object int") for _, m in got["logs"])


# ------------------------------------------------------------------- call protocol edges ----
class BareIter:
    """An awaitable whose iterator has neither throw() nor close() (a minimal __await__)."""

    def __init__(self, value):
        self.value = value

    def __await__(self):
        return iter(())


class BareStore(MemoryStore):
    def get_by_id(self, media_id):
        return BareWait(MemoryStore.get_by_id_nowait(self, media_id))

    async def update_status(self, media_id, status):
        MemoryStore.update_status_nowait(self, media_id, status)


class BareWait:
    """Suspends once with a bare yield through an iterator that has no throw() / close()."""

    def __init__(self, value):
        self.value = value

    def __await__(self):
        return _Once(self.value)


class _Once:
    def __init__(self, value):
        self.value, self.n = value, 0

    def __iter__(self):
        return self

    def __next__(self):
        self.n += 1
        if self.n == 1:
            return None
        raise StopIteration(self.value)


def _native_rig(store=None):
    helpers.HANDLER_IMPL = "python"
    r = Rig(medias=[trello_media("m1")], store=store)
    return r, native_handlers(r.h)


def test_handler_call_iterates_like_a_coroutine():
    """next() / iteration drive a HandlerCall as they drive the coroutine of the Python method."""
    r, nh = _native_rig(helpers.SuspendingStore([trello_media("m1")]))
    d = r.delivery(2, progress_msg("m1", "QUEUED", 5))
    call = nh.on_progress(d)
    assert next(call) is None  # suspended in the store read
    with pytest.raises(StopIteration):
        next(call)
    assert d.acked
    d = r.delivery(2, progress_msg("m1", "QUEUED", 5))
    assert list(nh.on_progress(d).__await__()) == [None] and d.acked  # iteration to the end


def test_handler_call_misuse_raises():
    r, nh = _native_rig()
    call = nh.on_progress(r.delivery(2, progress_msg("m1", "QUEUED", 5)))
    with pytest.raises(TypeError, match="non-None"):
        call.send(1)
    with pytest.raises(TypeError, match="1 to 3 arguments"):
        call.throw()
    with pytest.raises(StopIteration):
        call.send(None)  # completes synchronously (the in-memory store)
    with pytest.raises(RuntimeError, match="reuse"):
        call.send(None)


def test_throw_into_a_fresh_call_ends_it():
    """throw() before the first step raises at the start, like a fresh coroutine: nothing runs."""
    r, nh = _native_rig()
    d = r.delivery(2, progress_msg("m1", "QUEUED", 5))
    call = nh.on_progress(d)
    with pytest.raises(KeyError):
        call.throw(KeyError("x"))
    assert call.done and d.state == "pending" and r.http.count == 0
    call = nh.on_status(r.delivery(1, status_msg("m1", "QUEUED")))
    with pytest.raises(ValueError):
        call.throw(ValueError, "v")  # the (type, value) form


def test_throw_and_close_on_a_delegate_without_them():
    """A delegate iterator with no throw(): the exception is raised at the await itself (Q7: the
    progress handler warns and acks); with no close(), close() just abandons the call."""
    r, nh = _native_rig(BareStore([trello_media("m1")]))
    d = r.delivery(2, progress_msg("m1", "QUEUED", 5))
    call = nh.on_progress(d)
    assert call.send(None) is None and call.state == 1
    with pytest.raises(StopIteration):
        call.throw(ValueError("boom"))
    assert d.acked and r.msgs(40)[-1] == "failed to update media progress boom"
    d = r.delivery(2, progress_msg("m1", "QUEUED", 5))
    call = nh.on_progress(d)
    call.send(None)
    with pytest.raises(StopIteration):
        call.throw(ValueError)  # an exception class
    d = r.delivery(2, progress_msg("m1", "QUEUED", 5))
    call = nh.on_progress(d)
    call.send(None)
    assert call.close() is None and call.done and d.state == "pending"
    # the delegate's value comes back through StopIteration: the comment is posted
    d = r.delivery(2, progress_msg("m1", "QUEUED", 5))
    asyncio.run(helpers._await(nh.on_progress(d)))
    assert d.acked and r.http.urls("POST")


def test_a_hooks_plan_that_is_not_a_six_tuple_is_caught():
    """The DEPLOYED-hooks config plan comes from handlers._hooks_plan(); a wrong shape raises
    inside the hooks' try (index.js:92-122): warned, acked."""
    helpers.HANDLER_IMPL = "python"
    r = Rig(medias=[api_media("m2")])
    r.h._hooks_plan = lambda: (True, "-1001")
    nh = native_handlers(r.h)
    d = r.delivery(1, status_msg("m2", "DEPLOYED"))
    asyncio.run(helpers._await(nh.on_status(d)))
    assert d.acked and r.msgs(40) == ["failed to run deployed hooks: _hooks_plan() must return a 6-tuple"]


@pytest.mark.parametrize("client,attr", [("trello", "stats"), ("telegram", "base_url"), ("emby", "stats")])
def test_a_sink_client_missing_an_attribute(client, attr):
    """A stock client instance without one of its attributes: the move (Trello, outside the try)
    escapes as in the Python client (Q1); a hook's error is warned and the event acked (Q4)."""
    out = {}
    for impl in ("python", "native"):
        helpers.HANDLER_IMPL = "python"
        r = Rig(medias=[trello_media("m1", "QUEUED")])
        delattr(getattr(r.h, client), attr)
        target = native_handlers(r.h) if impl == "native" else r.h
        d = r.delivery(1, status_msg("m1", "DEPLOYED"))
        try:
            asyncio.run(helpers._await(target.on_status(d)))
            exc = None
        except AttributeError as e:
            exc = type(e).__name__
        out[impl] = (d.state, exc, [m for lvl, m in [(x["level"], x["msg"]) for x in r.stream.records()] if lvl == 40]
                     if r.log.flush() is None else None)
    assert out["native"][:2] == out["python"][:2]
    if client == "trello":
        assert out["native"][:2] == ("pending", "AttributeError")
    else:
        assert out["native"][0] == "acked" and len(out["native"][2]) == 1
