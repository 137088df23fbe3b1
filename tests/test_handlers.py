"""Branch-by-branch parity of the status / progress handlers with index.js:50-155.

Each test names the reference lines / quirk it pins.
"""
import asyncio

import pytest

import helpers
from beholder_amd.handlers import JsTypeError, js_truthy
from beholder_amd.sinks import HttpError
from beholder_amd.store import MediaNotFound, MemoryStore

from helpers import ENUM, Rig, api_media, cfg, progress_msg, status_msg, trello_media

TRELLO = "https://api.trello.com"


@pytest.fixture(autouse=True, params=["python", "native"])
def impl(request, monkeypatch):
    """Every case runs against the Python handlers and the compiled ones (ops/csrc/py_handlers.cpp)."""
    monkeypatch.setattr(helpers, "HANDLER_IMPL", request.param)
    return request.param


@pytest.fixture(autouse=True, params=["sync", "suspend"])
def io(request, monkeypatch):
    """...and with a store and sink client that answer within the call, and with ones that suspend
    at every call (production's shape: the socket clients always wait). Suspended, the compiled
    handlers return to the loop at each await and finish the event in their resume states
    (py_handlers.cpp: a Telegram failure resumed in state 5 must still skip Emby, Q4)."""
    monkeypatch.setattr(helpers, "SUSPEND", request.param == "suspend")
    return request.param


# ----------------------------------------------------------------- status ----
def test_status_trello_move_and_ack():
    """index.js:62-90,124: DB update, re-read, move card with pos 2, ack."""
    r = Rig(medias=[trello_media("m1", "QUEUED", card="CARD9")])
    d, exc = r.status(status_msg("m1", "DOWNLOADING"))
    assert exc is None and d.state == "acked"
    assert r.store.snapshot()["m1"].status == ENUM["DOWNLOADING"]
    assert r.calls() == [("PUT", f"{TRELLO}/1/cards/CARD9",
                          {"key": "TK", "token": "TT", "idList": "L-dl", "pos": "2"})]
    assert r.msgs() == [
        f"processing status update for media m1, status: {ENUM['DOWNLOADING']}",
        "moving media card m1 (card id CARD9)",
    ]


def test_status_non_trello_media_no_move():
    """index.js:79: only creator === 1 moves a card."""
    r = Rig(medias=[api_media("m2")])
    d, exc = r.status(status_msg("m2", "CONVERTING"))
    assert exc is None and d.acked
    assert r.calls() == []


def test_status_missing_list_warns_with_available_keys():
    """Q5 (index.js:80-89): no mapping -> warn with the status, text and keys; still acks."""
    r = Rig(medias=[trello_media("m1")])
    d, exc = r.status(status_msg("m1", "UPLOADING"))
    assert exc is None and d.acked
    assert r.calls() == []
    warn = r.msgs(40)
    assert warn == [f"unable to find list for status {ENUM['UPLOADING']} (UPLOADING) "
                    "avail ([queued,downloading,converting,deployed])"]


def test_status_list_pointer_js_truthiness():
    """index.js:81 `if (listPointer)`: an empty-string list id counts as missing."""
    r = Rig(config=cfg({"instance": {"flow_ids": {"queued": ""}}}), medias=[trello_media("m1")])
    d, exc = r.status(status_msg("m1", "QUEUED"))
    assert exc is None and r.calls() == [] and len(r.msgs(40)) == 1


def test_status_no_trello_short_circuit():
    """Q2 (index.js:68-72): DB update happens, then ack; no Trello, Telegram or Emby."""
    r = Rig(medias=[trello_media("m1")], no_trello=True)
    d, exc = r.status(status_msg("m1", "DEPLOYED"))
    assert exc is None and d.acked
    assert r.store.snapshot()["m1"].status == ENUM["DEPLOYED"]
    assert r.calls() == []
    assert r.store.get_calls == 0


def test_no_trello_env_is_js_truthy():
    """index.js:70 `if (process.env.NO_TRELLO)`: any non-empty string, even "0"."""
    assert cfg(env={"NO_TRELLO": "0"}).no_trello is True
    assert cfg(env={"NO_TRELLO": ""}).no_trello is False
    assert cfg(env={}).no_trello is False


def test_status_deployed_runs_telegram_then_emby():
    """index.js:92-119: DEPLOYED -> Telegram sendMessage then Emby refresh, then ack."""
    r = Rig(medias=[trello_media("m1", "UPLOADING", name="Cowboy Bebop", metadataId="1")])
    d, exc = r.status(status_msg("m1", "DEPLOYED"))
    assert exc is None and d.acked
    calls = r.calls()
    assert calls[0][0] == "PUT" and calls[0][2]["idList"] == "L-dep"
    assert calls[1] == ("GET", "https://api.telegram.org/bot123:TG/sendMessage", {
        "chat_id": "-1001", "text": "*New Anime:* Cowboy Bebop\nKitsu: https://kitsu.io/anime/1",
        "parse_mode": "markdown"})
    assert calls[2] == ("GET", "http://emby:8096/emby/library/refresh", {"api_key": "EMBYKEY"})
    assert "informing telegram that media 'm1' is available" in r.msgs()
    assert "telling emby to refresh at http://emby:8096" in r.msgs()


def test_status_deployed_uses_reread_db_status():
    """Q3 (index.js:76,94): the hooks key off the DB row, not the message status."""
    class StaleStore(helpers.SuspendingStore if helpers.SUSPEND else MemoryStore):
        async def update_status(self, media_id, status):  # write lost / lagging replica
            if helpers.SUSPEND:
                await asyncio.sleep(0)
            self.update_calls += 1

    r = Rig(medias=[api_media("m2", "DEPLOYED")])
    r.h.store = StaleStore([api_media("m2", "DEPLOYED")])
    d, exc = r.status(status_msg("m2", "QUEUED"))  # message says QUEUED, DB says DEPLOYED
    assert exc is None
    assert [c[1] for c in r.calls()] == ["https://api.telegram.org/bot123:TG/sendMessage",
                                         "http://emby:8096/emby/library/refresh"]


def test_status_telegram_failure_skips_emby_and_acks():
    """Q4 (index.js:92-122): one try block; Telegram failure skips Emby; warn; ack."""
    r = Rig(medias=[api_media("m2")])
    r.http.fail("GET", "https://api.telegram.org", status=500)
    d, exc = r.status(status_msg("m2", "DEPLOYED"))
    assert exc is None and d.acked
    assert [c[1] for c in r.calls()] == ["https://api.telegram.org/bot123:TG/sendMessage"]
    assert r.msgs(40) == ['failed to run deployed hooks: 500 - "\\"error\\""']


def test_status_emby_transport_error_is_swallowed():
    r = Rig(medias=[api_media("m2")])
    r.http.fail("GET", "http://emby:8096", message="ECONNREFUSED")
    d, exc = r.status(status_msg("m2", "DEPLOYED"))
    assert exc is None and d.acked
    assert r.msgs(40) == ["failed to run deployed hooks: ECONNREFUSED"]


def test_status_telegram_disabled_emby_only():
    r = Rig(config=cfg({"instance": {"telegram": {"enabled": False}}}), medias=[api_media("m2")])
    d, exc = r.status(status_msg("m2", "DEPLOYED"))
    assert [c[1] for c in r.calls()] == ["http://emby:8096/emby/library/refresh"]


def test_status_emby_requires_token_and_enabled():
    """index.js:110: keys.emby && keys.emby.token && instance.emby && instance.emby.enabled."""
    for over in ({"keys": {"emby": {"token": ""}}}, {"instance": {"emby": {"enabled": False}}}):
        r = Rig(config=cfg(over), medias=[api_media("m2")])
        r.status(status_msg("m2", "DEPLOYED"))
        assert [c[1] for c in r.calls()] == ["https://api.telegram.org/bot123:TG/sendMessage"]


def test_status_missing_telegram_keys_is_caught():
    """keys.telegram undefined -> TypeError inside the try -> warn, Emby skipped, ack."""
    import copy
    from beholder_amd.config import Config

    from helpers import BASE_CFG
    d0 = copy.deepcopy(BASE_CFG)
    del d0["keys"]["telegram"]
    r = Rig(config=Config.from_dict(d0), medias=[api_media("m2")])
    d, exc = r.status(status_msg("m2", "DEPLOYED"))
    assert exc is None and d.acked and r.calls() == []
    assert r.msgs(40) == ["failed to run deployed hooks: Cannot read property 'token' of undefined"]


def test_status_not_deployed_no_hooks():
    r = Rig(medias=[api_media("m2")])
    r.status(status_msg("m2", "CONVERTING"))
    assert r.calls() == []


@pytest.mark.parametrize("body", [b"\x0a\x02ab\x29", b"\xff\xff\xff"])
def test_status_decode_error_leaves_unacked(body):
    """Q1 (index.js:63): no try/catch — a decode failure escapes; message never acked.
    (protobufjs clamps a string that runs past the end, so ``0a 05 "ab"`` alone would decode.)"""
    r = Rig()
    d, exc = r.status(body)
    assert exc is not None and d.state == "pending"
    assert r.store.update_calls == 0


def test_status_unknown_media_leaves_unacked():
    """Q1 (index.js:76-79): reading `.creator` of a missing row throws -> un-acked."""
    r = Rig()
    d, exc = r.status(status_msg("nope", "QUEUED"))
    assert isinstance(exc, MediaNotFound) and d.state == "pending"
    assert r.store.update_calls == 1  # the UPDATE ran before the failing read


def test_status_unknown_enum_trello_media_throws():
    """Q6 (index.js:74,80): unknown status -> statusText undefined -> toLowerCase throws."""
    r = Rig(medias=[trello_media("m1")])
    d, exc = r.status(status_msg("m1", 99))
    assert isinstance(exc, JsTypeError) and d.state == "pending"


def test_status_unknown_enum_api_media_acks():
    """Q6: for non-Trello media statusText is never lowered, so the handler completes."""
    r = Rig(medias=[api_media("m2")])
    d, exc = r.status(status_msg("m2", 99))
    assert exc is None and d.acked


def test_status_trello_move_failure_leaves_unacked():
    """Q1: the Trello PUT is outside the try — a transport error escapes."""
    r = Rig(medias=[trello_media("m1")])
    r.http.fail("PUT", TRELLO, message="ECONNRESET")
    d, exc = r.status(status_msg("m1", "QUEUED"))
    assert isinstance(exc, HttpError) and d.state == "pending"


def test_status_trello_http_error_status_is_not_an_error():
    """trello npm resolves on any HTTP status: a 401 on the move still acks."""
    r = Rig(medias=[trello_media("m1")])
    r.http.fail("PUT", TRELLO, status=401)
    d, exc = r.status(status_msg("m1", "QUEUED"))
    assert exc is None and d.acked


# --------------------------------------------------------------- progress ----
def test_progress_trello_comment_with_host():
    """index.js:127-154 + Q8: counter{status lower}, comment text, comments counter, ack."""
    r = Rig(medias=[trello_media("m1", card="CARD1")])
    d = r.progress_(progress_msg("m1", "CONVERTING", 45, "worker-3"))
    assert d.acked
    assert r.progress.get({"status": "converting"}) == 1
    assert r.comments.get() == 1
    assert r.calls() == [("POST", f"{TRELLO}/1/cards/CARD1/actions/comments",
                          {"key": "TK", "token": "TT", "text": "CONVERTING: Progress **45%** (_worker-3_)"})]
    assert r.msgs() == [
        f"processing progress update on media m1 status {ENUM['CONVERTING']} percent 45",
        "creating comment on CARD1 with text: CONVERTING: Progress **45%** (_worker-3_)",
    ]


def test_progress_comment_without_host():
    """Q8: empty host is falsy -> no ` (_host_)` suffix."""
    r = Rig(medias=[trello_media("m1")])
    r.progress_(progress_msg("m1", "UPLOADING", 7, ""))
    assert r.calls()[0][2]["text"] == "UPLOADING: Progress **7%**"


def test_progress_api_media_no_comment_but_counted():
    r = Rig(medias=[api_media("m2")])
    d = r.progress_(progress_msg("m2", "DOWNLOADING", 10))
    assert d.acked and r.calls() == [] and r.comments.get() == 0
    assert r.progress.get({"status": "downloading"}) == 1


def test_progress_counter_increments_before_db_read():
    """index.js:136-140: the counter counts even when the DB read then fails."""
    r = Rig()
    d = r.progress_(progress_msg("missing", "QUEUED", 1))
    assert d.acked
    assert r.progress.get({"status": "queued"}) == 1
    assert r.msgs(40) == ["failed to update media progress media missing not found"]


def test_progress_unknown_enum_warns_acks_no_count():
    """Q6: unknown status -> caught; warn; ack; counter untouched."""
    r = Rig(medias=[trello_media("m1")])
    d = r.progress_(progress_msg("m1", 42, 3))
    assert d.acked and r.progress.values() == {}
    assert r.msgs(40) == ["failed to update media progress Cannot read property 'toLowerCase' of undefined"]


def test_progress_decode_error_still_acks():
    """Q7: decode errors are inside the try -> warn + ack."""
    r = Rig()
    d = r.progress_(b"\x0a\x05ab")
    assert d.acked and len(r.msgs(40)) == 1


def test_progress_comment_failure_acks_and_no_comment_count():
    """index.js:57,149-151: counter only after a successful POST; failure still acks."""
    r = Rig(medias=[trello_media("m1")])
    r.http.fail("POST", TRELLO, message="ETIMEDOUT")
    d = r.progress_(progress_msg("m1", "QUEUED", 1))
    assert d.acked and r.comments.get() == 0
    assert r.progress.get({"status": "queued"}) == 1


def test_progress_not_affected_by_no_trello():
    """Q2: NO_TRELLO does not affect the progress handler."""
    r = Rig(medias=[trello_media("m1")], no_trello=True)
    r.progress_(progress_msg("m1", "QUEUED", 1))
    assert len(r.calls()) == 1 and r.calls()[0][0] == "POST"


def test_comment_fallback_text():
    """index.js:54: `text || 'Failed to retrieve comment text.'`."""
    import asyncio
    r = Rig()
    asyncio.run(r.h.comment("C1", ""))
    assert r.calls()[0][2]["text"] == "Failed to retrieve comment text."
    assert r.comments.get() == 1


def test_progress_zero_progress_renders_zero():
    r = Rig(medias=[trello_media("m1")])
    r.progress_(progress_msg("m1", "QUEUED", 0))
    assert r.calls()[0][2]["text"] == "QUEUED: Progress **0%**"


def test_js_truthy():
    assert not js_truthy(None) and not js_truthy("") and not js_truthy(0) and not js_truthy(float("nan"))
    assert js_truthy("0") and js_truthy({}) and js_truthy([]) and js_truthy(-1) and js_truthy("false")


def test_suspending_rig_resumes_the_native_state_machine(impl, io):
    """The ``suspend`` cases really leave C: every await of a DEPLOYED status event suspends
    (update, re-read, Telegram, Emby) and the call completes in its resume states."""
    r = Rig(medias=[api_media("m2")])
    d, exc = r.status(status_msg("m2", "DEPLOYED"))
    assert exc is None and d.acked and len(r.calls()) == 2
    if impl == "native":
        st = r.impl.stats()
        assert (st["suspended"], st["completed_sync"]) == ((1, 0) if io == "suspend" else (0, 1))
