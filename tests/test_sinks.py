"""Trello / Telegram / Emby sinks over real HTTP (both clients -> local fake server).

Pins the outbound contract of SURVEY.md §2.4: methods, paths, query parameters,
and the error semantics of the two reference HTTP libraries.
"""
import asyncio

import pytest

from beholder_amd.bench.fakes import FakeHttpServer
from beholder_amd.metrics import Registry, parse_exposition
from beholder_amd.sinks import (AiohttpClient, EmbyClient, H1Client, HttpError, SinkObserver, TelegramClient, TrelloClient,
                                deployed_text, redact)


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


@pytest.fixture(params=["h1", "aiohttp"])
def http_cls(request):
    return H1Client if request.param == "h1" else AiohttpClient


@pytest.fixture
def server():
    with FakeHttpServer() as s:
        yield s


def test_trello_comment_and_move_over_http(server, http_cls):
    async def go():
        http = http_cls(timeout_s=5)
        t = TrelloClient("KEY", "TOK", http, base_url=server.url)
        await t.make_request("post", "/1/cards/C1/actions/comments", {"text": "DEPLOYED: Progress **5%** (_h_)"})
        await t.make_request("put", "/1/cards/C1", {"idList": "L9", "pos": 2})
        await http.close()
    run(go())
    assert server.requests == [
        ("POST", "/1/cards/C1/actions/comments", {"key": "KEY", "token": "TOK",
                                                  "text": "DEPLOYED: Progress **5%** (_h_)"}),
        ("PUT", "/1/cards/C1", {"key": "KEY", "token": "TOK", "idList": "L9", "pos": "2"}),
    ]


def test_trello_resolves_on_http_error_status(server, http_cls):
    """trello npm only rejects on transport errors (index.js:83 move failures surface only then)."""
    server.status_for["/1/cards"] = 401

    async def go():
        http = http_cls(timeout_s=5)
        r = await TrelloClient("k", "t", http, base_url=server.url).make_request("put", "/1/cards/x", {"pos": 2})
        strict = TrelloClient("k", "t", http, base_url=server.url, strict=True)
        with pytest.raises(HttpError):
            await strict.make_request("put", "/1/cards/x", {})
        await http.close()
        return r.status
    assert run(go()) == 401


def test_telegram_and_emby_over_http(server, http_cls):
    async def go():
        http = http_cls(timeout_s=5)
        await TelegramClient("123:ABC", http, base_url=server.url).send_message(
            "-100", deployed_text("Bebop", "1"), "markdown")
        await EmbyClient(server.url, "EK", http).refresh_library()
        await http.close()
    run(go())
    assert server.requests == [
        ("GET", "/bot123:ABC/sendMessage", {"chat_id": "-100", "parse_mode": "markdown",
                                            "text": "*New Anime:* Bebop\nKitsu: https://kitsu.io/anime/1"}),
        ("GET", "/emby/library/refresh", {"api_key": "EK"}),
    ]


def test_request_promise_semantics_reject_non_2xx(server, http_cls):
    server.status_for["/emby"] = 500

    async def go():
        http = http_cls(timeout_s=5)
        with pytest.raises(HttpError) as ei:
            await EmbyClient(server.url, "k", http).refresh_library()
        await http.close()
        return ei.value
    e = run(go())
    assert e.status == 500 and str(e).startswith("500 - ")


def test_transport_errors_never_leak_tokens(http_cls):
    async def go():
        http = http_cls(timeout_s=0.5)
        with pytest.raises(HttpError) as ei:
            await TelegramClient("SECRET:TOKEN", http, base_url="http://127.0.0.1:9").send_message("c", "t")
        with pytest.raises(HttpError) as ej:
            await TrelloClient("SECRETKEY", "SECRETTOK", http, base_url="http://127.0.0.1:9").make_request(
                "post", "/1/cards/x/actions/comments", {"text": "x"})
        await http.close()
        return str(ei.value) + str(ej.value)
    msg = run(go())
    assert "SECRET" not in msg
    assert redact("https://api.telegram.org/bot1:AB/sendMessage?chat_id=1") == "https://api.telegram.org/bot***/sendMessage"


def test_sink_metrics(server, http_cls):
    server.status_for["/emby"] = 503

    async def go():
        reg = Registry()
        obs = SinkObserver(reg)
        http = http_cls(timeout_s=5)
        await TrelloClient("k", "t", http, base_url=server.url, observer=obs).make_request("put", "/1/cards/a", {})
        with pytest.raises(HttpError):
            await EmbyClient(server.url, "k", http, observer=obs).refresh_library()
        refused = http_cls(timeout_s=0.5)
        with pytest.raises(HttpError):
            await EmbyClient("http://127.0.0.1:9", "k", refused, observer=obs).refresh_library()
        await refused.close()
        await http.close()
        return parse_exposition(reg.render())
    m = run(go())
    assert m['beholder_sink_requests_total{sink="trello",code="200"}'] == 1
    assert m['beholder_sink_requests_total{sink="emby",code="503"}'] == 1
    assert m['beholder_sink_requests_total{sink="emby",code="error"}'] == 1
    assert m['beholder_sink_request_seconds_count{sink="trello"}'] == 1


def test_aiohttp_client_works_under_the_native_driver(server):
    """aiohttp's timeout context needs a current task; handlers suspended on I/O are resumed by
    ops.Driver (no Task), so the client runs each request in its own task."""
    from beholder_amd.ops import Driver

    async def handler(http):
        await asyncio.sleep(0.001)  # first suspension: from here on the Driver steps us
        r = await http.request("GET", server.url + "/emby/library/refresh", params={"api_key": "k"})
        return r.status

    async def go():
        http = AiohttpClient(timeout_s=5)
        out = asyncio.get_running_loop().create_future()
        coro = handler(http)
        Driver(coro, lambda drv, exc: out.set_result(exc)).start(coro.send(None))
        exc = await out
        await http.close()
        return exc
    assert run(go()) is None


@pytest.mark.parametrize("impl", ["python", "native"])
def test_crlf_in_db_sourced_path_is_percent_encoded(server, impl, monkeypatch):
    """A creatorId holding CR/LF (it comes from the media table, index.js:83) must not split the
    request line toward Trello: the H1 client percent-encodes every byte outside 0x21-0x7E, for
    the Python handlers and for the compiled ones (which issue the request through the same
    client)."""
    import helpers
    from helpers import Rig, status_msg, trello_media
    monkeypatch.setattr(helpers, "HANDLER_IMPL", impl)
    evil = "abc\r\nX-Evil:1\r\nY:"  # no space: the old check only quoted on SP / non-ASCII

    async def go():
        http = H1Client(timeout_s=5)
        rig = Rig(medias=[trello_media("m1", "QUEUED", card=evil)], http=http)
        rig.h.trello = TrelloClient("KEY", "TOK", http, base_url=server.url)
        if impl == "native":
            from beholder_amd.handlers import native_handlers
            rig.impl = native_handlers(rig.h)
        await rig.impl.on_status(rig.delivery(helpers.STATUS_ID, status_msg("m1", "DOWNLOADING")))
        await http.close()
    run(go())
    assert len(server.requests) == 1
    method, path, query = server.requests[0]
    assert method == "PUT" and path == "/1/cards/abc%0D%0AX-Evil:1%0D%0AY:"
    assert query["key"] == "KEY" and query["token"] == "TOK"


def test_control_characters_in_authority_are_rejected():
    async def go():
        http = H1Client(timeout_s=1)
        try:
            with pytest.raises(HttpError):
                await http.request("GET", "http://127.0.0.1\r\nX: 1/path")
        finally:
            await http.close()
    run(go())
