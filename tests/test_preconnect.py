"""``service.http.preconnect``: sink connections opened at startup instead of inside the first
deliveries' handle latency (the warm-up tail of ``tcp_e2e``, docs/STATUS.md open items)."""
import asyncio
import socket

import pytest

from beholder_amd.config import ConfigError
from beholder_amd.service import Service
from beholder_amd.sinks import H1Client, RecordingHttpClient
from beholder_amd.store import MemoryStore
from beholder_amd.topics import STATUS
from beholder_amd.transport.memory import MemoryBroker
from beholder_amd.utils.log import Logger, MemoryStream

from helpers import cfg, status_msg, trello_media
from test_h1 import OK, Scripted


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_preconnected_connections_serve_a_burst_without_new_connects():
    async def go():
        s = await Scripted(lambda n, m, t, h: OK).start()
        c = H1Client(timeout_s=5)
        base = f"http://127.0.0.1:{s.port}"
        opened, err = await c.preconnect(base + "/1/cards", 8)
        before = s.connections
        rs = await asyncio.gather(*[c.request("GET", f"{base}/{i}") for i in range(8)])
        st = c.stats()
        await c.close()
        await s.stop()
        return opened, err, before, s.connections, rs, st
    opened, err, before, after, rs, st = run(go())
    assert (opened, err) == (8, None) and before == after == 8
    assert all(r.status == 200 for r in rs) and st["reused"] == 8 and st["connections"] == 8


def test_preconnect_never_exceeds_max_per_host():
    async def go():
        s = await Scripted(lambda n, m, t, h: OK).start()
        c = H1Client(timeout_s=5, max_per_host=3)
        base = f"http://127.0.0.1:{s.port}"
        first = await c.preconnect(base, 10)
        again = await c.preconnect(base, 10)  # the pool is full already
        await c.close()
        await s.stop()
        return first, again, s.connections
    first, again, conns = run(go())
    assert first == (3, None) and again == (0, None) and conns == 3


def test_preconnect_to_a_dead_origin_reports_instead_of_raising():
    async def go():
        c = H1Client(timeout_s=2)
        url = f"http://127.0.0.1:{_free_port()}/x"
        opened, err = await c.preconnect(url, 4)
        open_after = c._origin(f"http://127.0.0.1:{url.split(':')[2].split('/')[0]}").open
        await c.close()
        return opened, err, open_after
    opened, err, open_after = run(go())
    assert opened == 0 and isinstance(err, OSError) and open_after == 0  # no pool slot leaked


def test_preconnect_config_is_validated():
    assert cfg().data["service"]["http"]["preconnect"] == 0
    assert cfg({"service": {"http": {"preconnect": 50}}}).data["service"]["http"]["preconnect"] == 50
    for bad in (-1, "10", 1.5, True):
        with pytest.raises(ConfigError, match="preconnect"):
            cfg({"service": {"http": {"preconnect": bad}}})


def _service(c, http, medias=()):
    return Service(c, source=MemoryBroker().consumer(prefetch=100), store=MemoryStore(list(medias)), http=http,
                   logger=Logger(stream=MemoryStream()), serve_metrics=False)


def test_service_preconnects_each_sink_origin_the_handlers_will_call():
    async def go():
        trello = await Scripted(lambda n, m, t, h: OK).start()
        hooks = await Scripted(lambda n, m, t, h: OK).start()  # Telegram and Emby on one origin
        dead = _free_port()
        c = cfg({"service": {"http": {"preconnect": 3},
                             "endpoints": {"trello": f"http://127.0.0.1:{trello.port}",
                                           "telegram": f"http://127.0.0.1:{hooks.port}"}},
                 "instance": {"emby": {"host": f"http://127.0.0.1:{dead}"}}})
        http = H1Client(timeout_s=2)
        svc = _service(c, http)
        await svc.init()
        await svc.close()  # flushes the log
        msgs = [r["msg"] for r in svc.log.stream.records()]
        levels = {r["msg"]: r["level"] for r in svc.log.stream.records()}
        await http.close()
        await trello.stop()
        await hooks.stop()
        return trello.connections, hooks.connections, msgs, levels, dead
    t_conns, h_conns, msgs, levels, dead = run(go())
    assert t_conns == 3 and h_conns == 3
    pre = [m for m in msgs if m.startswith("preconnect to ")]
    assert len(pre) == 3
    bad = [m for m in pre if f":{dead}" in m]
    assert len(bad) == 1 and "0/3 connections" in bad[0] and levels[bad[0]] == 40  # warn, startup went on
    assert "initialized" in msgs


def test_service_preconnect_is_harmless_for_clients_without_a_pool():
    async def go():
        b = MemoryBroker()
        http = RecordingHttpClient()
        c = cfg({"service": {"http": {"preconnect": 5}}})  # a client without a pool opens none
        svc = Service(c, source=b.consumer(prefetch=100), store=MemoryStore([trello_media("m1", card="C1")]),
                      http=http, logger=Logger(stream=MemoryStream()), serve_metrics=False)
        await svc.init()
        b.publish(STATUS, status_msg("m1", "DEPLOYED"))
        b.finish()
        stats = await svc.run()
        await svc.close()
        return stats, [r["msg"] for r in svc.log.stream.records()]
    stats, msgs = run(go())
    assert stats["received"][STATUS] == 1 and stats["source"]["acked"] == 1
    assert sum(m.startswith("preconnect to ") for m in msgs) == 3  # trello, telegram, emby: 0 each, no error


def test_preconnect_resolves_a_host_name_once_for_the_batch(monkeypatch):
    from beholder_amd.utils import netconn
    if not netconn.enabled():
        pytest.skip("native connections switched off")

    async def go():
        s = await Scripted(lambda n, m, t, h: OK).start()
        loop = asyncio.get_running_loop()
        real = loop.getaddrinfo
        lookups = []

        async def counting(host, *a, **kw):
            lookups.append(host)
            return await real("127.0.0.1", *a, **kw)
        monkeypatch.setattr(loop, "getaddrinfo", counting)
        c = H1Client(timeout_s=5)
        opened, err = await c.preconnect(f"http://sink.invalid:{s.port}/", 6)
        r = await c.request("GET", f"http://sink.invalid:{s.port}/x")
        await c.close()
        await s.stop()
        return opened, err, lookups, r.status, s.connections
    opened, err, lookups, status, conns = run(go())
    assert (opened, err, status, conns) == (6, None, 200, 6)
    assert lookups == ["sink.invalid"]  # one lookup for six connections; the request reused one


def test_startup_waits_for_preconnect_at_most_preconnect_wait_s():
    """A sink that never answers the connect (dropped packets) holds startup for
    ``preconnect_wait_s``, not for the request timeout; close() cancels what is still running."""
    class Stuck(RecordingHttpClient):
        cancelled = 0

        async def preconnect(self, url, n):
            try:
                await asyncio.sleep(3600)
            except asyncio.CancelledError:
                Stuck.cancelled += 1
                raise

    async def go():
        c = cfg({"service": {"http": {"preconnect": 4, "preconnect_wait_s": 0.2}}})
        svc = _service(c, Stuck())
        loop = asyncio.get_running_loop()
        t0 = loop.time()
        await svc.init()
        dt = loop.time() - t0
        pending = len(svc._preconnecting)
        await svc.close()
        return dt, pending, [r["msg"] for r in svc.log.stream.records()]
    dt, pending, msgs = run(go())
    assert 0.2 <= dt < 2.0 and pending == 3 and Stuck.cancelled == 3  # trello, telegram, emby
    assert any("still connecting after 0.2 s" in m for m in msgs) and "initialized" in msgs
    with pytest.raises(ConfigError, match="preconnect_wait_s"):
        cfg({"service": {"http": {"preconnect_wait_s": -1}}})


def test_max_connecting_config_is_validated():
    assert cfg().data["service"]["http"]["max_connecting"] == 8
    for bad in (0, -1, "8", True, 1.5):
        with pytest.raises(ConfigError, match="max_connecting"):
            cfg({"service": {"http": {"max_connecting": bad}}})
    from beholder_amd.service import make_http_client
    assert make_http_client({"max_connecting": 3}).max_connecting == 3
    assert make_http_client({}).max_connecting == 8


def test_preconnected_connections_keep_alive_from_when_consuming_starts():
    """a startup that took longer than keepalive_s must not have its preconnected
    connections dropped at the first delivery: the service restarts their keep-alive clock when
    it starts consuming (H1Client.touch_idle)."""
    async def go():
        s = await Scripted(lambda n, m, t, h: OK).start()
        http = H1Client(timeout_s=5, keepalive_s=0.3)
        url = f"http://127.0.0.1:{s.port}"
        c = cfg({"service": {"http": {"preconnect": 2}, "endpoints": {"trello": url, "telegram": url}},
                 "instance": {"telegram": {"enabled": False}, "emby": {"enabled": False}}})
        svc = _service(c, http)
        real = svc._preconnect

        async def slow_preconnect(n, endpoints):
            await real(n, endpoints)
            await asyncio.sleep(0.5)  # startup outlasts keepalive_s after the connects
        svc._preconnect = slow_preconnect
        await svc.init()
        before = s.connections
        await http.request("GET", url + "/1/cards/x")
        reused = http.counts["reused"]
        await svc.close()
        await http.close()
        await s.stop()
        return before, s.connections, reused
    before, after, reused = run(go())
    assert before == 2 and after == 2 and reused == 1  # without the touch: dropped, a 3rd connect


def test_service_makes_the_tls_context_at_startup_only_for_https_sinks():
    """HTTPS sinks: the native TLS context (one-time OpenSSL warm-up, handshake threads) is made by
    ``Service.init``, not by the first connect of the first burst. Plain-HTTP sinks never make one.
    No connection is opened either way (preconnect stays 0)."""
    from beholder_amd.utils import netconn

    async def go(scheme):
        c = cfg({"service": {"endpoints": {"trello": f"{scheme}://127.0.0.1:1", "telegram": f"{scheme}://127.0.0.1:1"}}})
        http = H1Client(timeout_s=2)
        svc = _service(c, http)
        await svc.init()
        made = http._ntls
        opened = sum(o.open for o in http._origins.values())
        await svc.close()
        await http.close()
        return made, opened
    made, opened = run(go("https"))
    assert opened == 0
    if netconn.enabled():
        assert made is not None and made is not False and type(made).__name__ == "TlsContext"
    made, opened = run(go("http"))
    assert made is None and opened == 0
