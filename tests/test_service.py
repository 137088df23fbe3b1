"""Service wiring (index.js:23-160): end-to-end over memory/AMQP sources, policies, ordering, shutdown."""
import asyncio
import json
import urllib.request

import pytest

from beholder_amd.config import Config, ConfigError
from beholder_amd.metrics import parse_exposition
from beholder_amd.service import Service
from beholder_amd.sinks import RecordingHttpClient
from beholder_amd.store import MemoryStore
from beholder_amd.topics import PROGRESS, STATUS
from beholder_amd import topics as T
from beholder_amd.transport.amqp import AmqpBroker, AmqpSource
from beholder_amd.transport.memory import MemoryBroker
from beholder_amd.utils.log import Logger, MemoryStream

from helpers import BASE_CFG, cfg, progress_msg, status_msg, trello_media


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


def make_service(source, medias=(), config=None, http=None, **over):
    c = config or cfg({"service": over} if over else None)
    return Service(c, source=source, store=MemoryStore(list(medias)), http=http or RecordingHttpClient(),
                   logger=Logger(stream=MemoryStream()), serve_metrics=False)


def test_memory_broker_end_to_end_and_metrics():
    async def go():
        b = MemoryBroker()
        svc = make_service(b.consumer(prefetch=100), [trello_media("m1", card="C1")])
        await svc.init()
        b.publish(PROGRESS, progress_msg("m1", "CONVERTING", 10, "w1"))
        b.publish(PROGRESS, progress_msg("m1", "CONVERTING", 20, "w1"))
        b.publish(STATUS, status_msg("m1", "DEPLOYED"))
        b.finish()
        stats = await svc.run()
        text = svc.registry.render()
        await svc.close()
        return stats, text, svc
    stats, text, svc = run(go())
    assert stats["received"] == {STATUS: 1, PROGRESS: 2}
    m = parse_exposition(text)
    assert m['beholder_progress_updates_total{status="converting"}'] == 2
    assert m["beholder_trello_comments"] == 2
    assert m['beholder_deliveries{state="acked"}'] == 3
    assert "# TYPE beholder_handle_latency_seconds histogram" in text
    assert m['beholder_handle_latency_seconds_bucket{le="+Inf"}'] == 3
    assert m['beholder_queue_latency_seconds_count'] == 3  # receive -> handler start, per delivery
    assert "# TYPE beholder_event_loop_lag_seconds histogram" in text
    assert "# TYPE beholder_gc_pause_seconds histogram" in text
    # the init log line (index.js:157)
    assert "initialized" in [r["msg"] for r in svc.log.stream.records()]


def test_startup_requires_trello_keys():
    """index.js:25 dereferences config.keys.trello.* unconditionally."""
    with pytest.raises(ConfigError):
        Config.from_dict({"instance": {"flow_ids": {}}})
    with pytest.raises(ConfigError):
        Config.from_dict({"keys": {"trello": {"key": "k", "token": "t"}}})  # index.js:60 needs instance


def _poison_run(policy: str):
    """Two undecodable status messages + prefetch 2 over real AMQP (quirk Q1)."""
    async def go():
        broker = await AmqpBroker().start()
        try:
            src = AmqpSource(broker.url, prefetch=2)
            svc = make_service(src, [trello_media("m1")], on_status_error=policy)
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            broker.publish(STATUS, b"\x0a\x05ab")  # truncated -> decode throws (index.js:63)
            broker.publish(STATUS, b"\x0a\x05cd")
            for i in range(3):
                broker.publish(STATUS, status_msg("m1", "QUEUED"))
            await asyncio.sleep(0.5)
            st = broker.stats(STATUS)
            svc.request_stop()
            await task
            await svc.close()
            return st, svc.stats()
        finally:
            await broker.stop()
    return run(go())


def test_q1_poison_status_messages_stall_prefetch_window():
    """Reference behaviour: errors leave messages un-acked, so 2 poison messages with
    prefetch 2 stall the status consumer (the 3 good messages are never delivered)."""
    st, stats = _poison_run("leave_unacked")
    assert st["unacked"] == 2 and st["depth"] == 3 and st["acked"] == 0
    assert stats["handler_errors"][STATUS] == 2


def test_q1_fix_nack_drop_keeps_consuming():
    st, stats = _poison_run("nack_drop")
    assert st["dead_lettered"] == 2 and st["acked"] == 3 and st["depth"] == 0


def test_q1_fix_nack_requeue_redelivers():
    st, _ = _poison_run("nack_requeue")
    assert st["requeued"] >= 2  # poison messages cycle back (redelivered)


class SlowHttp(RecordingHttpClient):
    """Sink with real suspension so handlers overlap (index.js:43: up to prefetch in flight)."""

    def __init__(self, delay):
        super().__init__(delay_s=delay)
        self.inflight = 0
        self.max_inflight = 0

    async def request(self, method, url, *, params=None, timeout=None):
        self.inflight += 1
        self.max_inflight = max(self.max_inflight, self.inflight)
        try:
            return await super().request(method, url, params=params, timeout=timeout)
        finally:
            self.inflight -= 1


def test_inflight_bounded_by_prefetch():
    async def go():
        b = MemoryBroker()
        http = SlowHttp(0.01)
        svc = make_service(b.consumer(prefetch=1000, batch=1000), [trello_media("m%d" % i) for i in range(50)],
                           http=http, prefetch=8)
        await svc.init()
        for i in range(200):
            b.publish(PROGRESS, progress_msg("m%d" % (i % 50), "QUEUED", i))
        b.finish()
        await svc.run()
        await svc.close()
        return http
    http = run(go())
    assert http.count == 200 and 1 < http.max_inflight <= 8 + 1


def test_default_ordering_is_unordered_per_media():
    """Q9: concurrent handlers for one media can finish out of order."""
    comments = _ordering_run("none")
    assert comments != sorted(comments)


def test_per_media_ordering_serialises():
    comments = _ordering_run("per_media")
    assert comments == sorted(comments)


def _ordering_run(ordering):
    import random

    class JitterHttp(RecordingHttpClient):
        def __init__(self):
            super().__init__()
            self.rng = random.Random(3)

        async def request(self, method, url, *, params=None, timeout=None):
            await asyncio.sleep(self.rng.random() * 0.01)
            return await super().request(method, url, params=params, timeout=timeout)

    async def go():
        b = MemoryBroker()
        http = JitterHttp()
        svc = make_service(b.consumer(), [trello_media("m1")], http=http, ordering=ordering)
        await svc.init()
        for p in range(40):
            b.publish(PROGRESS, progress_msg("m1", "QUEUED", p))
        b.finish()
        await svc.run()
        await svc.close()
        from beholder_amd.sinks import parse_query
        return [int(parse_query(u)["text"].split("**")[1].rstrip("%")) for _, u in http.calls]
    return run(go())


def test_graceful_stop_drains_inflight():
    async def go():
        b = MemoryBroker()
        http = SlowHttp(0.05)
        src = b.consumer()
        svc = make_service(src, [trello_media("m1")], http=http)
        await svc.init()
        for p in range(5):
            b.publish(PROGRESS, progress_msg("m1", "QUEUED", p))
        task = asyncio.ensure_future(svc.run())
        await asyncio.sleep(0.01)
        svc.request_stop()
        await task
        await svc.close()
        return src, b
    src, b = run(go())
    st = src.settler.stats()
    assert st["acked"] == 5 and st["pending"] == 0
    assert b.depth(PROGRESS) == 0 and src.unacked == 0  # nothing requeued: the acks landed


def test_metrics_http_endpoint():
    async def go():
        import copy
        d = copy.deepcopy(BASE_CFG)
        d["service"] = {"metrics": {"enabled": True, "host": "127.0.0.1", "port": 0}}
        b = MemoryBroker()
        svc = Service(Config.from_dict(d), source=b.consumer(), store=MemoryStore([trello_media("m1")]),
                      http=RecordingHttpClient(), logger=Logger(stream=MemoryStream()))
        await svc.init()
        port = svc.metrics_server.bound_port
        b.publish(PROGRESS, progress_msg("m1", "QUEUED", 5))
        b.finish()
        await svc.run()
        loop = asyncio.get_running_loop()

        def fetch(path):
            with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=5) as r:
                return r.status, r.headers.get("Content-Type"), r.read().decode()
        res = {p: await loop.run_in_executor(None, fetch, p) for p in ("/metrics", "/healthz", "/stats")}
        await svc.close()
        return res
    res = run(go())
    status, ctype, body = res["/metrics"]
    assert status == 200 and ctype.startswith("text/plain; version=0.0.4")
    assert 'beholder_progress_updates_total{status="queued"} 1' in body
    assert "process_resident_memory_bytes" in body
    assert res["/healthz"][0] == 200
    assert json.loads(res["/stats"][2])["received"][PROGRESS] == 1


def test_amqp_end_to_end_service():
    async def go():
        broker = await AmqpBroker().start()
        try:
            http = RecordingHttpClient()
            svc = make_service(AmqpSource(broker.url), [trello_media("m1", card="C1")], http=http)
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            for p in range(20):
                broker.publish(PROGRESS, progress_msg("m1", "UPLOADING", p))
            broker.publish(STATUS, status_msg("m1", "DEPLOYED"))
            for _ in range(200):
                if broker.stats(PROGRESS)["acked"] == 20 and broker.stats(STATUS)["acked"] == 1:
                    break
                await asyncio.sleep(0.02)
            svc.request_stop()
            await task
            await svc.close()
            return broker.stats(PROGRESS), broker.stats(STATUS), http
        finally:
            await broker.stop()
    sp, ss, http = run(go())
    assert sp["acked"] == 20 and ss["acked"] == 1 and sp["unacked"] == 0
    assert http.count == 20 + 3  # 20 comments + move + telegram + emby


def test_graceful_stop_over_amqp_acks_inflight_not_redelivered():
    """SIGTERM during slow handlers: consumers are cancelled first, in-flight handlers finish and
    their acks reach the broker, nothing is redelivered."""
    async def go():
        broker = await AmqpBroker().start()
        try:
            http = SlowHttp(0.05)
            svc = make_service(AmqpSource(broker.url, prefetch=10), [trello_media("m1")], http=http)
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            for p in range(30):
                broker.publish(PROGRESS, progress_msg("m1", "QUEUED", p))
            await asyncio.sleep(0.02)  # some handlers are mid-request
            svc.request_stop()
            await task
            await svc.close()
            await asyncio.sleep(0.05)
            return broker.stats(PROGRESS), http.count
        finally:
            await broker.stop()
    st, calls = run(go())
    assert st["requeued"] == 0  # nothing that was handled comes back
    assert st["acked"] == calls and st["acked"] + st["depth"] == 30 and st["unacked"] == 0


def test_trace_spans():
    async def go():
        b = MemoryBroker()
        stream = MemoryStream()
        c = cfg({"service": {"trace": True}})
        svc = Service(c, source=b.consumer(), store=MemoryStore([trello_media("m1")]), http=RecordingHttpClient(),
                      logger=Logger(stream=stream, level="debug"), serve_metrics=False)
        await svc.init()
        b.publish(PROGRESS, progress_msg("m1", "QUEUED", 1))
        b.publish(STATUS, b"\x0a\x05ab")
        b.finish()
        await svc.run()
        await svc.close()
        return [r for r in stream.records() if r.get("msg") == "handled"]
    spans = run(go())
    assert sorted((s["span"], s["outcome"], s["state"]) for s in spans) == [
        (PROGRESS, "ok", "acked"), (STATUS, "unsettled", "pending")]
    assert all(s["handle_us"] >= 0 and s["queue_us"] >= 0 for s in spans)


def test_transport_metrics_exposed():
    async def go():
        broker = await AmqpBroker().start()
        try:
            svc = make_service(AmqpSource(broker.url), [trello_media("m1")])
            await svc.init()
            text = svc.registry.render()
            await svc.close()
            return parse_exposition(text)
        finally:
            await broker.stop()
    m = run(go())
    assert m['beholder_transport{kind="amqp",field="connected"}'] == 1
    assert m['beholder_transport{kind="amqp",field="reconnects"}'] == 0


class _FakeDelivery:
    def __init__(self, topic_id):
        self.topic_id, self.topic, self.settled, self.nacks = topic_id, T.TOPIC_NAMES_BY_ID[topic_id], False, []

    def nack(self, requeue):
        self.nacks.append(requeue)
        self.settled = True


@pytest.mark.parametrize("policy", ["nack_drop", "nack_requeue"])
def test_on_status_error_policy_applies_to_status_only(policy):
    """`service.on_status_error` is the Q1 knob: a progress handler error (it only raises on
    something like cancellation, Q7) leaves its delivery as the reference would."""
    async def go():
        svc = make_service(MemoryBroker().consumer(), [], on_status_error=policy)
        await svc.init()
        svc._on_handler_error(st, RuntimeError("boom"))
        svc._on_handler_error(pr, RuntimeError("boom"))
        await svc.close()
    st, pr = _FakeDelivery(T.STATUS_ID), _FakeDelivery(T.PROGRESS_ID)
    run(go())
    assert st.nacks == [policy == "nack_requeue"] and pr.nacks == [] and not pr.settled


def test_loop_lag_and_gc_pause_histograms():
    """The 100 ms log flusher's lateness is the loop lag; gc.callbacks time every collection; a
    closed service leaves no callback behind."""
    import gc
    import time as _time

    async def go():
        b = MemoryBroker()
        svc = make_service(b.consumer(prefetch=100))
        await svc.init()
        n_cb = len(gc.callbacks)
        task = asyncio.ensure_future(svc._flush_logs_periodically(0.01))
        await asyncio.sleep(0.03)
        _time.sleep(0.05)  # block the loop: the next wake-up is >= 40 ms late
        await asyncio.sleep(0.03)
        task.cancel()
        gc.collect()
        await svc.close()
        return svc, n_cb, len(gc.callbacks)
    svc, n_cb, after = asyncio.run(go())
    assert svc.loop_lag.count >= 3 and svc.loop_lag.max >= 30_000_000
    assert svc.gc_pause.count >= 1
    assert after == n_cb - 1


def test_the_loop_stays_responsive_under_sustained_load():
    """The dispatch loop yields to the event loop at least every other batch: a batch that came
    after the source waited needs no extra yield, one that did not gets `sleep(0)` (a timer keeps
    ticking while a 200k-event stream that never runs dry goes through)."""
    from beholder_amd.bench.generator import Workload, bench_config
    from beholder_amd.transport.ingest import BytesSource
    w = Workload(n_media=200, seed=5)
    data = w.framed(200_000)
    ticks = []

    async def go():
        svc = Service(Config.from_dict(bench_config()), source=BytesSource(data, batch=256), store=MemoryStore(w.media),
                      http=RecordingHttpClient(keep=0), logger=Logger(stream=MemoryStream()), serve_metrics=False)
        await svc.init()

        async def ticker():
            while True:
                await asyncio.sleep(0.002)
                ticks.append(1)
        t = asyncio.ensure_future(ticker())
        loop = asyncio.get_running_loop()
        t0 = loop.time()
        st = await svc.run()
        took = loop.time() - t0
        t.cancel()
        await svc.close()
        return st, took
    st, took = asyncio.run(go())
    assert st["source"]["acked"] == 200_000
    assert len(ticks) >= max(3, int(took / 0.002 * 0.1)), (len(ticks), took)  # starved: ~0


def test_signal_has_event_semantics():
    from beholder_amd.utils.waits import Signal

    async def go():
        s = Signal()
        assert not s.is_set()
        got = []

        async def waiter(i):
            await s.wait()
            got.append(i)
        ts = [asyncio.ensure_future(waiter(i)) for i in range(3)]
        await asyncio.sleep(0)
        assert got == []
        s.set()
        await asyncio.sleep(0)
        assert sorted(got) == [0, 1, 2] and s.is_set()
        await s.wait()  # set: returns at once
        s.clear()
        t = asyncio.ensure_future(s.wait())
        await asyncio.sleep(0)
        assert not t.done()
        s.set()
        await t
        for x in ts:
            await x
    asyncio.run(go())


def test_signal_wait_after_a_cancelled_waiter():
    """The one-waiter contract (utils/waits.py): a waiter cancelled mid-wait leaves the Signal
    usable; the next wait gets a fresh future and is woken by the next set()."""
    from beholder_amd.utils.waits import Signal

    async def go():
        s = Signal()
        t = asyncio.ensure_future(s.wait())
        await asyncio.sleep(0)
        t.cancel()
        try:
            await t
        except asyncio.CancelledError:
            pass
        t2 = asyncio.ensure_future(s.wait())
        await asyncio.sleep(0)
        pending = not t2.done()
        s.set()
        return pending, await asyncio.wait_for(t2, 1)
    assert asyncio.run(go()) == (True, True)
