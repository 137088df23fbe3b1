"""Opt-in sink rate limits and 429 retries (sinks/ratelimit.py). Off by default: reference
behaviour (requests as fast as events arrive; a 429 resolves like any status)."""
from __future__ import annotations

import asyncio

import pytest

import helpers
from beholder_amd.handlers import native_handlers
from beholder_amd.sinks import HttpResponse, RecordingHttpClient, TrelloClient
from beholder_amd.sinks.ratelimit import RetryPolicy, TokenBucket, from_config, guarded
from helpers import Rig, progress_msg, trello_media


class FakeClock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


def test_bucket_burst_then_refill():
    clk = FakeClock()
    b = TokenBucket(3, 1.0, clock=clk)
    assert [b.try_acquire() for _ in range(4)] == [True, True, True, False]
    clk.t = 0.34  # 3 tokens per second: one more
    assert b.try_acquire() and not b.try_acquire()
    with pytest.raises(ValueError):
        TokenBucket(0, 1)


def test_bucket_waiters_are_served_in_order_at_the_rate():
    async def go():
        b = TokenBucket(2, 0.1)  # 20 per second, burst 2
        order = []

        async def req(i):
            await b.acquire()
            order.append((i, asyncio.get_running_loop().time()))

        t0 = asyncio.get_running_loop().time()
        await asyncio.gather(*(req(i) for i in range(8)))
        return order, t0, b.stats()

    order, t0, st = asyncio.run(go())
    assert [i for i, _ in order] == list(range(8))  # FIFO
    assert order[-1][1] - t0 >= 0.25  # 6 waited for 1/20 s each (burst of 2 went at once)
    assert st["granted"] == 8 and st["delayed"] == 6 and st["waiting"] == 0


def test_cancelled_waiter_leaves_the_queue():
    async def go():
        b = TokenBucket(1, 10.0)
        assert b.try_acquire()
        t = asyncio.ensure_future(b.acquire())
        await asyncio.sleep(0)
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        return b.stats()

    assert asyncio.run(go())["waiting"] == 0


def test_retry_on_429_honours_retry_after():
    answers = [HttpResponse(429, b"{}", {"Retry-After": "0.01"}), HttpResponse(429, b"{}"),
               HttpResponse(200, b"{}")]
    sent = []

    async def send():
        sent.append(1)
        return answers[len(sent) - 1]

    pol = RetryPolicy(3, base_s=0.01)
    r = asyncio.run(guarded(None, pol, send))
    assert r.status == 200 and len(sent) == 3 and pol.retried == 2
    assert pol.delay(0, "2") == 2.0 and pol.delay(3, None) == 0.08 and pol.delay(10, "bad") == 10.24
    sent.clear()
    answers[:] = [HttpResponse(429, b"{}")] * 5
    r = asyncio.run(guarded(None, RetryPolicy(1, base_s=0.001), send))
    assert r.status == 429 and len(sent) == 2  # gave up after one retry: the 429 resolves (trello semantics)


def test_from_config():
    assert from_config(None) == (None, None)
    b, r = from_config({"rate_limit": {"requests": 100, "per_s": 10}, "retry_429": 2})
    assert b.capacity == 100 and b.rate == 10 and r.retries == 2


@pytest.mark.parametrize("impl", ["python", "native"])
def test_trello_comments_are_paced_when_limited(impl, monkeypatch):
    """With a limit the compiled handlers take the client's own make_request (limiter inside);
    every comment still goes out, in order, at the configured rate."""
    monkeypatch.setattr(helpers, "HANDLER_IMPL", impl)
    r = Rig(medias=[trello_media("m1", card="C1")])
    r.h.trello = TrelloClient("TK", "TT", r.http, limiter=TokenBucket(5, 0.1))  # 50/s, burst 5
    target = r.h if impl == "python" else native_handlers(r.h)

    async def go():
        t0 = asyncio.get_running_loop().time()
        ds = [r.delivery(2, progress_msg("m1", "UPLOADING", i)) for i in range(15)]
        await asyncio.gather(*(helpers._await(target.on_progress(d)) for d in ds))
        return asyncio.get_running_loop().time() - t0, ds

    dt, ds = asyncio.run(go())
    assert all(d.acked for d in ds)
    texts = [q["text"] for _, _, q in r.calls()]
    assert texts == [f"UPLOADING: Progress **{i}%**" for i in range(15)]
    assert dt >= 0.18  # 10 of 15 waited for 1/50 s each
    assert r.comments.get() == 15


def test_service_builds_policies_from_config():
    from beholder_amd.config import Config
    from beholder_amd.service import Service
    from beholder_amd.store import MemoryStore
    from beholder_amd.transport.memory import MemoryBroker

    d = {k: v for k, v in helpers.BASE_CFG.items()}
    d["service"] = {"metrics": {"enabled": False},
                    "sinks": {"trello": {"rate_limit": {"requests": 100, "per_s": 10}, "retry_429": 2}}}

    async def go():
        svc = Service(Config.from_dict(d, env={}), source=MemoryBroker().consumer(prefetch=100), store=MemoryStore(),
                      http=RecordingHttpClient(), logger=helpers.Logger(stream=helpers.MemoryStream()))
        await svc.init()
        st = svc.stats()
        await svc.close()
        return svc, st

    svc, st = asyncio.run(go())
    assert svc.trello.limiter.capacity == 100 and svc.trello.retry.retries == 2
    assert svc.telegram.limiter is None and st["rate_limits"]["trello"]["granted"] == 0
