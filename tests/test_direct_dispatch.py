"""Deliveries handed over from the AMQP read callback, and the NetPoller batch around them.

At a low rate every delivery used to cost two extra trips through the event loop: one to wake
the service's task that dispatches the batch, one for the ack flush scheduled with call_soon.
Now the source hands the deliveries to the waiting service from its read callback
(``AmqpSource.direct``), inside a NetPoller batch scope (``_enter`` / ``_exit``): the Postgres
queries the handlers issue go out together at its end. Acks settled inside any NetPoller batch
are flushed at its end (``NetPoller.defer``). These tests pin the scope, the ordering and the
failure path; the chaos, service and oracle suites run over the same code."""
import asyncio

import pytest

from beholder_amd.sinks import H1Client
from beholder_amd.store import MemoryStore
from beholder_amd.topics import PROGRESS
from beholder_amd.transport.amqp import AmqpBroker, AmqpSource
from beholder_amd.utils import netconn
from beholder_amd.utils.log import Logger, MemoryStream

import test_h1
from helpers import cfg, progress_msg, trello_media



def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


@pytest.mark.skipif(not netconn.enabled(), reason="BEHOLDER_NATIVE_IO=0: no NetPoller")
def test_poller_batch_scope_defers_callables_to_its_end():
    """defer() is False outside a batch; inside one the callable runs once, at the end of the
    outermost scope; a failing callable goes to sys.unraisablehook and the others still run."""
    import sys

    async def go():
        loop = asyncio.get_running_loop()
        s = await test_h1.Scripted(lambda n, m, t, h: test_h1.OK).start()
        c = H1Client(timeout_s=5)
        try:
            await c.request("GET", f"http://127.0.0.1:{s.port}/")  # a pooled NetConn: the poller exists
            p = loop._beholder_netpoller
            calls = []
            outside = p.defer(lambda: calls.append("outside"))
            p._enter()
            p._enter()
            inside = p.defer(lambda: calls.append("a"))
            p.defer(lambda: 1 / 0)
            p.defer(lambda: calls.append("b"))
            p._exit()
            nested_end = list(calls)  # the inner _exit ends nothing
            seen = []
            old = sys.unraisablehook
            sys.unraisablehook = lambda u: seen.append(type(u.exc_value).__name__)
            try:
                p._exit()
            finally:
                sys.unraisablehook = old
            with pytest.raises(RuntimeError, match="without _enter"):
                p._exit()
            return outside, inside, nested_end, calls, seen
        finally:
            await c.close()
            await s.stop()
    outside, inside, nested_end, calls, seen = run(go())
    assert outside is False and inside is True
    assert nested_end == [] and calls == ["a", "b"] and seen == ["ZeroDivisionError"]


class _Recording(MemoryStore):
    """Records the order handlers reach the store, and can hold them there."""

    def __init__(self, medias, hold=None):
        super().__init__(medias)
        self.order = []
        self.hold = hold

    async def get_by_id(self, media_id):
        self.order.append(media_id)
        if self.hold is not None:
            await self.hold.wait()
        return await super().get_by_id(media_id)


def _service(src, store, **over):
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    return Service(cfg({"service": over} if over else None), source=src, store=store, http=RecordingHttpClient(),
                   logger=Logger(stream=MemoryStream()), serve_metrics=False)


def test_deliveries_at_a_low_rate_are_handed_over_without_waking_the_consumer():
    async def go():
        broker = await AmqpBroker().start()
        try:
            src = AmqpSource(broker.url, prefetch=20)
            store = _Recording([trello_media(f"m{i}") for i in range(30)])
            svc = _service(src, store)
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            await asyncio.sleep(0.05)
            for i in range(30):
                broker.publish(PROGRESS, progress_msg(f"m{i}", "QUEUED", i))
                await asyncio.sleep(0.005)  # one at a time
            for _ in range(200):
                if broker.stats(PROGRESS)["acked"] == 30:
                    break
                await asyncio.sleep(0.01)
            handed = (src.direct_batches, src.idle_wakeups)
            svc.request_stop()
            await task
            await svc.close()
            return handed, broker.stats(PROGRESS), store.order, src.direct
        finally:
            await broker.stop()
    (direct, wakeups), st, order, after = run(go())
    assert st["acked"] == 30 and st["unacked"] == 0
    assert direct >= 25 and wakeups <= 5, (direct, wakeups)  # the task slept through them
    assert order == [f"m{i}" for i in range(30)]
    assert after is None  # the service took its dispatcher back when it stopped


def test_a_full_prefetch_window_queues_the_rest_in_delivery_order():
    """prefetch 4 with held handlers: the hand-over takes what the window allows and the rest
    queues for the consumer's task. Deliveries arriving while the task works through the queue
    wait behind it, so handlers start in delivery order."""
    async def go():
        broker = await AmqpBroker().start()
        try:
            hold = asyncio.Event()
            src = AmqpSource(broker.url, prefetch=50)
            store = _Recording([trello_media(f"m{i}") for i in range(40)], hold=hold)
            svc = _service(src, store, prefetch=4)  # the service's window, smaller than the broker's
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            await asyncio.sleep(0.05)
            for i in range(20):
                broker.publish(PROGRESS, progress_msg(f"m{i}", "QUEUED", i))
            await asyncio.sleep(0.1)
            held = list(store.order)
            hold.set()
            for i in range(20, 40):
                broker.publish(PROGRESS, progress_msg(f"m{i}", "QUEUED", i))
                await asyncio.sleep(0.002)
            for _ in range(300):
                if broker.stats(PROGRESS)["acked"] == 40:
                    break
                await asyncio.sleep(0.01)
            svc.request_stop()
            await task
            await svc.close()
            return held, store.order, broker.stats(PROGRESS)
        finally:
            await broker.stop()
    held, order, st = run(go())
    # only the window's worth started (as on the task's own path, test_inflight_bounded_by_prefetch:
    # the delivery that finds the window full has started already)
    assert held == [f"m{i}" for i in range(len(held))] and 4 <= len(held) <= 5
    assert order == [f"m{i}" for i in range(40)] and st["acked"] == 40


def test_a_failing_hand_over_is_raised_from_run():
    """An error escaping the dispatch itself (not a handler's: those are the handlers' own
    business) ends the direct hand-over and surfaces from Service.run, as it would from the
    consumer's own loop."""
    async def go():
        broker = await AmqpBroker().start()
        try:
            src = AmqpSource(broker.url, prefetch=10)
            svc = _service(src, MemoryStore([trello_media("m1")]))
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            await asyncio.sleep(0.05)
            assert src.direct is not None

            def broken(batch):
                raise MemoryError("dispatch failed")
            src.direct = broken
            broker.publish(PROGRESS, progress_msg("m1", "QUEUED", 1))
            with pytest.raises(MemoryError, match="dispatch failed"):
                await asyncio.wait_for(task, 5)
            gone = src.direct
            await svc.close()
            return gone
        finally:
            await broker.stop()
    assert run(go()) is None
