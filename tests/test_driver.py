"""Native Task-free coroutine driver (`ops/csrc/py_driver.cpp`) used for handlers that
suspend on I/O (index.js:62,127 handlers awaiting the DB / HTTP)."""
import asyncio
import gc
import weakref

import pytest

from beholder_amd.ops import Driver


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


def drive(coro_fn, *args, payload=None):
    """Starts coro like dispatch_batch does and returns (driver, outcome-future)."""
    loop = asyncio.get_running_loop()
    out = loop.create_future()
    coro = coro_fn(*args)
    first = coro.send(None)
    d = Driver(coro, lambda drv, exc: out.set_result((drv, exc)), payload)
    d.start(first)
    return d, out


def test_results_exceptions_and_payload():
    async def h(x):
        await asyncio.sleep(0)  # bare yield: rescheduled through call_soon
        await asyncio.sleep(0.001)
        f = asyncio.get_running_loop().create_future()
        asyncio.get_running_loop().call_soon(f.set_result, x * 2)
        v = await f
        if x == 3:
            raise ValueError(f"boom {v}")
        return v

    async def go():
        outs = [drive(h, x, payload=f"p{x}")[1] for x in range(5)]
        res = await asyncio.gather(*outs)
        return [(type(e).__name__ if e else None, str(e) if e else None) for _, e in res], res[0][0]
    res, drv = run(go())
    assert res[3] == ("ValueError", "boom 6") and [r for i, r in enumerate(res) if i != 3] == [(None, None)] * 4
    assert drv.done() and drv.steps >= 3 and drv.payload is None  # payload released on completion


def test_awaited_exception_is_thrown_into_the_coroutine():
    async def h():
        f = asyncio.get_running_loop().create_future()
        asyncio.get_running_loop().call_soon(f.set_exception, KeyError("k"))
        try:
            await f
        except KeyError as e:
            return f"caught {e}"

    async def go():
        d, out = drive(h)
        return await out
    drv, exc = run(go())
    assert exc is None


def test_cancel_while_waiting_and_before_rearm():
    async def hang():
        await asyncio.sleep(10)

    async def swallow():
        try:
            await asyncio.sleep(10)
        except asyncio.CancelledError:
            return "cleaned up"

    async def yields_then_waits():
        await asyncio.sleep(0)
        await asyncio.sleep(10)

    async def go():
        d1, o1 = drive(hang)
        d2, o2 = drive(swallow)
        d3, o3 = drive(yields_then_waits)
        assert d3.cancel()  # pending on a bare-yield reschedule: cancelled at the next await
        await asyncio.sleep(0.01)
        assert d1.cancel() and d2.cancel()
        (a, ea), (b, eb), (c, ec) = await asyncio.gather(o1, o2, o3)
        return ea, a.cancelled, eb, ec, d1.cancel()
    ea, cancelled, eb, ec, again = run(go())
    assert isinstance(ea, asyncio.CancelledError) and cancelled
    assert eb is None  # the coroutine handled the cancellation and returned
    assert isinstance(ec, asyncio.CancelledError)
    assert again is False  # cancelling a finished driver is a no-op


def test_non_future_yield_raises_runtime_error_inside_the_coroutine():
    import types

    @types.coroutine
    def bad():
        yield 42

    async def h():
        try:
            await bad()
        except RuntimeError as e:
            return str(e)

    async def go():
        loop = asyncio.get_running_loop()
        out = loop.create_future()
        coro = h()
        first = coro.send(None)  # 42 reaches the dispatcher
        Driver(coro, lambda drv, exc: out.set_result(exc)).start(first)
        return await out
    assert run(go()) is None


def test_keyboard_interrupt_reaches_the_loop_after_on_done():
    seen = []

    async def h():
        await asyncio.sleep(0)
        raise KeyboardInterrupt

    async def go():
        coro = h()
        Driver(coro, lambda drv, exc: seen.append(type(exc).__name__)).start(coro.send(None))
        await asyncio.sleep(0.05)
    with pytest.raises(KeyboardInterrupt):
        asyncio.run(go())
    assert seen == ["KeyboardInterrupt"]


def test_start_twice_and_bad_args():
    async def go():
        async def h():
            await asyncio.sleep(0.001)
        coro = h()
        d = Driver(coro, lambda drv, exc: None)
        d.start(coro.send(None))
        with pytest.raises(RuntimeError):
            d.start(None)
        with pytest.raises(TypeError):
            Driver(coro, "not callable")
        await asyncio.sleep(0.01)
    run(go())


def test_no_reference_leaks():
    class Payload:
        pass

    async def h(p):
        await asyncio.sleep(0.001)

    async def go():
        p = Payload()
        ref = weakref.ref(p)
        d, out = drive(h, p, payload=p)
        del p
        await out
        dref = weakref.ref(d) if hasattr(d, "__weakref__") else None
        del d, out
        return ref, dref
    ref, _ = run(go())
    gc.collect()
    assert ref() is None


# ---------------------------------------------------------------- IOFuture ---

def test_iofuture_is_an_asyncio_future_for_tasks_gather_and_wait_for():
    from beholder_amd.ops import native
    IOFuture = native.IOFuture

    async def go():
        loop = asyncio.get_running_loop()
        f = IOFuture(loop)
        assert asyncio.isfuture(f) and not f.done() and f.get_loop() is loop
        with pytest.raises(asyncio.InvalidStateError):
            f.result()
        loop.call_soon(f.set_result, 42)
        assert await f == 42 and f.done()
        e = IOFuture()
        loop.call_soon(e.set_exception, KeyError("k"))
        with pytest.raises(KeyError):
            await e
        fs = [IOFuture() for _ in range(3)]
        for i, x in enumerate(fs):
            loop.call_soon(x.resolve, i)  # outside a Driver, resolve behaves like set_result
        assert await asyncio.gather(*fs) == [0, 1, 2]
        slow = IOFuture()
        with pytest.raises(asyncio.TimeoutError):
            await asyncio.wait_for(slow, 0.01)
        assert slow.cancelled()
        with pytest.raises(asyncio.CancelledError):
            slow.result()
        late = []
        done = IOFuture()
        done.set_result(1)
        done.add_done_callback(lambda fut: late.append(fut.result()))  # already done: scheduled
        assert late == []
        await asyncio.sleep(0)
        cb = late.append
        g = IOFuture()
        g.add_done_callback(cb)
        g.add_done_callback(cb)
        assert g.remove_done_callback(cb) == 2
        with pytest.raises(asyncio.InvalidStateError):
            done.set_result(2)
        return late
    assert run(go()) == [1]


def test_iofuture_resolve_resumes_a_driver_synchronously():
    from beholder_amd.ops import native
    order = []

    async def handler(fut):
        v = await fut
        order.append(("resumed", v))

    async def go():
        f = native.IOFuture()
        coro = handler(f)
        Driver(coro, lambda drv, exc: order.append(("done", exc))).start(coro.send(None))
        f.resolve("row")
        order.append("after resolve")
        g = native.IOFuture()
        coro = handler(g)
        Driver(coro, lambda drv, exc: order.append(("done", type(exc).__name__))).start(coro.send(None))
        g.reject(ValueError("bad"))
        order.append("after reject")
    run(go())
    assert order == [("resumed", "row"), ("done", None), "after resolve", ("done", "ValueError"), "after reject"]


def test_iofuture_sync_callback_errors_go_to_the_loop_handler():
    from beholder_amd.ops import native
    seen = []

    async def handler(fut):
        await fut

    async def go():
        loop = asyncio.get_running_loop()
        loop.set_exception_handler(lambda lp, ctx: seen.append(type(ctx.get("exception")).__name__))
        f = native.IOFuture()
        coro = handler(f)

        def on_done(drv, exc):
            raise RuntimeError("on_done failed")
        Driver(coro, on_done).start(coro.send(None))
        f.resolve(1)  # must not raise into the protocol callback that resolves it
    run(go())
    assert seen == ["RuntimeError"]


# ---- Window: the native in-flight set (the prefetch window) -------------------------
def test_window_suspend_full_flag_errors_and_wakes():
    from beholder_amd.ops import Window
    errors, wakes = [], []

    async def h(fut, fail=False):
        await fut
        if fail:
            raise ValueError("boom")

    async def go():
        loop = asyncio.get_running_loop()
        w = Window(3, lambda p, e: errors.append((p, str(e))), lambda: wakes.append(len(w)))
        futs = [loop.create_future() for _ in range(4)]
        full = []
        for i, f in enumerate(futs[:3]):
            c = h(f, fail=(i == 1))
            full.append(w.suspend(f"d{i}", c, c.send(None)))
        assert full == [False, False, True] and len(w) == 3 and w.limit == 3
        assert sorted(d.payload for d in w) == ["d0", "d1", "d2"]  # iteration is a snapshot
        futs[1].set_result(None)
        await asyncio.sleep(0)
        assert errors == [("d1", "boom")] and wakes == [2]  # full -> not full
        c = h(futs[3])
        assert w.suspend("d3", c, c.send(None)) is True
        futs[0].set_result(None)
        futs[2].set_result(None)
        await asyncio.sleep(0)
        assert wakes == [2, 2]  # one more full -> not full transition, 1 left: no wake
        futs[3].set_result(None)
        await asyncio.sleep(0)
        assert len(w) == 0 and wakes == [2, 2, 0]  # emptied
        assert w.stats()["suspended"] == 4
        return w

    w = run(go())
    assert not w


def test_window_cancelled_drivers_are_not_errors_and_tracked_drivers_release():
    from beholder_amd.ops import Window
    errors, wakes = [], []

    async def h(fut):
        await fut

    async def go():
        loop = asyncio.get_running_loop()
        w = Window(10, lambda p, e: errors.append(p), lambda: wakes.append(len(w)))
        f = loop.create_future()
        c = h(f)
        w.suspend("a", c, c.send(None))
        (drv,) = list(w)
        drv.cancel()
        await asyncio.sleep(0)
        assert len(w) == 0 and errors == [] and drv.cancelled  # CancelledError is not a handler error
        # a Driver with its own on_done, counted against the window via track/release
        f2 = loop.create_future()
        c2 = h(f2)
        done = []
        d2 = Driver(c2, lambda d, e: (w.release(d, e), done.append(e)), "b")
        w.track(d2)
        d2.start(c2.send(None))
        assert len(w) == 1
        f2.set_exception(RuntimeError("x"))
        await asyncio.sleep(0)
        assert len(w) == 0 and errors == ["b"] and isinstance(done[0], RuntimeError)

    run(go())
    with pytest.raises(ValueError):
        __import__("beholder_amd.ops", fromlist=["Window"]).Window(0)


def test_window_drops_finished_drivers():
    from beholder_amd.ops import Window

    async def h(fut):
        await fut

    async def go():
        loop = asyncio.get_running_loop()
        w = Window(100)
        for _ in range(50):
            f = loop.create_future()
            c = h(f)
            w.suspend(None, c, c.send(None))
            f.set_result(1)
        await asyncio.sleep(0)
        assert len(w) == 0

    run(go())
    gc.collect()
    assert not [o for o in gc.get_objects() if type(o).__name__ == "Driver"]
