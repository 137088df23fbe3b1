"""The H1Call's coroutine protocol at its edges (ops/csrc/py_h1call.cpp): the awaitable the H1
client's native path returns for every sink request (index.js:53,83,99,112).

tests/test_h1_fast.py compares the native path with the Python request loop on the wire; this file
drives an H1Call the ways a Task never does but a caller may: by iteration, by throw() / close()
in each state (before the first step, waiting for a reply, queued for a connection, delegated to
the Python loop), by dropping it unfinished, and reusing it after the end. Whatever happens, the
pool's accounting must come out whole: no connection left busy, none counted open that is closed.
Last, h1_setup / h1_fast refuse malformed arguments (the module's setup is restored afterwards).
"""
import asyncio
import gc

import pytest

from beholder_amd.ops import native
from beholder_amd.sinks import H1Client
from beholder_amd.sinks import h1 as h1mod

from test_h1_fast import OK, Raw

pytestmark = pytest.mark.skipif(h1mod._NATIVE_CALL is None or not H1Client().native_call,
                                reason="native I/O switched off (BEHOLDER_NATIVE_IO=0)")


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


def _server(target):
    if target.startswith("/slow"):
        return "hang"
    if target.startswith("/redirect"):
        return b"HTTP/1.1 302 Found\r\nLocation: /slow\r\nContent-Length: 0\r\n\r\n"
    return OK


async def _client(max_per_host=100):
    s = await Raw(_server).start()
    c = H1Client(timeout_s=5, max_per_host=max_per_host)
    base = f"http://127.0.0.1:{s.port}"
    await c.request("GET", base + "/warm")  # a warm pool: the native path takes the next requests
    return s, c, base


def _whole(c) -> tuple:
    """(connections busy, open count that matches the idle + busy ones)."""
    idle = sum(len(o.idle) for o in c._origins.values())
    return len(c._busy), sum(o.open for o in c._origins.values()) == idle + len(c._busy)


def test_iterating_a_call_drives_it_to_its_response():
    async def go():
        s, c, base = await _client()
        try:
            aw = c.request("GET", base + "/a")
            while True:
                try:
                    y = next(aw)  # the reply's future, then StopIteration(response)
                except StopIteration as e:
                    resp = e.value
                    break
                await y
            assert aw.native is True
            with pytest.raises(RuntimeError, match="reuse"):
                next(aw)
            return resp.status, _whole(c)
        finally:
            await c.close()
            await s.stop()
    assert run(go()) == (200, (0, True))


def test_throw_before_the_first_step_ends_the_call():
    async def go():
        s, c, base = await _client()
        try:
            aw = c.request("GET", base + "/a")
            with pytest.raises(ValueError, match="v"):
                aw.throw(ValueError, "v")
            aw2 = c.request("GET", base + "/a")
            e = KeyError("k")
            with pytest.raises(KeyError) as info:
                aw2.throw(KeyError, e)  # an instance of the class: raised as it is
            assert info.value is e
            aw4 = c.request("GET", base + "/a")
            with pytest.raises(ValueError):
                aw4.throw(ValueError)  # the class alone: instantiated with no arguments
            aw3 = c.request("GET", base + "/a")
            with pytest.raises(TypeError, match="deriving from BaseException"):
                aw3.throw(42)
            aw3.close()
            return s.connections, len(s.raw), _whole(c)
        finally:
            await c.close()
            await s.stop()
    assert run(go()) == (1, 1, (0, True))  # nothing was sent


def test_throw_while_waiting_for_the_reply_goes_to_the_request_loop():
    """An exception thrown in at the await (a Task's cancel, a wrapper's timeout) is the request
    loop's to handle (h1.py _exchange): the connection is dropped, the pool stays whole."""
    async def go():
        s, c, base = await _client()
        try:
            aw = c.request("GET", base + "/slow")
            assert aw.send(None) is not None and aw.native is True
            with pytest.raises(asyncio.CancelledError):
                aw.throw(asyncio.CancelledError())
            r = await c.request("GET", base + "/a")
            return r.status, _whole(c)
        finally:
            await c.close()
            await s.stop()
    assert run(go()) == (200, (0, True))


def test_calls_dropped_unfinished_release_their_connection():
    """A call garbage-collected while waiting for its reply, or while delegated to the Python loop
    (following a redirect), ends like a closed coroutine: its connection is dropped, not leaked."""
    async def go():
        s, c, base = await _client()
        try:
            aw = c.request("GET", base + "/slow")
            aw.send(None)
            del aw
            gc.collect()
            waiting = _whole(c)
            aw = c.request("GET", base + "/redirect")
            aw.send(None)  # sent natively, waiting for the reply
            await asyncio.sleep(0.1)  # the 302 has arrived
            aw.send(None)  # the Python request loop follows it: /slow sent, waiting (delegated)
            await asyncio.sleep(0.05)
            del aw
            gc.collect()
            await asyncio.sleep(0.05)
            r = await c.request("GET", base + "/a")
            return waiting, r.status, _whole(c)
        finally:
            await c.close()
            await s.stop()
    waiting, status, whole = run(go())
    assert waiting == (0, True) and status == 200 and whole == (0, True)


def test_queued_calls_thrown_closed_or_dropped_leave_the_queue():
    """With the only connection busy a request queues (ST_QUEUED). A foreign exception thrown in
    leaves the queue and propagates; close() and dropping the call leave it too; the connection
    then serves the next request."""
    async def go():
        s, c, base = await _client(max_per_host=1)
        try:
            hog = c.request("GET", base + "/slow")
            hog.send(None)  # holds the only connection
            q1 = c.request("GET", base + "/q1", timeout=5)
            q1.send(None)
            with pytest.raises(LookupError):
                q1.throw(LookupError("not the waiter's own"))
            q2 = c.request("GET", base + "/q2", timeout=5)
            q2.send(None)
            q2.close()
            q3 = c.request("GET", base + "/q3", timeout=5)
            q3.send(None)
            del q3
            gc.collect()
            waiters = sum(len([w for w in o.waiters if not w.done()]) for o in c._origins.values())
            hog.close()  # the hog's connection is dropped; the next request connects anew
            r = await c.request("GET", base + "/a")
            return waiters, r.status, _whole(c), [h.split(b" ")[1] for h in s.raw]
        finally:
            await c.close()
            await s.stop()
    waiters, status, whole, targets = run(go())
    assert waiters == 0 and status == 200 and whole == (0, True)
    assert b"/q1" not in targets and b"/q2" not in targets and b"/q3" not in targets


def test_close_in_each_state():
    async def go():
        s, c, base = await _client()
        try:
            fresh = c.request("GET", base + "/a")
            assert fresh.close() is None  # never started: nothing to undo
            delegated = c.request("GET", base + "/redirect")  # on the warm connection
            delegated.send(None)
            await asyncio.sleep(0.1)  # the 302 is in: the next step hands the call to the Python loop
            delegated.send(None)
            assert delegated.close() is None  # closes the Python loop's coroutine
            with pytest.raises(RuntimeError, match="reuse"):
                delegated.send(None)
            await c.request("GET", base + "/a")  # a connection again
            waiting = c.request("GET", base + "/slow")
            waiting.send(None)
            assert waiting.close() is None
            with pytest.raises(RuntimeError, match="reuse"):
                waiting.send(None)
            await asyncio.sleep(0.05)
            return _whole(c)
        finally:
            await c.close()
            await s.stop()
    assert run(go()) == (0, True)


@pytest.fixture
def restore_h1_setup():
    yield
    native.h1_setup(h1mod.H1Client, h1mod._Conn, h1mod._Origin, h1mod.HttpResponse)


def test_h1_setup_refuses_malformed_classes(restore_h1_setup):
    # the connection class's member names, as plain class attributes instead of __slots__ members
    NoSlots = type("NoSlots", (), {n: None for n in h1mod._Conn.__slots__})

    with pytest.raises(TypeError, match="client_cls must be a class"):
        native.h1_setup(1, h1mod._Conn, h1mod._Origin, h1mod.HttpResponse)
    with pytest.raises(TypeError, match="expected a class"):
        native.h1_setup(h1mod.H1Client, 1, h1mod._Origin, h1mod.HttpResponse)
    with pytest.raises(TypeError, match="is not a __slots__ member"):
        native.h1_setup(h1mod.H1Client, NoSlots, h1mod._Origin, h1mod.HttpResponse)

    class Dicty(h1mod.HttpResponse):  # slots inherited, but a __dict__ added
        pass
    with pytest.raises(TypeError, match="__slots__ only"):
        native.h1_setup(h1mod.H1Client, h1mod._Conn, h1mod._Origin, Dicty)
    native.h1_setup(h1mod.H1Client, h1mod._Conn, h1mod._Origin, h1mod.HttpResponse)

    async def go():  # and the restored setup serves requests natively again
        s, c, base = await _client()
        try:
            aw = c.request("GET", base + "/a")
            r = await aw
            return r.status, aw.native
        finally:
            await c.close()
            await s.stop()
    assert run(go()) == (200, True)


def test_h1_fast_refuses_malformed_arguments():
    with pytest.raises(TypeError, match="h1_fast"):
        native.h1_fast()
    with pytest.raises(TypeError, match="h1_fast"):
        native.h1_fast(1, 2, 3, 4, 5, 6, 7)
    assert native.h1_fast(object(), "GET", "http://127.0.0.1:1/") is None  # not a stock client


class _Step:
    """A non-coroutine awaitable: suspends once, then returns ``value``."""

    def __init__(self, value):
        self.value = value

    def __await__(self):
        yield None
        return self.value


def test_the_python_continuations_may_be_any_awaitable_and_fail_cleanly():
    """The call hands over to H1Client._request (a first request to an origin) or _resume (an
    error or a redirect at the await). _resume may return any awaitable; one that raises, or that
    returns something not awaitable, fails the call; _request must be a coroutine function."""
    async def go():
        s, c, base = await _client()
        out = []
        try:
            c._resume = lambda *a: _Step("resumed")
            out.append(await c.request("GET", base + "/redirect"))  # the 302: _resume's awaitable
            c._resume = lambda *a: 42
            with pytest.raises(TypeError, match="must return an awaitable"):
                await c.request("GET", base + "/redirect")

            def boom(*a):
                raise LookupError("resume failed")
            c._resume = boom
            with pytest.raises(LookupError, match="resume failed"):
                await c.request("GET", base + "/redirect")
            del c._resume
            cold = H1Client(timeout_s=5)  # no origin yet: the whole request is _request's
            cold._request = lambda *a: _Step("not a coroutine")
            with pytest.raises(TypeError, match="coroutine function"):
                await cold.request("GET", base + "/a")
            cold._request = boom
            with pytest.raises(LookupError):
                await cold.request("GET", base + "/a")
            await cold.close()
            await asyncio.sleep(0.05)
            return out, _whole(c)
        finally:
            await c.close()
            await s.stop()
    out, whole = run(go())
    assert out == ["resumed"] and whole[1]


def test_a_failing_release_is_reported_not_raised():
    """Cleanup paths (a call closed while waiting, a connection handed back) call the client's
    _release; if that raises, the error goes to sys.unraisablehook and the caller carries on."""
    import sys
    seen = []
    old = sys.unraisablehook
    sys.unraisablehook = lambda u: seen.append(type(u.exc_value).__name__)

    async def go():
        s, c, base = await _client()
        try:
            aw = c.request("GET", base + "/slow")
            aw.send(None)
            real = c._release

            def bad(*a):
                raise RuntimeError("release failed")
            c._release = bad
            assert aw.close() is None  # abandon: busy.discard + _release (raises: reported)
            c._release = real
            r = await c.request("GET", base + "/a")
            return r.status
        finally:
            await c.close()
            await s.stop()
    try:
        assert run(go()) == 200
    finally:
        sys.unraisablehook = old
    assert "RuntimeError" in seen


def test_deadline_from_a_loop_with_its_own_clock():
    """A request timeout is a deadline on the running loop's clock: loop.time() of a loop class
    that overrides it (the stock BaseEventLoop.time is read in C)."""
    class OwnClock(asyncio.SelectorEventLoop):
        def time(self):
            return super().time()

    async def go():
        s, c, base = await _client()
        try:
            with pytest.raises(h1mod.HttpError, match="ETIMEDOUT"):
                await c.request("GET", base + "/slow", timeout=0.1)
            return (await c.request("GET", base + "/a", timeout=5)).status
        finally:
            await c.close()
            await s.stop()
    loop = OwnClock()
    try:
        assert loop.run_until_complete(asyncio.wait_for(go(), 20)) == 200
    finally:
        loop.close()


@pytest.mark.parametrize("after", ["not_a_coroutine", "raises"])
def test_a_queued_call_resumed_into_a_failing_after_queue(after):
    """A queued request resumed by something other than a live connection (here: the slot the
    hog's dropped connection freed) continues in H1Client._after_queue; if that fails, the
    request fails with its error and the pool stays whole."""
    async def go():
        s, c, base = await _client(max_per_host=1)
        try:
            hog = c.request("GET", base + "/slow")
            hog.send(None)

            async def queued():
                return await c.request("GET", base + "/q", timeout=5)
            t = asyncio.ensure_future(queued())
            await asyncio.sleep(0.02)

            def boom(*a):
                raise LookupError("after_queue failed")
            c._after_queue = (lambda *a: 42) if after == "not_a_coroutine" else boom
            hog.close()  # the connection is dropped: its slot goes to the queued request
            res = (await asyncio.gather(t, return_exceptions=True))[0]
            del c._after_queue
            r = await c.request("GET", base + "/a")
            return type(res).__name__, str(res), r.status, _whole(c)
        finally:
            await c.close()
            await s.stop()
    name, text, status, whole = run(go())
    assert status == 200 and whole[1]
    if after == "not_a_coroutine":
        assert name == "TypeError" and "_after_queue must be a coroutine function" in text
    else:
        assert name == "LookupError"


def test_a_failing_sweeper_arm_hands_the_connection_back():
    """Sending on a pooled connection arms the idle sweeper when none runs (h1.py _arm); if that
    raises, the request fails with its error and the connection goes back to the pool accounting
    (dropped), not left busy."""
    async def go():
        s, c, base = await _client()
        try:
            c._sweeper = None  # no sweep running: the next native send arms one

            def boom(loop):
                raise LookupError("arm failed")
            c._arm = boom
            with pytest.raises(LookupError, match="arm failed"):
                await c.request("GET", base + "/a")
            del c._arm
            whole = _whole(c)
            r = await c.request("GET", base + "/a")
            return whole, r.status, _whole(c)
        finally:
            await c.close()
            await s.stop()
    whole, status, after = run(go())
    assert whole == (0, True) and status == 200 and after == (0, True)


def test_a_reply_whose_pool_bookkeeping_fails_drops_the_connection():
    """After the reply, the native path hands the connection back to the idle pool itself (h1.py
    _release with no waiter). If that bookkeeping raises (here the origin's waiter queue cannot
    be sized), the request fails with the error and the connection is dropped, not left busy.
    Dropping it wakes the origin's waiters, which meets the same broken queue: that second error
    goes to sys.unraisablehook."""
    import sys

    class BadLen(list):
        def __len__(self):
            raise LookupError("waiters broken")

    async def go():
        s, c, base = await _client()
        try:
            o = next(iter(c._origins.values()))
            good = o.waiters
            o.waiters = BadLen()
            with pytest.raises(LookupError, match="waiters broken"):
                await c.request("GET", base + "/a")
            o.waiters = good
            whole = _whole(c)
            r = await c.request("GET", base + "/a")
            return whole, r.status, _whole(c)
        finally:
            await c.close()
            await s.stop()
    seen = []
    old = sys.unraisablehook
    sys.unraisablehook = lambda u: seen.append(type(u.exc_value).__name__)
    try:
        whole, status, after = run(go())
    finally:
        sys.unraisablehook = old
    assert whole == (0, True) and status == 200 and after == (0, True)
    assert seen == ["LookupError"]
