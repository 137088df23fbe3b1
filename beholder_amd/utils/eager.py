"""Eager coroutine execution for the dispatch hot path.

Every delivery runs an ``async`` handler (index.js:62,127). With an in-memory
store and buffered sinks most handlers never actually suspend, and creating an
``asyncio.Task`` per message (~10 µs) would dominate the cost. :func:`run_eager`
drives the coroutine synchronously until it either finishes — no task, no
loop round-trip — or hits its first real suspension point, at which point the
*already-started* coroutine is handed to a Task that continues from there.
(Python 3.12's ``eager_task_factory`` does the same; this is for 3.10.)
"""
from __future__ import annotations

import asyncio
import types
from typing import Any, Callable, Coroutine, Optional

DONE = 0
ERROR = 1
PENDING = 2


@types.coroutine
def _continue(coro, first_yield):
    """Generator-based coroutine resuming ``coro`` after it yielded ``first_yield``."""
    try:
        yield first_yield
    except BaseException as exc:  # cancellation / throw at the first suspension point
        try:
            nxt = coro.throw(exc)
        except StopIteration as stop:
            return stop.value
        return (yield from _continue(coro, nxt))
    # The Task resumes us with send(None), exactly what `coro` expects from
    # the future it awaited (Future.__await__ returns self.result()).
    return (yield from coro)


async def _drive(coro, first_yield):
    return await _continue(coro, first_yield)


def run_eager(coro: Coroutine, loop: Optional[asyncio.AbstractEventLoop] = None):
    """Run ``coro`` eagerly. Returns ``(DONE, value)``, ``(ERROR, exc)`` or ``(PENDING, task)``."""
    try:
        fut = coro.send(None)
    except StopIteration as stop:
        return DONE, stop.value
    except BaseException as exc:  # noqa: BLE001 — handler errors are data here
        return ERROR, exc
    loop = loop or asyncio.get_running_loop()
    return PENDING, loop.create_task(_drive(coro, fut))


def spawn_eager(coro: Coroutine, on_done: Callable[[int, Any], None],
                loop: Optional[asyncio.AbstractEventLoop] = None) -> Optional[asyncio.Task]:
    """Run eagerly and report the outcome via ``on_done(kind, value)`` (DONE/ERROR).

    Returns the Task if the coroutine suspended, else ``None``.
    """
    kind, val = run_eager(coro, loop)
    if kind != PENDING:
        on_done(kind, val)
        return None
    task: asyncio.Task = val

    def _cb(t: asyncio.Task) -> None:
        if t.cancelled():
            on_done(ERROR, asyncio.CancelledError())
            return
        exc = t.exception()
        if exc is not None:
            on_done(ERROR, exc)
        else:
            on_done(DONE, t.result())

    task.add_done_callback(_cb)
    return task
