"""A lighter asyncio.Event for the consumer's hot waits.

The dispatch loop waits for a free prefetch slot (service.py ``_wait_slots``) and for the next
AMQP batch (transport/amqp/source.py ``batches``) many thousand times a second under load.
``asyncio.Event`` keeps a deque of waiter futures and goes through its Python ``wait`` /
``set`` bodies each time; :class:`Signal` latches a flag and shares one future between its
waiters, which is all these single-consumer waits need.
"""
from __future__ import annotations

import asyncio
from typing import Optional


class Signal:
    """``set()`` / ``clear()`` / ``is_set()`` / ``await wait()`` with asyncio.Event's meaning:
    ``wait()`` returns at once while set, else when ``set()`` is next called. Every waiter of
    one wait shares its future, so a waiter cancelled mid-wait cancels the others too: this is
    for one waiting task at a time (the dispatch loop), not a general asyncio.Event."""

    __slots__ = ("_flag", "_fut")

    def __init__(self) -> None:
        self._flag = False
        self._fut: Optional[asyncio.Future] = None

    def is_set(self) -> bool:
        return self._flag

    def set(self) -> None:
        self._flag = True
        f = self._fut
        if f is not None:
            self._fut = None
            if not f.done():
                f.set_result(None)

    def clear(self) -> None:
        self._flag = False

    async def wait(self) -> bool:
        if self._flag:
            return True
        f = self._fut
        if f is None or f.done():
            f = self._fut = asyncio.get_running_loop().create_future()
        await f
        return True
