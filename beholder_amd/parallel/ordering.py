"""Opt-in per-``mediaId`` serialisation (SURVEY.md §5 "race detection", quirk Q9).

The reference runs up to ``prefetch`` (100) handlers concurrently with no
per-media ordering (index.js:43,62,127): two progress ticks for the same
media can post their Trello comments out of order, and a status move can
race a comment. ``service.ordering: per_media`` routes deliveries through a
:class:`KeyedSerializer`: deliveries with the same key run strictly one after
another (in arrival order); different keys still run concurrently.
Default is ``none`` (reference behaviour).
"""
from __future__ import annotations

import asyncio
import collections
import functools
from typing import Any, Callable, Deque, Dict, Optional


class KeyedSerializer:
    """Serialise ``dispatch(item, on_finish) -> bool`` calls per ``key_fn(item)``.

    ``dispatch`` returns True when the item's work finished synchronously (eager
    completion; ``on_finish`` is then not called), or False and calls
    ``on_finish()`` exactly once later. Items whose key is ``None`` are
    dispatched immediately (unordered).
    """

    def __init__(self, dispatch: Callable[[Any, Optional[Callable[[], None]]], bool],
                 key_fn: Optional[Callable[[Any], Any]] = None):
        self._dispatch = dispatch
        self._key_fn = key_fn or (lambda item: None)
        self._chains: Dict[Any, Deque[Any]] = {}
        self._idle: Optional[asyncio.Event] = None
        self.max_chain = 0
        self.serialized = 0  # items that had to wait behind another with the same key

    @property
    def active_keys(self) -> int:
        return len(self._chains)

    def submit(self, item: Any) -> None:
        try:
            key = self._key_fn(item)
        except Exception:  # undecodable: let the handler see (and report) it
            key = None
        if key is None:
            self._dispatch(item, None)
            return
        q = self._chains.get(key)
        if q is not None:
            q.append(item)
            self.serialized += 1
            if len(q) > self.max_chain:
                self.max_chain = len(q)
            return
        self._chains[key] = collections.deque()
        self._run_chain(key, item)

    def _run_chain(self, key: Any, item: Any) -> None:
        # Trampoline: eager completions loop here instead of recursing.
        fin = None
        while True:
            if fin is None:
                fin = functools.partial(self._advance, key)
            if not self._dispatch(item, fin):
                return  # suspended: fin() resumes the chain
            q = self._chains.get(key)
            if not q:
                self._chains.pop(key, None)
                self._maybe_idle()
                return
            item = q.popleft()

    def _advance(self, key: Any) -> None:
        q = self._chains.get(key)
        if not q:
            self._chains.pop(key, None)
            self._maybe_idle()
            return
        self._run_chain(key, q.popleft())

    def _maybe_idle(self) -> None:
        if not self._chains and self._idle is not None:
            self._idle.set()

    async def drain(self, timeout: Optional[float] = None) -> bool:
        """Wait until every chain has finished. Returns False on timeout."""
        if not self._chains:
            return True
        self._idle = asyncio.Event()
        try:
            await asyncio.wait_for(self._idle.wait(), timeout)
            return True
        except asyncio.TimeoutError:
            return False
