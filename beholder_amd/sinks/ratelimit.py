"""Outbound rate limiting and 429 retries for the sinks (opt-in; off = reference behaviour).

The reference comments on a Trello card for every progress tick of a Trello-created media
(index.js:142-147) and sends requests as fast as events arrive. Trello allows 100 requests per
10 s per token (300 per key). Above that it answers 429. The `trello` npm client resolves on
any status (sinks/trello.py), so the reference silently loses those comments, and it still
counts them in `beholder_trello_comments` (index.js:57). Both behaviours stay the default here.
`service.sinks.<sink>` can turn on:

* ``rate_limit: {requests: N, per_s: T}``: a token bucket. A request that finds a token goes
  out at once (no suspension, so the handler's fast path stays synchronous). Otherwise it waits
  its turn in FIFO order. Waiting handlers hold prefetch slots, so the broker stops delivering
  and the backlog stays in the queue, not in memory.
* ``retry_429: N``: re-send a 429 answer up to N times, after ``Retry-After`` seconds (or an
  exponential backoff from ``retry_base_s``, capped at ``retry_max_s``).
"""
from __future__ import annotations

import asyncio
import collections
import time
from typing import Any, Callable, Deque, Mapping, Optional


class TokenBucket:
    """``capacity`` tokens, refilled continuously at ``capacity / per_s`` tokens per second."""

    def __init__(self, requests: float, per_s: float, clock: Callable[[], float] = time.monotonic):
        if requests <= 0 or per_s <= 0:
            raise ValueError("rate_limit needs requests > 0 and per_s > 0")
        self.capacity = float(requests)
        self.rate = float(requests) / float(per_s)
        self.tokens = self.capacity
        self.clock = clock
        self.last = clock()
        self._waiters: Deque[asyncio.Future] = collections.deque()
        self._timer: Optional[asyncio.TimerHandle] = None
        self.granted = 0
        self.delayed = 0
        self.waited_s = 0.0

    def _refill(self) -> None:
        now = self.clock()
        if now > self.last:
            self.tokens = min(self.capacity, self.tokens + (now - self.last) * self.rate)
            self.last = now

    def try_acquire(self) -> bool:
        """Take a token without waiting (only when nobody is queued: FIFO)."""
        if self._waiters:
            return False
        self._refill()
        if self.tokens >= 1.0:
            self.tokens -= 1.0
            self.granted += 1
            return True
        return False

    async def acquire(self) -> None:
        if self.try_acquire():
            return
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._waiters.append(fut)
        self.delayed += 1
        t0 = self.clock()
        self._arm(loop)
        try:
            await fut
        except BaseException:
            if fut in self._waiters:
                self._waiters.remove(fut)
            elif fut.done() and not fut.cancelled():
                self.tokens += 1.0  # granted just as we were cancelled: give it back
            raise
        finally:
            self.waited_s += self.clock() - t0

    def _arm(self, loop) -> None:
        if self._timer is not None or not self._waiters:
            return
        self._refill()
        delay = max(0.0, (1.0 - self.tokens) / self.rate)
        self._timer = loop.call_later(delay, self._wake, loop)

    def _wake(self, loop) -> None:
        self._timer = None
        self._refill()
        while self._waiters and self.tokens >= 1.0:
            fut = self._waiters.popleft()
            if fut.done():
                continue
            self.tokens -= 1.0
            self.granted += 1
            fut.set_result(None)
        self._arm(loop)

    def stats(self) -> dict:
        return {"granted": self.granted, "delayed": self.delayed, "waiting": len(self._waiters),
                "waited_s": round(self.waited_s, 6)}


class RetryPolicy:
    """Re-send on HTTP 429: ``Retry-After`` (seconds) when present, else exponential backoff."""

    def __init__(self, retries: int, base_s: float = 1.0, max_s: float = 30.0):
        self.retries = int(retries)
        self.base_s = float(base_s)
        self.max_s = float(max_s)
        self.retried = 0

    def delay(self, attempt: int, retry_after: Optional[str]) -> float:
        if retry_after:
            try:
                return min(self.max_s, max(0.0, float(retry_after)))
            except ValueError:
                pass
        return min(self.max_s, self.base_s * (2 ** attempt))


def from_config(section: Optional[Mapping[str, Any]]):
    """``(TokenBucket or None, RetryPolicy or None)`` for one sink's ``service.sinks.<name>``."""
    section = dict(section or {})
    rl = section.get("rate_limit")
    bucket = TokenBucket(float(rl["requests"]), float(rl["per_s"])) if rl else None
    n = int(section.get("retry_429") or 0)
    retry = RetryPolicy(n, float(section.get("retry_base_s", 1.0)), float(section.get("retry_max_s", 30.0))) \
        if n > 0 else None
    return bucket, retry


async def guarded(limiter: Optional[TokenBucket], retry: Optional[RetryPolicy], send):
    """``await send()`` (an HttpResponse) behind the bucket, re-sent on 429 per ``retry``."""
    attempt = 0
    while True:
        if limiter is not None and not limiter.try_acquire():
            await limiter.acquire()
        r = await send()
        if retry is None or r.status != 429 or attempt >= retry.retries:
            return r
        await asyncio.sleep(retry.delay(attempt, r.headers.get("retry-after")))
        attempt += 1
        retry.retried += 1
