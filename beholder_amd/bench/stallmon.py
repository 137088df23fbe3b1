"""Stall monitor for bench processes: event-loop lag and GC pauses as timed intervals.

Every process of the production-shaped bench (the consumer, and the AMQP / Postgres / HTTP fakes
it talks to) runs one. It records

* **loop lag**: a task sleeps ``period_s`` and measures how late it wakes. A wake-up later than
  ``threshold_us`` (1 ms: longer than any one loop iteration of a healthy process at saturation,
  where the consumer's p50 receive->ack is ~0.4 ms with 100 deliveries in flight) is a *stall* interval ``[due, woke]`` during which the loop ran nothing else
  (a long callback, a GC pass, the process descheduled by the kernel or by the cgroup quota);
* **GC pauses** (``gc.callbacks``), as intervals too.

All intervals are CLOCK_MONOTONIC, which every process on the host shares, so the consumer's
slow deliveries can be matched against the stalls of *each* process (:func:`attribute`): a
slow delivery that overlaps a Postgres-fake stall waited on a PG reply, one that overlaps a
consumer stall waited on its own loop. This is the attribution the bench line reports for the
slowest 0.1% of ``tcp_e2e`` / ``tls_e2e`` deliveries.
"""
from __future__ import annotations

import asyncio
import gc
import json
import time
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

Interval = Tuple[int, int]


class StallMonitor:
    """``work``: a cheap callable returning a running count of the process's work (the consumer's
    settled deliveries). Each loop stall then records how much work the loop did inside it
    (``stall_work``: [stall us, work done]): a stall that settled hundreds of deliveries was one
    long callback working through a batch, one that settled none was the loop blocked or the
    process descheduled."""

    def __init__(self, period_s: float = 0.001, threshold_us: float = 1000.0, max_events: int = 20000,
                 work: Optional[Callable[[], int]] = None):
        self.period_ns = int(period_s * 1e9)
        self.threshold_ns = int(threshold_us * 1e3)
        self.max_events = max_events
        self.work = work
        self.stall_work: List[Tuple[float, int]] = []
        self.loop_stalls: List[Interval] = []
        self.gc_pauses: List[Interval] = []
        # every measured lateness, in a fixed-size native histogram: a list of one int per tick
        # grew the consumer's RSS by ~2 MB a minute (1,000 ticks/s), which a paced soak billed to
        # the service as a leak (scripts/paced_soak.py, profiles/box_r6_psoak/)
        from ..ops import Histogram
        self.lags_ns = Histogram()
        self.gc_pause_ns: List[int] = []
        self._task: Optional[asyncio.Task] = None
        self._gc_t0 = 0
        self.dropped = 0

    # -- gc.callbacks ------------------------------------------------------------------------
    def _gc_cb(self, phase, info):
        if phase == "start":
            self._gc_t0 = time.monotonic_ns()
        elif self._gc_t0:
            t1 = time.monotonic_ns()
            d = t1 - self._gc_t0
            self.gc_pause_ns.append(d)
            if d >= self.threshold_ns:
                self._add(self.gc_pauses, (self._gc_t0, t1))
            self._gc_t0 = 0

    def _add(self, where: list, iv: Interval) -> None:
        if len(self.loop_stalls) + len(self.gc_pauses) < self.max_events:
            where.append(iv)
        else:
            self.dropped += 1

    async def _run(self) -> None:
        period = self.period_ns / 1e9
        mono = time.monotonic_ns
        work = self.work
        while True:
            due = mono() + self.period_ns
            w0 = work() if work is not None else 0
            await asyncio.sleep(period)
            now = mono()
            lag = now - due
            if lag < 0:
                lag = 0
            self.lags_ns.record(lag)
            if lag >= self.threshold_ns:
                self._add(self.loop_stalls, (due, now))
                if work is not None and len(self.stall_work) < 1000:
                    self.stall_work.append((round(lag / 1e3, 1), work() - w0))

    def start(self, loop: Optional[asyncio.AbstractEventLoop] = None) -> "StallMonitor":
        loop = loop or asyncio.get_event_loop()
        gc.callbacks.append(self._gc_cb)
        self._task = loop.create_task(self._run())
        return self

    def reset(self) -> None:
        """Forget what was recorded so far (the end of a warm-up)."""
        self.loop_stalls.clear()
        self.gc_pauses.clear()
        self.lags_ns.reset()
        self.gc_pause_ns.clear()
        self.stall_work.clear()
        self.dropped = 0

    def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            self._task = None
        try:
            gc.callbacks.remove(self._gc_cb)
        except ValueError:
            pass

    def summary(self) -> Dict[str, object]:
        lags = self.lags_ns
        return {
            "loop_lag_p99_us": round(lags.percentile(99) / 1e3, 1) if lags.count else None,
            "loop_lag_p999_us": round(lags.percentile(99.9) / 1e3, 1) if lags.count else None,
            "loop_lag_max_us": round(lags.max / 1e3, 1) if lags.count else None,
            "loop_stalls": len(self.loop_stalls),
            "loop_stalled_ms": round(sum(b - a for a, b in self.loop_stalls) / 1e6, 2),
            "gc_pauses": len(self.gc_pause_ns),
            "gc_max_pause_us": round(max(self.gc_pause_ns) / 1e3, 1) if self.gc_pause_ns else None,
            "gc_stalls": len(self.gc_pauses),
            # the longest stalls with the work done inside each ([stall us, work], see the class)
            "stall_work": sorted(self.stall_work, reverse=True)[:5] if self.work is not None else None,
        }

    def dump(self) -> Dict[str, object]:
        """Summary plus the stall intervals (for :func:`attribute` in another process)."""
        return {**self.summary(), "stall_intervals": [list(x) for x in self.loop_stalls + self.gc_pauses]}

    def dump_line(self, name: str) -> str:
        return "STALLS " + json.dumps({"name": name, **self.dump()}, separators=(",", ":"))


def fake_monitor() -> StallMonitor:
    """For a bench fake, once its state is built and before READY: the setup's objects move out of
    the collected generations (``gc.freeze``) so the young-generation passes a busy fake still runs
    stay short, and a :class:`StallMonitor` starts on the running loop. The real servers these
    fakes stand in for (RabbitMQ, Postgres, api.trello.com) have no Python GC; a fake's own pauses
    must not be billed to the consumer, and what remains is measured, not guessed."""
    gc.collect()
    gc.freeze()
    return StallMonitor().start(asyncio.get_running_loop())


def parse_stall_lines(text: str) -> List[dict]:
    out = []
    for ln in text.split("\n"):
        if ln.startswith("STALLS "):
            try:
                out.append(json.loads(ln[7:]))
            except ValueError:
                pass
    return out


def _overlap(a0: int, a1: int, ivs: Sequence[Interval], starts: Sequence[int], longest: Optional[int] = None) -> int:
    """Total overlap of [a0, a1) with the sorted, possibly overlapping intervals ``ivs``, whose
    longest is ``longest`` ns: no interval that starts earlier than ``a0 - longest`` can still
    run at ``a0``, so the scan starts there (a stall that began long before the delivery and is
    still going is the one the attribution most needs to see: ADVICE r4)."""
    import bisect
    if longest is None:
        longest = max((e - s for s, e in ivs), default=0)
    i = bisect.bisect_left(starts, a0 - max(longest, 0))
    covered = 0
    cur0 = cur1 = None
    for s, e in ivs[i:]:
        if s >= a1:
            break
        s, e = max(s, a0), min(e, a1)
        if e <= s:
            continue
        if cur1 is None or s > cur1:
            if cur1 is not None:
                covered += cur1 - cur0
            cur0, cur1 = s, e
        else:
            cur1 = max(cur1, e)
    if cur1 is not None:
        covered += cur1 - cur0
    return covered


def attribute(slow: Iterable[Tuple[int, int, int]], sources: Dict[str, Iterable[Interval]],
              min_share: float = 0.25) -> Dict[str, object]:
    """Blames each slow delivery ``(recv, start, settle)`` on the process whose stalls cover the
    largest part of its ``[start, settle]`` window, if that part is at least ``min_share`` of the
    window; otherwise on ``"none"`` (no process stalled: the time went to ordinary queueing
    behind the other deliveries in flight). Returns counts per source and the share of the slow
    deliveries' total time each source's stalls cover."""
    prepared = {}
    for name, ivs in sources.items():
        iv = sorted((int(a), int(b)) for a, b in ivs)
        prepared[name] = (iv, [a for a, _ in iv], max((b - a for a, b in iv), default=0))
    counts: Dict[str, int] = {name: 0 for name in prepared}
    counts["none"] = 0
    covered_ns: Dict[str, int] = {name: 0 for name in prepared}
    total_ns = 0
    n = 0
    for _recv, start, settle in slow:
        n += 1
        dur = max(1, settle - start)
        total_ns += dur
        best, best_ns = "none", 0
        for name, (iv, starts, longest) in prepared.items():
            c = _overlap(start, settle, iv, starts, longest)
            covered_ns[name] += c
            if c > best_ns:
                best, best_ns = name, c
        if best_ns < min_share * dur:
            best = "none"
        counts[best] += 1
    return {"deliveries": n, "blamed": counts,
            "time_share": {k: round(v / total_ns, 3) if total_ns else 0.0 for k, v in covered_ns.items()}}
