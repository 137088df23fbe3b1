"""File-descriptor source: framed stdin / file / pipe / FIFO via the native reader.

The native :class:`~beholder_amd.ops.Ingest` owns a reader thread that reads
the fd in large chunks, splits frames and copies them into a bounded byte ring
without holding the GIL; this source pops whole batches of
:class:`~beholder_amd.ops.Delivery` objects for the event loop.

Waiting for data never blocks the loop and never involves another thread: a
non-blocking ``pop`` is tried first (the common case under load). When it
comes back empty the source *arms* the ring and parks on the ring's eventfd
(``loop.add_reader``); the reader thread's next push writes that fd once, and
the loop pops on readiness. One cross-thread hop per idle wake-up (reader →
loop), none under load (the ring is not armed while it has records).

Backpressure (BASELINE config 4): ``policy='block'`` makes the reader stall
when the ring is full (the kernel pipe then fills and the producer blocks);
``policy='drop_newest'`` drops and counts per topic
(``stats()['dropped_by_topic']``).

Ack semantics: there is no broker behind a file, so an ack just settles the
delivery (latency + counters). A delivery that is never acked (quirk Q1) is
reported through ``on_abandon`` — optionally appended to a dead-letter file
in the same frame format so it can be replayed.
"""
from __future__ import annotations

import asyncio
import os
import sys
import threading
from typing import Optional, Sequence

from ..ops import Ingest, Settler, frame
from .base import Source


def _grow_pipe(fd: int, size: int) -> None:
    """If ``fd`` is a pipe, ask for a ``size``-byte kernel buffer (Linux F_SETPIPE_SZ, capped by
    /proc/sys/fs/pipe-max-size). The default is 64 KiB. A bigger buffer means fewer reads by the
    reader thread, and fewer writer wake-ups, when events arrive faster than they are consumed."""
    import fcntl
    import stat
    try:
        if not stat.S_ISFIFO(os.fstat(fd).st_mode):
            return
        try:
            with open("/proc/sys/fs/pipe-max-size") as f:
                size = min(size, int(f.read()))
        except (OSError, ValueError):
            pass
        fcntl.fcntl(fd, getattr(fcntl, "F_SETPIPE_SZ", 1031), size)
    except OSError:
        pass  # not permitted / not Linux: keep the default buffer


class FdSource(Source):
    kind = "fd"

    def __init__(self, fd: Optional[int] = None, path: Optional[str] = None, *,
                 capacity_bytes: int = 64 << 20, capacity_events: int = 0, policy: str = "block",
                 batch: int = 512, chunk_bytes: int = 1 << 20, dead_letter: Optional[str] = None):
        if fd is None and path is None:
            fd = sys.stdin.fileno()
        self._fd = fd
        self._path = path
        self._own_fd = path is not None
        self.batch = batch
        self.chunk_bytes = chunk_bytes
        self.idle_wakeups = 0  # times the loop parked on the eventfd and was woken
        self._dl_path = dead_letter
        self._dl_file = None
        self._dl_lock = threading.Lock()
        self.abandoned_frames = 0
        self._settler = Settler(on_abandon=self._on_abandon)
        self.policy = policy
        self._ingest = Ingest(capacity_bytes=capacity_bytes, capacity_events=capacity_events,
                              policy=policy, settler=self._settler)
        self._started = False
        self._closed = False

    def describe(self) -> str:
        where = self._path if self._path is not None else ("stdin" if self._fd == 0 else f"fd {self._fd}")
        return f"{self.kind} {where} (framed; policy {self.policy})"

    # -- Source API -------------------------------------------------------------
    async def start(self, topics: Sequence[str] = ()) -> None:
        if self._started:
            return
        fd = self._fd
        if self._path is not None:
            fd = os.open(self._path, os.O_RDONLY)
            self._fd = fd
        _grow_pipe(fd, self.chunk_bytes)
        self._ingest.start_reader(fd, chunk_bytes=self.chunk_bytes, own_fd=self._own_fd)
        self._started = True

    async def batches(self):
        ing = self._ingest
        loop = asyncio.get_running_loop()
        n = self.batch
        pop, arm, clear = ing.pop, ing.arm, ing.clear_notify
        efd = ing.notify_fd
        waiter: list = [None]

        def on_ready():  # the selector saw the eventfd: drain it, wake the parked generator
            clear()
            w = waiter[0]
            if w is not None and not w.done():
                w.set_result(None)

        loop.add_reader(efd, on_ready)
        try:
            while True:
                got = pop(n, 0.0)
                if got is None:
                    return
                if got:
                    yield got
                    continue
                if not arm():  # a record / EOF arrived between the pop and arm(): pop again
                    continue
                w = waiter[0] = loop.create_future()
                await w
                waiter[0] = None
                self.idle_wakeups += 1
        finally:
            if not loop.is_closed():
                loop.remove_reader(efd)

    async def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        self._ingest.close()
        if self._dl_file is not None:
            self._dl_file.close()
            self._dl_file = None

    @property
    def settler(self) -> Settler:
        return self._settler

    @property
    def ingest(self) -> Ingest:
        return self._ingest

    def stats(self) -> dict:
        s = self._ingest.stats()
        s.update(self._settler.stats())
        s["abandoned_frames_written"] = self.abandoned_frames
        s["idle_wakeups"] = self.idle_wakeups
        return s

    def ready(self) -> bool:
        return self._started and not self._closed

    # -- dead letters -------------------------------------------------------------
    def _on_abandon(self, tag: int, topic_id: int, content: bytes) -> None:
        if self._dl_path is None:
            return
        with self._dl_lock:
            if self._closed:  # after close(): append and flush immediately
                with open(self._dl_path, "ab") as f:
                    f.write(frame(topic_id, content))
            else:
                if self._dl_file is None:
                    self._dl_file = open(self._dl_path, "ab")
                self._dl_file.write(frame(topic_id, content))
            self.abandoned_frames += 1


class BytesSource(FdSource):
    """Feeds an in-memory framed buffer through the same ring (tests / tools)."""

    kind = "bytes"

    def __init__(self, data: bytes, **kw):
        r, w = os.pipe()
        super().__init__(fd=r, **kw)
        self._own_fd = True
        self._data = data
        self._wfd = w
        self._writer: Optional[threading.Thread] = None

    async def start(self, topics: Sequence[str] = ()) -> None:
        await super().start(topics)

        def pump():
            try:
                mv = memoryview(self._data)
                while mv:
                    n = os.write(self._wfd, mv[:1 << 20])
                    mv = mv[n:]
            except OSError:
                pass
            finally:
                os.close(self._wfd)

        self._writer = threading.Thread(target=pump, name="bytes-source", daemon=True)
        self._writer.start()

    async def close(self) -> None:
        await super().close()
        if self._writer is not None:
            self._writer.join(timeout=5)



class NdjsonSource(FdSource):
    """Line-oriented input: one JSON record per line (see :mod:`.framing` for the record shape).

    A reader thread parses lines and pushes ``(topic_id, payload)`` into the same native ring
    the binary reader uses, so everything downstream (batches, deliveries, acks, backpressure)
    is identical. Malformed lines are counted and logged to stderr, not fatal.
    """

    kind = "ndjson"

    def __init__(self, fd: Optional[int] = None, path: Optional[str] = None, **kw):
        super().__init__(fd=fd, path=path, **kw)
        self.bad_lines = 0
        self._thread: Optional[threading.Thread] = None

    async def start(self, topics: Sequence[str] = ()) -> None:
        if self._started:
            return
        fd = self._fd
        if self._path is not None:
            fd = os.open(self._path, os.O_RDONLY)
            self._fd = fd
        from .framing import ndjson_line_to_frame

        def run():
            try:
                with os.fdopen(fd, "r", encoding="utf-8", closefd=self._own_fd) as f:
                    for line in f:
                        line = line.strip()
                        if not line:
                            continue
                        try:
                            tid, payload = ndjson_line_to_frame(line)
                        except (ValueError, KeyError, TypeError) as e:
                            self.bad_lines += 1
                            print(f"beholder: skipping malformed ndjson line: {e}", file=sys.stderr)
                            continue
                        try:
                            self._ingest.push(tid, payload)
                        except RuntimeError:  # closed
                            return
            finally:
                self._ingest.set_eof()

        self._thread = threading.Thread(target=run, daemon=True, name="ndjson-reader")
        self._thread.start()
        self._started = True

    def stats(self) -> dict:
        s = super().stats()
        s["bad_lines"] = self.bad_lines
        return s
