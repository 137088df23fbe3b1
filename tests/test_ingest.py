"""Native ingest runtime: framing, ring wrap-around, backpressure, reader thread, EOF, errors."""
import os
import threading
import time

import pytest

from beholder_amd.ops import Ingest, frame, frames
from beholder_amd.transport.framing import iter_frames, ndjson_to_frames


def drain(ing, timeout=2.0):
    out = []
    deadline = time.time() + timeout
    while time.time() < deadline:
        got = ing.pop(1000, 0.05)
        if got is None:
            return out
        out.extend(got)
    raise AssertionError("ingest did not drain")


def test_frame_format():
    assert frame(2, b"abc") == b"\x04\x00\x00\x00\x02abc"
    assert list(iter_frames(frames([(1, b""), (2, b"xy")]))) == [(1, b""), (2, b"xy")]


def test_feed_split_at_every_byte():
    data = frames([(1, b"hello"), (2, b""), (1, b"x" * 300)])
    for cut in range(len(data) + 1):
        ing = Ingest(capacity_bytes=1 << 16)
        assert ing.feed(data[:cut]) + ing.feed(data[cut:]) == 3
        ing.set_eof()
        got = drain(ing)
        assert [(d.topic_id, d.content) for d in got] == [(1, b"hello"), (2, b""), (1, b"x" * 300)]
        assert [d.tag for d in got] == [1, 2, 3]


def test_wraparound_many_times():
    ing = Ingest(capacity_bytes=4096)
    sent = []
    got = []
    for i in range(5000):
        p = bytes([i % 251]) * (i % 90)
        sent.append((1 + i % 2, p))
        ing.push(1 + i % 2, p)
        if i % 7 == 0:
            got.extend((d.topic_id, d.content) for d in ing.pop(64, 0.0))
    ing.set_eof()
    got.extend((d.topic_id, d.content) for d in drain(ing))
    assert got == sent


def test_drop_newest_accounting():
    ing = Ingest(capacity_bytes=1 << 16, capacity_events=10, policy="drop_newest")
    acc = sum(ing.push(2, b"p") for _ in range(25))
    assert acc == 10
    st = ing.stats()
    assert st["dropped_total"] == 15 and st["dropped_by_topic"] == {2: 15} and st["depth"] == 10


def test_block_policy_stalls_producer_until_consumed():
    ing = Ingest(capacity_bytes=1 << 16, capacity_events=4, policy="block")
    done = threading.Event()

    def prod():
        for _ in range(12):
            ing.push(1, b"x")
        done.set()

    t = threading.Thread(target=prod)
    t.start()
    time.sleep(0.1)
    assert not done.is_set() and ing.depth == 4
    n = 0
    while n < 12:
        n += len(ing.pop(3, 1.0))
    t.join(5)
    assert done.is_set() and ing.stats()["blocked_ns"] > 0 and ing.stats()["dropped_total"] == 0


def test_reader_thread_pipe_eof():
    r, w = os.pipe()
    ing = Ingest(capacity_bytes=1 << 20)
    ing.start_reader(r, own_fd=True)
    data = frames([(1, b"a%d" % i) for i in range(20000)])

    def writer():
        mv = memoryview(data)
        while mv:
            n = os.write(w, mv[:777])
            mv = mv[n:]
        os.close(w)

    threading.Thread(target=writer).start()
    got = drain(ing, 10)
    assert len(got) == 20000 and got[-1].content == b"a19999"
    st = ing.stats()
    assert st["eof"] and st["error"] is None and st["frames_read"] == 20000
    assert ing.pop(10, 0.0) is None


def test_reader_truncated_stream_reports_error():
    r, w = os.pipe()
    ing = Ingest()
    ing.start_reader(r, own_fd=True)
    os.write(w, frame(1, b"ok") + b"\x09\x00\x00\x00\x01abc")
    os.close(w)
    got = drain(ing)
    assert [d.content for d in got] == [b"ok"]
    assert "truncated" in ing.stats()["error"]


def test_corrupt_frame_zero_length():
    ing = Ingest()
    with pytest.raises(ValueError):
        ing.feed(b"\x00\x00\x00\x00")


def test_oversized_frame_rejected():
    ing = Ingest(capacity_bytes=1 << 16)  # max_frame = 16 KiB
    with pytest.raises(ValueError):
        ing.feed(b"\xff\xff\x00\x00\x01")


def test_close_unblocks_reader_and_pop():
    r, w = os.pipe()
    ing = Ingest()
    ing.start_reader(r)
    t0 = time.time()
    ing.close()
    assert time.time() - t0 < 2
    assert ing.pop(10, 0.1) is None
    os.close(r)
    os.close(w)


def test_ndjson_frames():
    data = ndjson_to_frames(['{"topic": "v1.telemetry.progress", "json": {"mediaId": "m", "status": "DEPLOYED",'
                             ' "progress": 5}}', '{"topic": "v1.telemetry.status", "b64": "CgFt"}'])
    fr = list(iter_frames(data))
    assert fr[0][0] == 2 and fr[1] == (1, b"\x0a\x01m")


# ---- event-loop wake-up: eventfd, one hop, no executor (transport/ingest.py FdSource.batches) ----

def test_arm_signals_notify_fd_once():
    ing = Ingest(capacity_bytes=1 << 16)
    efd = ing.notify_fd
    assert ing.notify_fd == efd  # created once, owned by the Ingest
    assert ing.arm() is True  # empty: parked
    import select
    assert select.select([efd], [], [], 0)[0] == []
    ing.push(0, b"a")
    ing.push(0, b"b")  # second push while disarmed: no extra signal needed
    assert select.select([efd], [], [], 0)[0] == [efd]
    ing.clear_notify()
    assert select.select([efd], [], [], 0)[0] == []
    assert ing.arm() is False  # records queued: pop instead of parking
    assert [d.content for d in ing.pop(10, 0.0)] == [b"a", b"b"]
    assert ing.arm() is True
    ing.set_eof()  # EOF wakes a parked loop too
    assert select.select([efd], [], [], 0)[0] == [efd]
    ing.clear_notify()
    assert ing.pop(10, 0.0) is None
    assert ing.arm() is False  # drained: never park again
    ing.close()


def test_idle_fdsource_uses_no_executor_thread():
    """An idle FdSource parks on the ring's eventfd (loop.add_reader): nothing is submitted to the
    loop's default executor, and every idle wake-up is one reader->loop hop."""
    import asyncio
    import concurrent.futures

    from beholder_amd.transport.ingest import FdSource

    class CountingExecutor(concurrent.futures.ThreadPoolExecutor):
        submitted = 0

        def submit(self, *a, **kw):
            CountingExecutor.submitted += 1
            return super().submit(*a, **kw)

    async def go():
        loop = asyncio.get_running_loop()
        ex = CountingExecutor(max_workers=1)
        loop.set_default_executor(ex)
        r, w = os.pipe()
        src = FdSource(fd=r)
        await src.start()
        got = []

        async def consume():
            async for batch in src.batches():
                for d in batch:
                    got.append(d.content)
                    d.ack()

        task = asyncio.ensure_future(consume())
        for i in range(5):  # idle between events: each one is a separate park + wake-up
            await asyncio.sleep(0.02)
            os.write(w, frame(0, b"e%d" % i))
        await asyncio.sleep(0.05)
        os.close(w)
        await asyncio.wait_for(task, 5)
        st = src.stats()
        await src.close()
        os.close(r)
        ex.shutdown()
        return got, st

    got, st = asyncio.run(go())
    assert got == [b"e0", b"e1", b"e2", b"e3", b"e4"]
    assert CountingExecutor.submitted == 0
    assert st["idle_wakeups"] >= 5
    assert st["acked"] == 5


def test_paced_write_rate_and_order():
    from array import array

    from beholder_amd.ops.bench_native import paced_write
    chunks = [frame(i % 2, b"x%03d" % i) for i in range(200)]
    ends = array("Q")
    pos = 0
    for c in chunks:
        pos += len(c)
        ends.append(pos)
    r, w = os.pipe()
    out = bytearray()

    def rd():
        while True:
            b = os.read(r, 1 << 16)
            if not b:
                return
            out.extend(b)

    t = threading.Thread(target=rd)
    t.start()
    from beholder_amd.ops import mono_ns
    before = mono_ns()
    elapsed, writes, t0 = paced_write(w, b"".join(chunks), ends.tobytes(), 2000.0)  # 200 frames at 2k/s
    assert before <= t0 <= mono_ns()  # frame 0's due time, on the Delivery clock
    os.close(w)
    t.join()
    os.close(r)
    assert bytes(out) == b"".join(chunks)
    assert 0.09 <= elapsed < 1.0  # the last frame is due at 199/2000 s
    assert 2 <= writes <= 200
    with pytest.raises(ValueError):
        paced_write(1, b"ab", array("Q", [3]).tobytes(), 10.0)  # end beyond data
    with pytest.raises(ValueError):
        paced_write(1, b"ab", array("Q", [1]).tobytes(), 0.0)
    with pytest.raises(ValueError):
        paced_write(1, b"abc", array("Q", [2, 1]).tobytes(), 10.0)  # ends must not decrease
    r, w = os.pipe()
    os.close(r)  # the consumer went away: EPIPE, not a signal
    try:
        with pytest.raises(OSError):
            paced_write(w, b"abcd", array("Q", [2, 4]).tobytes(), 1000.0)
    finally:
        os.close(w)


def test_queue_latency_is_receive_to_start():
    from beholder_amd.ops import Delivery, Settler, mono_ns
    s = Settler()
    d = Delivery(b"x", 0, 1, s, mono_ns() - 5_000_000)  # received 5 ms ago
    d.start()
    d.ack()
    assert s.queue_latency.count == 1
    assert s.queue_latency.percentile(50) >= 4_000_000
    assert s.handle_latency.percentile(50) < 4_000_000
    s.reset_latency()
    assert s.queue_latency.count == 0


def test_settler_slow_trace_threshold_capacity_and_stop():
    from beholder_amd.ops import Delivery, Settler, mono_ns
    s = Settler()
    s.trace_slow(50_000_000, 2)  # >= 50 ms from start to settle, room for two

    def settle(start_ago_ns):
        d = Delivery(b"x", 0, 1, s, mono_ns() - start_ago_ns - 10)
        d.start()
        if start_ago_ns:  # pretend the handler started earlier
            time.sleep(start_ago_ns / 1e9)
        d.ack()
    settle(0)          # fast: not traced
    for _ in range(3):
        settle(60_000_000)  # slow: two fit, one is counted as dropped
    recs, dropped = s.slow_deliveries()
    assert len(recs) == 2 and dropped == 1
    assert all(recv <= start <= settle_ and settle_ - start >= 50_000_000 for recv, start, settle_ in recs)
    s.trace_slow(0)
    assert s.slow_deliveries() == ([], 0)
    with pytest.raises(ValueError):
        s.trace_slow(1, 1 << 40)
