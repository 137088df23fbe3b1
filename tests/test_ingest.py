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
