"""Delivery / Settler ack semantics (index.js:71,124,151,154; quirk Q1)."""
import gc

import pytest

from beholder_amd.ops import Delivery, Settler


def test_ack_once():
    s = Settler()
    d = Delivery(b"x", 1, 7, s)
    assert d.message.content == b"x" and d.topic == "v1.telemetry.status" and d.tag == 7
    d.start()
    d.ack()
    assert d.acked and d.state == "acked"
    with pytest.raises(RuntimeError):
        d.ack()
    with pytest.raises(RuntimeError):
        d.nack()
    assert s.stats() == {"created": 1, "acked": 1, "nacked": 0, "rejected": 0, "abandoned": 0, "pending": 0}
    assert s.handle_latency.count == 1 and s.ingest_latency.count == 1


def test_nack_reject_and_callback():
    calls = []
    s = Settler(on_settle=lambda d, kind, requeue: calls.append((d.tag, kind, requeue)))
    Delivery(b"", 2, 1, s).nack()
    Delivery(b"", 2, 2, s).nack(requeue=False)
    Delivery(b"", 2, 3, s).reject()
    Delivery(b"", 2, 4, s).ack()
    assert calls == [(1, "nack", True), (2, "nack", False), (3, "reject", False), (4, "ack", False)]
    assert s.nacked == 2 and s.rejected == 1 and s.acked == 1


def test_abandoned_delivery_reported():
    """A delivery freed while pending was never acked (Q1)."""
    seen = []
    s = Settler(on_abandon=lambda tag, tid, content: seen.append((tag, tid, content)))
    d = Delivery(b"payload", 1, 42, s)
    del d
    gc.collect()
    assert seen == [(42, 1, b"payload")] and s.abandoned == 1 and s.pending == 0


def test_settle_callback_error_propagates():
    def boom(d, k, r):
        raise ConnectionError("channel closed")
    s = Settler(on_settle=boom)
    d = Delivery(b"", 1, 1, s)
    with pytest.raises(ConnectionError):
        d.ack()


def test_delivery_without_settler():
    d = Delivery(b"abc")
    d.ack()
    assert d.acked and d.topic is None


def test_extra_roundtrip():
    d = Delivery(b"", extra={"routing_key": "q"})
    assert d.extra == {"routing_key": "q"}
    d.extra = None
    assert d.extra is None
