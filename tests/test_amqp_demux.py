"""Native AMQP delivery demux (ops.AmqpDemux) vs the Python frame path."""
import pytest

from beholder_amd.ops import AmqpDemux, Settler
from beholder_amd.transport.amqp import wire


def deliver(ch, ctag, tag, body, redelivered=False, frame_max=131072):
    return (wire.encode_method(ch, "basic.deliver", consumer_tag=ctag, delivery_tag=tag, redelivered=redelivered,
                               exchange="", routing_key="q")
            + wire.encode_content(ch, 60, body, {"delivery_mode": 2}, frame_max))


def stream():
    return b"".join([
        deliver(1, "c1", 1, b"hello"),
        wire.encode_heartbeat(),
        deliver(1, "c1", 2, b"x" * 300, redelivered=True, frame_max=100),   # body split over 4 frames
        wire.encode_method(2, "channel.close", reply_code=406, reply_text="PRECONDITION_FAILED", class_id=60,
                           method_id=80),
        deliver(1, "unknown", 3, b"slow"),                                  # passthrough (3 frames)
        deliver(1, "c1", 4, b""),                                           # zero-length body
    ])


def run(data, chunk=None):
    s = Settler()
    dm = AmqpDemux(s, 0)
    extra = object()
    dm.add_consumer(1, "c1", 2, extra)
    out = []
    if chunk is None:
        out.extend(dm.feed(data))
    else:
        for i in range(0, len(data), chunk):
            out.extend(dm.feed(data[i:i + chunk]))
    return out, extra, dm


def summarize(out):
    res = []
    for it in out:
        if isinstance(it, tuple):
            t, ch, payload = it
            res.append(("frame", t, ch, wire.decode_method(payload).name if t == 1 else len(payload)))
        else:
            res.append(("delivery", it.tag, it.topic_id, it.content, it.redelivered))
    return res


def test_native_assembly_and_passthrough_order():
    out, extra, dm = run(stream())
    assert summarize(out) == [
        ("delivery", 1, 2, b"hello", False),
        ("delivery", 2, 2, b"x" * 300, True),
        ("frame", 1, 2, "channel.close"),
        ("frame", 1, 1, "basic.deliver"),
        ("frame", 2, 1, len(wire.encode_content(1, 60, b"slow", {"delivery_mode": 2}, 131072)) - 8 - 12),
        ("frame", 3, 1, 4),
        ("delivery", 4, 2, b"", False),
    ]
    assert out[0].extra is extra and out[0].state == "pending"
    st = dm.stats()
    assert st["deliveries"] == 3 and st["heartbeats"] == 1


@pytest.mark.parametrize("chunk", [1, 2, 3, 7, 64, 333])
def test_any_split_gives_same_result(chunk):
    whole = summarize(run(stream())[0])
    assert summarize(run(stream(), chunk)[0]) == whole


def test_errors():
    dm = AmqpDemux(Settler(), 0)
    with pytest.raises(ValueError):
        dm.feed(b"\x08\x00\x00\x00\x00\x00\x00\x00")  # bad frame-end
    dm = AmqpDemux(Settler(), 16)
    with pytest.raises(ValueError):
        dm.feed(deliver(1, "c1", 1, b"x" * 64))


def test_remove_and_reset():
    s = Settler()
    dm = AmqpDemux(s, 0)
    dm.add_consumer(1, "c1", 1, None)
    dm.remove_consumer(1, "c1")
    assert all(isinstance(x, tuple) for x in dm.feed(deliver(1, "c1", 1, b"a")))
    dm.add_consumer(1, "c1", 1, None)
    dm.reset_channel(1)
    assert dm.stats()["consumers"] == 0
