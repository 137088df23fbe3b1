"""Fuzzing of the native parsers that face untrusted bytes (network / stdin).

Any input must yield a result or a Python exception — never a crash, hang or
corrupted state. Covers AmqpDemux.feed (AMQP socket bytes) and Ingest.feed
(stdin frame stream); the protobuf codec is fuzzed in test_codec.py.
"""
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from beholder_amd.ops import AmqpDemux, Ingest, Settler
from beholder_amd.transport.amqp import wire


def _valid_stream(n, body):
    out = b""
    for i in range(n):
        out += (wire.encode_method(1, "basic.deliver", consumer_tag="c", delivery_tag=i + 1, redelivered=False,
                                   exchange="", routing_key="q")
                + wire.encode_content(1, 60, body, None, 64))
    return out


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.binary(max_size=300), st.lists(st.integers(1, 64), max_size=8))
def test_demux_random_bytes_never_crash(data, cuts):
    dm = AmqpDemux(Settler(), 4096)
    dm.add_consumer(1, "c", 2, None)
    i = 0
    for c in cuts + [len(data)]:
        try:
            dm.feed(data[i:i + c])
        except ValueError:
            return
        i += c


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(1, 5), st.binary(max_size=200), st.integers(0, 10_000), st.integers(0, 255))
def test_demux_mutated_valid_stream(n, body, pos, byte):
    data = bytearray(_valid_stream(n, body))
    if data:
        data[pos % len(data)] = byte
    dm = AmqpDemux(Settler(), 0)
    dm.add_consumer(1, "c", 2, None)
    try:
        out = dm.feed(bytes(data))
    except ValueError:
        return
    for it in out:
        if not isinstance(it, tuple):
            assert it.topic_id == 2 and len(it.content) <= len(body) + 256


@settings(max_examples=400, deadline=None)
@given(st.binary(max_size=400))
def test_ingest_feed_random_bytes(data):
    ing = Ingest(capacity_bytes=1 << 16)
    try:
        ing.feed(data)
    except ValueError:
        return
    ing.set_eof()
    got = []
    while True:
        b = ing.pop(1000, 0.0)
        if b is None:
            break
        got.extend(b)
    assert sum(len(d.content) + 5 for d in got) <= len(data)


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.dictionaries(st.text(max_size=8), st.one_of(st.text(max_size=30), st.integers(-5, 5), st.booleans()),
                       max_size=4),
       st.sampled_from([None, "application/protobuf"]), st.sampled_from([None, "gzip"]),
       st.integers(0, 10_000), st.integers(0, 255), st.booleans())
def test_demux_header_capture(headers, ctype, cenc, pos, byte, mutate):
    """capture_headers: the raw `headers` table of each delivery equals wire.encode_table (any
    preceding content-type / content-encoding properties skipped); corrupted header frames
    never crash and never yield a table that overruns the frame."""
    props = {"headers": headers or None, "content_type": ctype, "content_encoding": cenc, "delivery_mode": 2}
    data = bytearray(wire.encode_method(1, "basic.deliver", consumer_tag="c", delivery_tag=1, redelivered=False,
                                        exchange="", routing_key="q")
                     + wire.encode_content(1, 60, b"body", props, 4096))
    if mutate:
        data[pos % len(data)] = byte
    dm = AmqpDemux(Settler(), 0)
    dm.capture_headers = True
    dm.add_consumer(1, "c", 2, None)
    try:
        out = dm.feed(bytes(data))
    except ValueError:
        return
    ds = [it for it in out if not isinstance(it, tuple)]
    for d in ds:
        if d.headers is not None:
            assert len(d.headers) >= 4 and len(d.headers) <= len(data)
    if not mutate:
        assert len(ds) == 1
        assert ds[0].headers == (wire.encode_table(headers) if headers else None)
