"""Jaeger tracing (utils/tracing.py): context propagation, samplers, the Thrift compact
emitBatch packet (decoded here by an independent reader), the UDP reporter, and spans of a
running service fed over AMQP with ``uber-trace-id`` headers."""
from __future__ import annotations

import asyncio
import socket
import struct

import pytest

from beholder_amd.config import Config
from beholder_amd.service import Service
from beholder_amd.sinks import RecordingHttpClient
from beholder_amd.store import MemoryStore
from beholder_amd.topics import PROGRESS, STATUS
from beholder_amd.transport.amqp import AmqpBroker, AmqpSource
from beholder_amd.transport.amqp.wire import encode_table
from beholder_amd.utils import tracing as tr
from beholder_amd.utils.log import Logger, MemoryStream

from helpers import BASE_CFG, progress_msg, status_msg, trello_media


# ------------------------------------------------ independent compact reader --
class Reader:
    """Thrift compact protocol reader written from the spec (not from tracing.py)."""

    def __init__(self, b: bytes):
        self.b, self.i = b, 0

    def byte(self):
        v = self.b[self.i]
        self.i += 1
        return v

    def varint(self):
        shift = n = 0
        while True:
            c = self.byte()
            n |= (c & 0x7F) << shift
            shift += 7
            if not c & 0x80:
                return n

    def zigzag(self):
        n = self.varint()
        return (n >> 1) ^ -(n & 1)

    def value(self, t):
        if t in (1, 2):
            return t == 1
        if t in (4, 5, 6):
            return self.zigzag()
        if t == 3:
            return self.byte()
        if t == 7:
            v = struct.unpack_from("<d", self.b, self.i)[0]
            self.i += 8
            return v
        if t == 8:
            n = self.varint()
            v = self.b[self.i:self.i + n]
            self.i += n
            return v
        if t == 9:
            h = self.byte()
            size, et = h >> 4, h & 15
            if size == 15:
                size = self.varint()
            return [self.value(et) for _ in range(size)]
        if t == 12:
            return self.struct()
        raise AssertionError(f"type {t}")

    def struct(self):
        out, last = {}, 0
        while True:
            h = self.byte()
            if h == 0:
                return out
            t, delta = h & 15, h >> 4
            fid = last + delta if delta else self.zigzag()
            out[fid] = self.value(t)
            last = fid

    def message(self):
        assert self.byte() == 0x82
        vt = self.byte()
        assert vt & 0x1F == 1 and vt >> 5 == 4  # version 1, ONEWAY
        seq = self.varint()
        name = self.value(8).decode()
        return name, seq, self.struct()


def tags_of(lst):
    out = {}
    for t in lst:
        k = t[1].decode()
        out[k] = {0: lambda: t[3].decode(), 1: lambda: t[4], 2: lambda: t[5], 3: lambda: t[6],
                  4: lambda: t[7]}[t[2]]()
    return out


def u64(v):
    return v & ((1 << 64) - 1)


# ------------------------------------------------------------------ context --
def test_uber_trace_id_round_trip_and_garbage():
    ctx = tr.parse_uber_trace_id("abcdef0123456789abcdef0123456789:1f:2e:1")
    assert ctx == tr.SpanContext(0xabcdef0123456789abcdef0123456789, 0x1f, 0x2e, 1) and ctx.sampled
    assert tr.parse_uber_trace_id(tr.format_uber_trace_id(ctx)) == ctx
    assert tr.parse_uber_trace_id("ab%3A1%3A0%3A0") == tr.SpanContext(0xab, 1, 0, 0)
    for bad in ("", "1:2:3", "x:1:0:1", "0:1:0:1", "1:0:0:1", None, 5):
        assert tr.parse_uber_trace_id(bad) is None


def test_traceparent():
    ctx = tr.parse_traceparent("00-4bf92f3577b34da6a3ce929d0e0e4736-00f067aa0ba902b7-01")
    assert ctx == tr.SpanContext(0x4bf92f3577b34da6a3ce929d0e0e4736, 0x00f067aa0ba902b7, 0, 1)
    assert tr.parse_traceparent("00-00000000000000000000000000000000-00f067aa0ba902b7-01") is None
    assert tr.parse_traceparent("zz") is None


def test_extract_from_dict_raw_amqp_table_and_garbage():
    h = {"x": 1, "uber-trace-id": "a:b:c:1"}
    assert tr.extract(h) == tr.SpanContext(0xa, 0xb, 0xc, 1)
    assert tr.extract(encode_table(h)) == tr.SpanContext(0xa, 0xb, 0xc, 1)
    assert tr.extract({"traceparent": "00-4bf92f3577b34da6a3ce929d0e0e4736-00f067aa0ba902b7-00"}).sampled is False
    assert tr.extract(b"\x00\x00\x00\x09garbage") is None
    assert tr.extract(None) is None and tr.extract({"a": "b"}) is None


# ----------------------------------------------------------------- samplers --
def test_samplers():
    assert tr.make_sampler("const", 1).is_sampled(5) and not tr.make_sampler("const", 0).is_sampled(5)
    p = tr.make_sampler("probabilistic", 0.25)
    assert p.is_sampled((1 << 61) - 1) and not p.is_sampled(1 << 61)
    assert sum(p.is_sampled(i * 0x9E3779B97F4A7C15 & ((1 << 64) - 1)) for i in range(4000)) in range(850, 1150)
    now = [0.0]
    r = tr.RateLimitingSampler(2.0, clock=lambda: now[0])
    assert [r.is_sampled(1) for _ in range(3)] == [True, True, False]
    now[0] = 0.5
    assert r.is_sampled(1) and not r.is_sampled(1)
    with pytest.raises(ValueError):
        tr.make_sampler("adaptive", 1)


def test_upstream_decision_wins():
    t = tr.Tracer("svc", tr.ConstSampler(True), tr.InMemoryReporter())
    assert t.start_span("x", child_of=tr.SpanContext(1, 2, 0, 0)) is None  # upstream: not sampled
    s = t.start_span("x", child_of=tr.SpanContext(7, 8, 0, 1))
    assert s.context.trace_id == 7 and s.context.parent_id == 8 and s.references == [(0, tr.SpanContext(7, 8, 0, 1))]
    assert "sampler.type" not in s.tags
    t2 = tr.Tracer("svc", tr.ConstSampler(False), tr.InMemoryReporter())
    assert t2.start_span("x") is None


# ------------------------------------------------------------ thrift packet --
def test_emit_batch_packet_decodes_per_jaeger_idl():
    t = tr.Tracer("beholder", tr.ConstSampler(True), tr.InMemoryReporter())
    parent = tr.SpanContext((0xF123 << 64) | 0xFEDCBA9876543210, 0x8000000000000001, 0, 1)
    s = t.start_span("v1.telemetry.progress", child_of=parent, start_us=1_700_000_000_000_000,
                     tags={"s": "ü", "n": -3, "b": True, "f": 1.5, "raw": b"\x00\x01"})
    s.log_kv({"event": "error", "message": "boom"}, timestamp_us=1_700_000_000_000_123)
    s.finish(end_us=1_700_000_000_000_250)
    pkt = tr.encode_emit_batch("beholder", {"hostname": "h1", "jaeger.version": "Python-beholder"}, [s], seq_id=7)
    name, seq, args = Reader(pkt).message()
    assert name == "emitBatch" and seq == 7
    batch = args[1]
    assert batch[1][1] == b"beholder" and tags_of(batch[1][2]) == {"hostname": "h1",
                                                                    "jaeger.version": "Python-beholder"}
    (span,) = batch[2]
    assert u64(span[1]) == 0xFEDCBA9876543210 and u64(span[2]) == 0xF123
    assert u64(span[3]) == s.context.span_id and u64(span[4]) == 0x8000000000000001
    assert span[5] == b"v1.telemetry.progress" and span[7] == 1
    assert span[8] == 1_700_000_000_000_000 and span[9] == 250
    ((ref_type, ref_lo, ref_hi, ref_span),) = [(r[1], u64(r[2]), u64(r[3]), u64(r[4])) for r in span[6]]
    assert (ref_type, ref_lo, ref_hi, ref_span) == (0, 0xFEDCBA9876543210, 0xF123, 0x8000000000000001)
    assert tags_of(span[10]) == {"s": "ü", "n": -3, "b": True, "f": 1.5, "raw": b"\x00\x01"}
    (log,) = span[11]
    assert log[1] == 1_700_000_000_000_123 and tags_of(log[2]) == {"event": "error", "message": "boom"}


def test_udp_reporter_batches_into_packets_under_the_limit():
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    rx.settimeout(5)
    rep = tr.UdpReporter("svc", "127.0.0.1", rx.getsockname()[1], max_packet=1200)
    t = tr.Tracer("svc", tr.ConstSampler(True), rep)
    for i in range(40):
        t.start_span(f"op{i}", tags={"pad": "x" * 50}).finish()
    t.close()
    got = 0
    pkts = 0
    while got < 40:
        data = rx.recv(65535)
        assert len(data) <= 1200
        _, _, args = Reader(data).message()
        got += len(args[1][2])
        pkts += 1
    assert pkts > 1 and rep.stats()["spans"] == 40 and rep.stats()["dropped"] == 0
    big = tr.Tracer("svc", tr.ConstSampler(True), tr.UdpReporter("svc", "127.0.0.1", 9, max_packet=200))
    big.start_span("huge", tags={"pad": "y" * 500}).finish()
    assert big.reporter.stats()["dropped"] == 1
    rx.close()


def test_tracer_from_config_env():
    assert tr.tracer_from_config({}, env={}) is None
    t = tr.tracer_from_config({}, env={"JAEGER_AGENT_HOST": "127.0.0.1", "JAEGER_AGENT_PORT": "6999",
                                       "JAEGER_SERVICE_NAME": "bh", "JAEGER_SAMPLER_TYPE": "probabilistic",
                                       "JAEGER_SAMPLER_PARAM": "0.5", "JAEGER_TAGS": "env=prod,x=${NOPE_X:d}"})
    assert t.service_name == "bh" and t.sampler.type == "probabilistic" and t.sampler.param == 0.5
    assert t.reporter.addr == ("127.0.0.1", 6999) and t.tags["env"] == "prod" and t.tags["x"] == "d"
    assert tr.tracer_from_config({"enabled": True}, env={"JAEGER_DISABLED": "true"}) is None


# ------------------------------------------------------------- service e2e --
@pytest.mark.parametrize("native_demux", [True, False])
def test_service_spans_join_upstream_traces_over_amqp(native_demux):
    """Messages published with uber-trace-id headers: each delivery span is a child of the
    producer's span, carries mediaId / outcome, and a throwing status handler (Q1) is an error span."""
    rep = tr.InMemoryReporter()

    async def go():
        broker = await AmqpBroker().start()
        try:
            d = {k: v for k, v in BASE_CFG.items()}
            d["service"] = {"metrics": {"enabled": False}, "tracing": {"enabled": True}}
            svc = Service(Config.from_dict(d, env={}), source=AmqpSource(broker.url, capture_headers=True, native=native_demux),
                          store=MemoryStore([trello_media("m1", card="C1")]), http=RecordingHttpClient(),
                          logger=Logger(stream=MemoryStream()))
            svc.tracer = tr.Tracer("beholder", tr.ConstSampler(True), rep)
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            for i in range(5):
                broker.publish(PROGRESS, progress_msg("m1", "UPLOADING", i),
                               properties={"headers": {"uber-trace-id": f"{0xabc0 + i:x}:{0x100 + i:x}:0:1"}})
            broker.publish(PROGRESS, progress_msg("m1", "UPLOADING", 9),
                           properties={"headers": {"uber-trace-id": "abcd:99:0:0"}})  # upstream: not sampled
            broker.publish(STATUS, b"\xff\xff")  # undecodable: the status handler throws (Q1)
            broker.publish(STATUS, status_msg("m1", "QUEUED"))  # no headers: a new root trace
            for _ in range(300):
                if broker.stats(PROGRESS)["acked"] == 6 and broker.stats(STATUS)["acked"] == 1:
                    break
                await asyncio.sleep(0.02)
            svc.request_stop()
            await task
            await svc.close()
        finally:
            await broker.stop()

    asyncio.run(asyncio.wait_for(go(), 60))
    by_trace = {s.context.trace_id: s for s in rep.spans}
    for i in range(5):
        s = by_trace[0xabc0 + i]
        assert s.context.parent_id == 0x100 + i and s.operation == PROGRESS
        assert s.tags["mediaId"] == "m1" and s.tags["beholder.outcome"] == "acked"
        assert s.tags["span.kind"] == "consumer" and s.tags["beholder.queue_us"] >= 0 and s.duration_us >= 0
    assert 0xabcd not in by_trace
    status_spans = [s for s in rep.spans if s.operation == STATUS]
    assert len(status_spans) == 2
    err = [s for s in status_spans if s.tags.get("error")]
    ok = [s for s in status_spans if not s.tags.get("error")]
    assert len(err) == 1 and err[0].tags["beholder.outcome"] == "pending" and err[0].logs[0][1]["event"] == "error"
    assert ok[0].context.parent_id == 0 and ok[0].tags["sampler.type"] == "const"
    assert len(rep.spans) == 7


def test_unsampled_deliveries_stay_on_the_native_dispatch_path():
    """With a sampler that says no, only deliveries whose upstream trace is sampled get spans;
    the rest run through the native dispatch loop in batches. Every delivery is acked."""
    rep = tr.InMemoryReporter()

    async def go():
        broker = await AmqpBroker().start()
        try:
            d = {k: v for k, v in BASE_CFG.items()}
            d["service"] = {"metrics": {"enabled": False}, "tracing": {"enabled": True}}
            svc = Service(Config.from_dict(d, env={}), source=AmqpSource(broker.url, capture_headers=True),
                          store=MemoryStore([trello_media("m1", card="C1")]), http=RecordingHttpClient(),
                          logger=Logger(stream=MemoryStream()))
            svc.tracer = tr.Tracer("beholder", tr.ConstSampler(False), rep)
            calls = []
            orig = svc._dispatch_now
            svc._dispatch_now = lambda *a, **kw: calls.append(1) or orig(*a, **kw)
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            for i in range(50):
                props = {"headers": {"uber-trace-id": f"{0x5000 + i:x}:{0x10 + i:x}:0:1"}} if i % 17 == 3 else \
                    {"headers": {"x-other": "y"}}
                broker.publish(PROGRESS, progress_msg("m1", "UPLOADING", i), properties=props)
            for _ in range(300):
                if broker.stats(PROGRESS)["acked"] == 50:
                    break
                await asyncio.sleep(0.02)
            svc.request_stop()
            await task
            await svc.close()
            return broker.stats(PROGRESS), calls
        finally:
            await broker.stop()

    st, calls = asyncio.run(asyncio.wait_for(go(), 60))
    assert st["acked"] == 50
    traced = sorted(s.context.trace_id for s in rep.spans)
    assert traced == [0x5000 + i for i in range(50) if i % 17 == 3]
    assert len(calls) == len(traced)  # only the sampled ones took the Python dispatch path
