"""Distributed tracing: one Jaeger span per handled delivery.

The reference ships the tracing stack through triton-core: jaeger-client and opentracing
(yarn.lock:1023-1032, 1996-2008). beholder's own code never creates a span (SURVEY.md §5,
"Tracing / profiling"). This module gives the rebuild the same capability and nothing more:

* **Inbound context.** Each message's headers are read for ``uber-trace-id`` (jaeger-client's
  text-map format ``{trace-id}:{span-id}:{parent-span-id}:{flags}``, hex, also URL-encoded)
  and for W3C ``traceparent``. When an upstream producer sent a trace, the delivery span
  joins it as a CHILD_OF reference. The parent's sampling decision is respected.
* **Samplers.** ``const``, ``probabilistic`` and ``ratelimiting``, with jaeger-client's
  semantics and its ``sampler.type`` / ``sampler.param`` root-span tags.
* **Reporter.** Spans are batched and sent to a jaeger-agent over UDP (port 6831). Each
  packet is an ``Agent.emitBatch`` oneway message in the Thrift *compact* protocol
  (jaeger-idl ``agent.thrift`` / ``jaeger.thrift``), at most 65,000 bytes per packet, as
  jaeger-client does. An in-memory reporter serves tests.
* **Configuration.** The ``service.tracing`` section and jaeger-client's ``initTracerFromEnv``
  variables: ``JAEGER_SERVICE_NAME``, ``JAEGER_AGENT_HOST``, ``JAEGER_AGENT_PORT``,
  ``JAEGER_SAMPLER_TYPE``, ``JAEGER_SAMPLER_PARAM``, ``JAEGER_TAGS`` and ``JAEGER_DISABLED``.

Spans cover the handler: start = handler call, finish = settle or error. The time the
message waited in the ingest ring is the ``beholder.queue_us`` tag. A span carries the
topic, delivery tag, redelivery flag, ``mediaId`` and outcome (acked / nacked / rejected /
pending = quirk Q1). On a handler error it also carries ``error=true`` and an error log.
"""
from __future__ import annotations

import os
import random
import socket
import struct
import threading
import time
from typing import Any, Dict, Iterable, List, Mapping, NamedTuple, Optional, Sequence, Tuple

UBER_TRACE_ID = "uber-trace-id"
TRACEPARENT = "traceparent"
DEFAULT_AGENT_PORT = 6831
MAX_PACKET = 65000  # jaeger-client UDP sender limit
_MASK64 = (1 << 64) - 1


# ---------------------------------------------------------------- context ---
class SpanContext(NamedTuple):
    trace_id: int  # up to 128 bits
    span_id: int
    parent_id: int
    flags: int  # bit 0 = sampled, bit 1 = debug

    @property
    def sampled(self) -> bool:
        return bool(self.flags & 1)


def parse_uber_trace_id(value: Any) -> Optional[SpanContext]:
    """``{trace-id}:{span-id}:{parent-span-id}:{flags}`` (hex; ``%3A`` separators accepted)."""
    if isinstance(value, (bytes, bytearray)):
        value = bytes(value).decode("latin-1")
    if not isinstance(value, str):
        return None
    parts = value.replace("%3A", ":").replace("%3a", ":").split(":")
    if len(parts) != 4:
        return None
    try:
        trace_id, span_id, parent_id, flags = (int(p, 16) for p in parts)
    except ValueError:
        return None
    if trace_id == 0 or span_id == 0 or trace_id >> 128 or span_id >> 64 or parent_id >> 64 or flags >> 8:
        return None
    return SpanContext(trace_id, span_id, parent_id, flags)


def format_uber_trace_id(ctx: SpanContext) -> str:
    return f"{ctx.trace_id:x}:{ctx.span_id:x}:{ctx.parent_id:x}:{ctx.flags:x}"


def parse_traceparent(value: Any) -> Optional[SpanContext]:
    """W3C ``00-{32 hex trace-id}-{16 hex parent-id}-{2 hex flags}``."""
    if isinstance(value, (bytes, bytearray)):
        value = bytes(value).decode("latin-1")
    if not isinstance(value, str):
        return None
    parts = value.strip().split("-")
    if len(parts) < 4 or len(parts[0]) != 2 or len(parts[1]) != 32 or len(parts[2]) != 16 or len(parts[3]) != 2:
        return None
    try:
        version, trace_id, span_id, flags = int(parts[0], 16), int(parts[1], 16), int(parts[2], 16), int(parts[3], 16)
    except ValueError:
        return None
    if version == 0xFF or trace_id == 0 or span_id == 0:
        return None
    return SpanContext(trace_id, span_id, 0, flags & 1)


def extract(headers: Any) -> Optional[SpanContext]:
    """Trace context from message headers: a dict, raw AMQP field-table bytes (the native
    demux keeps them undecoded), or None."""
    if headers is None:
        return None
    if isinstance(headers, (bytes, bytearray)):
        if b"uber-trace-id" not in headers and b"traceparent" not in headers.lower():
            return None  # no trace context: skip decoding the table
        from ..transport.amqp.wire import AmqpError, _Reader
        try:
            headers = _Reader(bytes(headers)).table()
        except (AmqpError, ValueError, struct.error, UnicodeDecodeError):
            return None
    if not isinstance(headers, Mapping):
        return None
    ctx = None
    for k, v in headers.items():
        lk = str(k).lower()
        if lk == UBER_TRACE_ID:
            ctx = parse_uber_trace_id(v)
            if ctx is not None:
                return ctx
        elif lk == TRACEPARENT and ctx is None:
            ctx = parse_traceparent(v)
    return ctx


# --------------------------------------------------------------- samplers ---
class ConstSampler:
    type = "const"

    def __init__(self, decision: bool):
        self.decision = bool(decision)
        self.param = 1 if self.decision else 0

    def is_sampled(self, trace_id: int) -> bool:
        return self.decision


class ProbabilisticSampler:
    """Samples trace ids below ``rate * 2**63`` (the low 64 bits), as jaeger-client does."""

    type = "probabilistic"

    def __init__(self, rate: float):
        self.param = min(1.0, max(0.0, float(rate)))
        self.boundary = int(self.param * (1 << 63))

    def is_sampled(self, trace_id: int) -> bool:
        return (trace_id & ((1 << 63) - 1)) < self.boundary


class RateLimitingSampler:
    """At most ``max_per_second`` new traces per second (token bucket, burst = max(1, rate))."""

    type = "ratelimiting"

    def __init__(self, max_per_second: float, clock=time.monotonic):
        self.param = float(max_per_second)
        self.capacity = max(1.0, self.param)
        self.credits = self.capacity
        self.clock = clock
        self.last = clock()

    def is_sampled(self, trace_id: int) -> bool:
        now = self.clock()
        self.credits = min(self.capacity, self.credits + (now - self.last) * self.param)
        self.last = now
        if self.credits >= 1.0:
            self.credits -= 1.0
            return True
        return False


def make_sampler(kind: str, param: Any):
    kind = (kind or "const").lower()
    if kind == "const":
        return ConstSampler(bool(float(param)) if param is not None else True)
    if kind == "probabilistic":
        return ProbabilisticSampler(0.001 if param is None else float(param))
    if kind in ("ratelimiting", "rate_limiting"):
        return RateLimitingSampler(1.0 if param is None else float(param))
    raise ValueError(f"unknown sampler type {kind!r} (const|probabilistic|ratelimiting)")


# ------------------------------------------------------------------- spans ---
TagValue = Any


class Span:
    __slots__ = ("tracer", "context", "operation", "start_us", "duration_us", "tags", "logs", "references",
                 "finished")

    def __init__(self, tracer: "Tracer", context: SpanContext, operation: str, start_us: int,
                 references: Sequence[Tuple[int, SpanContext]] = (), tags: Optional[Dict[str, TagValue]] = None):
        self.tracer = tracer
        self.context = context
        self.operation = operation
        self.start_us = start_us
        self.duration_us = 0
        self.tags: Dict[str, TagValue] = dict(tags or {})
        self.logs: List[Tuple[int, Dict[str, TagValue]]] = []
        self.references = list(references)
        self.finished = False

    def set_tag(self, key: str, value: TagValue) -> "Span":
        self.tags[key] = value
        return self

    def log_kv(self, fields: Dict[str, TagValue], timestamp_us: Optional[int] = None) -> "Span":
        self.logs.append((timestamp_us if timestamp_us is not None else _now_us(), dict(fields)))
        return self

    def finish(self, end_us: Optional[int] = None) -> None:
        if self.finished:
            return
        self.finished = True
        end = end_us if end_us is not None else _now_us()
        self.duration_us = max(0, end - self.start_us)
        self.tracer.reporter.report(self)


def _now_us() -> int:
    return time.time_ns() // 1000


# ----------------------------------------------------- thrift compact (jaeger) --
# compact type ids
_CT_TRUE, _CT_FALSE, _CT_I32, _CT_I64, _CT_DOUBLE, _CT_BINARY, _CT_LIST, _CT_STRUCT = 1, 2, 5, 6, 7, 8, 9, 12
# jaeger.thrift TagType
TAG_STRING, TAG_DOUBLE, TAG_BOOL, TAG_LONG, TAG_BINARY = 0, 1, 2, 3, 4
REF_CHILD_OF, REF_FOLLOWS_FROM = 0, 1


def _varint(out: bytearray, n: int) -> None:
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return


def _zigzag64(n: int) -> int:
    return ((n << 1) ^ (n >> 63)) & _MASK64


def _signed64(u: int) -> int:
    u &= _MASK64
    return u - (1 << 64) if u >> 63 else u


class _Compact:
    """Minimal Thrift compact-protocol writer (structs, lists, i32/i64/double/bool/string)."""

    def __init__(self):
        self.out = bytearray()
        self._last = [0]

    def field(self, fid: int, ctype: int) -> None:
        delta = fid - self._last[-1]
        if 0 < delta <= 15:
            self.out.append((delta << 4) | ctype)
        else:
            self.out.append(ctype)
            _varint(self.out, ((fid << 1) ^ (fid >> 15)) & 0xFFFF)
        self._last[-1] = fid

    def begin_struct(self) -> None:
        self._last.append(0)

    def end_struct(self) -> None:
        self.out.append(0)  # STOP
        self._last.pop()

    def i32(self, fid: int, v: int) -> None:
        self.field(fid, _CT_I32)
        _varint(self.out, ((v << 1) ^ (v >> 31)) & 0xFFFFFFFF)

    def i64(self, fid: int, v: int) -> None:
        self.field(fid, _CT_I64)
        _varint(self.out, _zigzag64(v))

    def double(self, fid: int, v: float) -> None:
        self.field(fid, _CT_DOUBLE)
        self.out += struct.pack("<d", v)

    def boolean(self, fid: int, v: bool) -> None:
        self.field(fid, _CT_TRUE if v else _CT_FALSE)

    def binary(self, fid: int, v: bytes) -> None:
        self.field(fid, _CT_BINARY)
        _varint(self.out, len(v))
        self.out += v

    def string(self, fid: int, v: str) -> None:
        self.binary(fid, v.encode("utf-8", "replace"))

    def list_begin(self, fid: int, elem_type: int, size: int) -> None:
        self.field(fid, _CT_LIST)
        if size < 15:
            self.out.append((size << 4) | elem_type)
        else:
            self.out.append(0xF0 | elem_type)
            _varint(self.out, size)


def _write_tag(w: _Compact, key: str, v: TagValue) -> None:
    w.begin_struct()
    w.string(1, str(key))
    if isinstance(v, bool):
        w.i32(2, TAG_BOOL)
        w.boolean(5, v)
    elif isinstance(v, int) and -(1 << 63) <= v < (1 << 63):
        w.i32(2, TAG_LONG)
        w.i64(6, v)
    elif isinstance(v, float):
        w.i32(2, TAG_DOUBLE)
        w.double(4, v)
    elif isinstance(v, (bytes, bytearray)):
        w.i32(2, TAG_BINARY)
        w.binary(7, bytes(v))
    else:
        w.i32(2, TAG_STRING)
        w.string(3, str(v))
    w.end_struct()


def _write_tags(w: _Compact, fid: int, tags: Mapping[str, TagValue]) -> None:
    w.list_begin(fid, _CT_STRUCT, len(tags))
    for k, v in tags.items():
        _write_tag(w, k, v)


def encode_span(w: _Compact, s: Span) -> None:
    ctx = s.context
    w.begin_struct()
    w.i64(1, _signed64(ctx.trace_id))
    w.i64(2, _signed64(ctx.trace_id >> 64))
    w.i64(3, _signed64(ctx.span_id))
    w.i64(4, _signed64(ctx.parent_id))
    w.string(5, s.operation)
    if s.references:
        w.list_begin(6, _CT_STRUCT, len(s.references))
        for kind, ref in s.references:
            w.begin_struct()
            w.i32(1, kind)
            w.i64(2, _signed64(ref.trace_id))
            w.i64(3, _signed64(ref.trace_id >> 64))
            w.i64(4, _signed64(ref.span_id))
            w.end_struct()
    w.i32(7, ctx.flags)
    w.i64(8, s.start_us)
    w.i64(9, s.duration_us)
    if s.tags:
        _write_tags(w, 10, s.tags)
    if s.logs:
        w.list_begin(11, _CT_STRUCT, len(s.logs))
        for ts, fields in s.logs:
            w.begin_struct()
            w.i64(1, ts)
            _write_tags(w, 2, fields)
            w.end_struct()
    w.end_struct()


def encode_emit_batch(service_name: str, process_tags: Mapping[str, TagValue], spans: Iterable[Span],
                      seq_id: int = 0) -> bytes:
    """One UDP packet for jaeger-agent: ``Agent.emitBatch(Batch)`` (oneway), Thrift compact."""
    spans = list(spans)
    w = _Compact()
    w.out.append(0x82)  # compact protocol id
    w.out.append(0x81)  # version 1 | ONEWAY (4) << 5
    _varint(w.out, seq_id & 0x7FFFFFFF)
    name = b"emitBatch"
    _varint(w.out, len(name))
    w.out += name
    w.begin_struct()              # emitBatch_args
    w.field(1, _CT_STRUCT)        # 1: Batch batch
    w.begin_struct()
    w.field(1, _CT_STRUCT)        # 1: Process process
    w.begin_struct()
    w.string(1, service_name)
    if process_tags:
        _write_tags(w, 2, process_tags)
    w.end_struct()
    w.list_begin(2, _CT_STRUCT, len(spans))  # 2: list<Span> spans
    for s in spans:
        encode_span(w, s)
    w.end_struct()                # Batch
    w.end_struct()                # args
    return bytes(w.out)


# --------------------------------------------------------------- reporters ---
class InMemoryReporter:
    def __init__(self):
        self.spans: List[Span] = []

    def report(self, span: Span) -> None:
        self.spans.append(span)

    def flush(self) -> None:
        pass

    def close(self) -> None:
        pass

    def stats(self) -> Dict[str, int]:
        return {"spans": len(self.spans)}


class UdpReporter:
    """Batches finished spans into ``emitBatch`` packets for a jaeger-agent (UDP, fire and forget).

    A batch is sent when adding a span would push the packet past ``max_packet`` bytes,
    when ``max_spans`` have accumulated, on :meth:`flush` (the service calls it after each
    delivery batch and every 100 ms) and on :meth:`close`. A span that does not fit in one
    packet on its own is dropped and counted.
    """

    def __init__(self, service_name: str, host: str = "127.0.0.1", port: int = DEFAULT_AGENT_PORT,
                 process_tags: Optional[Mapping[str, TagValue]] = None, max_packet: int = MAX_PACKET,
                 max_spans: int = 100):
        self.service_name = service_name
        self.addr = (host, int(port))
        self.process_tags = dict(process_tags or {})
        self.max_packet = int(max_packet)
        self.max_spans = int(max_spans)
        self._spans: List[Span] = []
        self._size = 0
        self._seq = 0
        self._lock = threading.Lock()
        self._sock: Optional[socket.socket] = None
        self._overhead = len(encode_emit_batch(service_name, self.process_tags, []))
        self.counts = {"spans": 0, "packets": 0, "dropped": 0, "send_errors": 0}

    def _span_size(self, s: Span) -> int:
        w = _Compact()
        encode_span(w, s)
        return len(w.out)

    def report(self, span: Span) -> None:
        n = self._span_size(span)
        if self._overhead + n + 5 > self.max_packet:
            self.counts["dropped"] += 1
            return
        with self._lock:
            if self._spans and self._overhead + self._size + n + 5 > self.max_packet:
                self._send_locked()
            self._spans.append(span)
            self._size += n
            if len(self._spans) >= self.max_spans:
                self._send_locked()

    def _send_locked(self) -> None:
        spans, self._spans, self._size = self._spans, [], 0
        if not spans:
            return
        self._seq += 1
        pkt = encode_emit_batch(self.service_name, self.process_tags, spans, self._seq)
        try:
            if self._sock is None:
                fam = socket.AF_INET6 if ":" in self.addr[0] else socket.AF_INET
                self._sock = socket.socket(fam, socket.SOCK_DGRAM)
                self._sock.setblocking(False)
            self._sock.sendto(pkt, self.addr)
            self.counts["packets"] += 1
            self.counts["spans"] += len(spans)
        except OSError:
            self.counts["send_errors"] += 1
            self.counts["dropped"] += len(spans)

    def flush(self) -> None:
        with self._lock:
            self._send_locked()

    def close(self) -> None:
        self.flush()
        if self._sock is not None:
            self._sock.close()
            self._sock = None

    def stats(self) -> Dict[str, int]:
        return dict(self.counts, buffered=len(self._spans))


# ------------------------------------------------------------------ tracer ---
class Tracer:
    def __init__(self, service_name: str, sampler, reporter, tags: Optional[Mapping[str, TagValue]] = None,
                 rng: Optional[random.Random] = None):
        self.service_name = service_name
        self.sampler = sampler
        self.reporter = reporter
        self.tags = dict(tags or {})
        self._rng = rng or random.Random()

    def _id(self, bits: int = 64) -> int:
        v = 0
        while v == 0:
            v = self._rng.getrandbits(bits)
        return v

    def sample(self, child_of: Optional[SpanContext] = None):
        """The sampling decision alone: ``(context, references, root_tags)`` for a span to
        record, or None. Cheap enough to run for every message; only sampled ones pay for a Span."""
        if child_of is not None:
            if not child_of.sampled:
                return None  # the upstream decision wins (jaeger-client semantics)
            return (SpanContext(child_of.trace_id, self._id(), child_of.span_id, child_of.flags),
                    [(REF_CHILD_OF, child_of)], None)
        trace_id = self._id()
        if not self.sampler.is_sampled(trace_id):
            return None
        return (SpanContext(trace_id, self._id(), 0, 1), [],
                {"sampler.type": self.sampler.type, "sampler.param": self.sampler.param})

    def start_sampled(self, decision, operation: str, start_us: Optional[int] = None,
                      tags: Optional[Dict[str, TagValue]] = None) -> Span:
        ctx, refs, root_tags = decision
        span_tags = dict(root_tags or {})
        span_tags.update(tags or {})
        return Span(self, ctx, operation, start_us if start_us is not None else _now_us(), refs, span_tags)

    def start_span(self, operation: str, child_of: Optional[SpanContext] = None, start_us: Optional[int] = None,
                   tags: Optional[Dict[str, TagValue]] = None) -> Optional[Span]:
        """A recording span, or None when this trace is not sampled (nothing to do then)."""
        decision = self.sample(child_of)
        if decision is None:
            return None
        return self.start_sampled(decision, operation, start_us, tags)

    def flush(self) -> None:
        self.reporter.flush()

    def close(self) -> None:
        self.reporter.close()


def _parse_tags(spec: Optional[str]) -> Dict[str, str]:
    """``JAEGER_TAGS``: ``k=v,k2=v2`` (``${ENV:default}`` values resolved like jaeger-client)."""
    out: Dict[str, str] = {}
    for item in (spec or "").split(","):
        if "=" not in item:
            continue
        k, v = item.split("=", 1)
        v = v.strip()
        if v.startswith("${") and v.endswith("}"):
            name, _, default = v[2:-1].partition(":")
            v = os.environ.get(name, default)
        out[k.strip()] = v
    return out


def tracer_from_config(section: Optional[Mapping[str, Any]], env: Optional[Mapping[str, str]] = None,
                       reporter=None) -> Optional[Tracer]:
    """``service.tracing`` + jaeger-client env variables → a Tracer, or None when disabled."""
    env = os.environ if env is None else env
    section = dict(section or {})
    enabled = bool(section.get("enabled", False)) or bool(env.get("JAEGER_AGENT_HOST"))
    if str(env.get("JAEGER_DISABLED", "")).lower() in ("true", "1"):
        enabled = False
    if not enabled:
        return None
    service = env.get("JAEGER_SERVICE_NAME") or section.get("service_name") or "beholder"
    smp = dict(section.get("sampler") or {})
    sampler = make_sampler(env.get("JAEGER_SAMPLER_TYPE") or smp.get("type", "probabilistic"),
                           env.get("JAEGER_SAMPLER_PARAM", smp.get("param", 0.001)))
    tags = {"hostname": socket.gethostname(), "jaeger.version": "Python-beholder"}
    tags.update({str(k): v for k, v in (section.get("tags") or {}).items()})
    tags.update(_parse_tags(env.get("JAEGER_TAGS")))
    if reporter is None:
        agent = dict(section.get("agent") or {})
        reporter = UdpReporter(service, env.get("JAEGER_AGENT_HOST") or agent.get("host", "127.0.0.1"),
                               int(env.get("JAEGER_AGENT_PORT") or agent.get("port", DEFAULT_AGENT_PORT)),
                               process_tags=tags, max_packet=int(agent.get("max_packet", MAX_PACKET)))
    return Tracer(service, sampler, reporter, tags)
