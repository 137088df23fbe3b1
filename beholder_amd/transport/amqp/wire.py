"""AMQP 0-9-1 wire codec: frames, method arguments, field tables, content headers.

Only the subset beholder and its test broker need (connection, channel,
exchange, queue, basic, confirm classes). Spec: AMQP 0-9-1 (RabbitMQ
flavour: ``l`` is int64 in field tables, ``x`` is a byte array).

The reference reaches RabbitMQ through triton-core → amqplib 0.5.5
(yarn.lock:111-121); no AMQP library is installed here, so this is a
from-scratch implementation of the protocol itself.
"""
from __future__ import annotations

import datetime
import decimal
import struct
from typing import Any, Dict, List, Optional, Tuple

PROTOCOL_HEADER = b"AMQP\x00\x00\x09\x01"

FRAME_METHOD = 1
FRAME_HEADER = 2
FRAME_BODY = 3
FRAME_HEARTBEAT = 8
FRAME_END = 0xCE
FRAME_MIN_SIZE = 4096

REPLY_SUCCESS = 200
CONTENT_TOO_LARGE = 311
NO_ROUTE = 312
NO_CONSUMERS = 313
CONNECTION_FORCED = 320
INVALID_PATH = 402
ACCESS_REFUSED = 403
NOT_FOUND = 404
RESOURCE_LOCKED = 405
PRECONDITION_FAILED = 406
FRAME_ERROR = 501
SYNTAX_ERROR = 502
COMMAND_INVALID = 503
CHANNEL_ERROR = 504
UNEXPECTED_FRAME = 505
NOT_IMPLEMENTED = 540
INTERNAL_ERROR = 541


class AmqpError(Exception):
    """Protocol or broker error (``reply_code``/``reply_text`` from a close method)."""

    def __init__(self, message: str, reply_code: int = 0, class_id: int = 0, method_id: int = 0):
        super().__init__(message)
        self.reply_code = reply_code
        self.class_id = class_id
        self.method_id = method_id


class FrameError(AmqpError):
    pass


# (class_id, method_id) -> (name, [(arg_name, type)], has_content)
_o, _s, _l, _L, _ss, _ls, _b, _t, _ts = ("octet", "short", "long", "longlong", "shortstr", "longstr", "bit",
                                         "table", "timestamp")
METHODS: Dict[Tuple[int, int], Tuple[str, List[Tuple[str, str]], bool]] = {
    (10, 10): ("connection.start", [("version_major", _o), ("version_minor", _o), ("server_properties", _t),
                                    ("mechanisms", _ls), ("locales", _ls)], False),
    (10, 11): ("connection.start_ok", [("client_properties", _t), ("mechanism", _ss), ("response", _ls),
                                       ("locale", _ss)], False),
    (10, 20): ("connection.secure", [("challenge", _ls)], False),
    (10, 21): ("connection.secure_ok", [("response", _ls)], False),
    (10, 30): ("connection.tune", [("channel_max", _s), ("frame_max", _l), ("heartbeat", _s)], False),
    (10, 31): ("connection.tune_ok", [("channel_max", _s), ("frame_max", _l), ("heartbeat", _s)], False),
    (10, 40): ("connection.open", [("virtual_host", _ss), ("capabilities", _ss), ("insist", _b)], False),
    (10, 41): ("connection.open_ok", [("known_hosts", _ss)], False),
    (10, 50): ("connection.close", [("reply_code", _s), ("reply_text", _ss), ("class_id", _s),
                                    ("method_id", _s)], False),
    (10, 51): ("connection.close_ok", [], False),
    (10, 60): ("connection.blocked", [("reason", _ss)], False),
    (10, 61): ("connection.unblocked", [], False),
    (20, 10): ("channel.open", [("out_of_band", _ss)], False),
    (20, 11): ("channel.open_ok", [("channel_id", _ls)], False),
    (20, 20): ("channel.flow", [("active", _b)], False),
    (20, 21): ("channel.flow_ok", [("active", _b)], False),
    (20, 40): ("channel.close", [("reply_code", _s), ("reply_text", _ss), ("class_id", _s),
                                 ("method_id", _s)], False),
    (20, 41): ("channel.close_ok", [], False),
    (40, 10): ("exchange.declare", [("ticket", _s), ("exchange", _ss), ("type", _ss), ("passive", _b),
                                    ("durable", _b), ("auto_delete", _b), ("internal", _b), ("nowait", _b),
                                    ("arguments", _t)], False),
    (40, 11): ("exchange.declare_ok", [], False),
    (40, 20): ("exchange.delete", [("ticket", _s), ("exchange", _ss), ("if_unused", _b), ("nowait", _b)], False),
    (40, 21): ("exchange.delete_ok", [], False),
    (50, 10): ("queue.declare", [("ticket", _s), ("queue", _ss), ("passive", _b), ("durable", _b),
                                 ("exclusive", _b), ("auto_delete", _b), ("nowait", _b), ("arguments", _t)], False),
    (50, 11): ("queue.declare_ok", [("queue", _ss), ("message_count", _l), ("consumer_count", _l)], False),
    (50, 20): ("queue.bind", [("ticket", _s), ("queue", _ss), ("exchange", _ss), ("routing_key", _ss),
                              ("nowait", _b), ("arguments", _t)], False),
    (50, 21): ("queue.bind_ok", [], False),
    (50, 30): ("queue.purge", [("ticket", _s), ("queue", _ss), ("nowait", _b)], False),
    (50, 31): ("queue.purge_ok", [("message_count", _l)], False),
    (50, 40): ("queue.delete", [("ticket", _s), ("queue", _ss), ("if_unused", _b), ("if_empty", _b),
                                ("nowait", _b)], False),
    (50, 41): ("queue.delete_ok", [("message_count", _l)], False),
    (60, 10): ("basic.qos", [("prefetch_size", _l), ("prefetch_count", _s), ("global_", _b)], False),
    (60, 11): ("basic.qos_ok", [], False),
    (60, 20): ("basic.consume", [("ticket", _s), ("queue", _ss), ("consumer_tag", _ss), ("no_local", _b),
                                 ("no_ack", _b), ("exclusive", _b), ("nowait", _b), ("arguments", _t)], False),
    (60, 21): ("basic.consume_ok", [("consumer_tag", _ss)], False),
    (60, 30): ("basic.cancel", [("consumer_tag", _ss), ("nowait", _b)], False),
    (60, 31): ("basic.cancel_ok", [("consumer_tag", _ss)], False),
    (60, 40): ("basic.publish", [("ticket", _s), ("exchange", _ss), ("routing_key", _ss), ("mandatory", _b),
                                 ("immediate", _b)], True),
    (60, 50): ("basic.return", [("reply_code", _s), ("reply_text", _ss), ("exchange", _ss),
                                ("routing_key", _ss)], True),
    (60, 60): ("basic.deliver", [("consumer_tag", _ss), ("delivery_tag", _L), ("redelivered", _b),
                                 ("exchange", _ss), ("routing_key", _ss)], True),
    (60, 70): ("basic.get", [("ticket", _s), ("queue", _ss), ("no_ack", _b)], False),
    (60, 71): ("basic.get_ok", [("delivery_tag", _L), ("redelivered", _b), ("exchange", _ss),
                                ("routing_key", _ss), ("message_count", _l)], True),
    (60, 72): ("basic.get_empty", [("cluster_id", _ss)], False),
    (60, 80): ("basic.ack", [("delivery_tag", _L), ("multiple", _b)], False),
    (60, 90): ("basic.reject", [("delivery_tag", _L), ("requeue", _b)], False),
    (60, 100): ("basic.recover_async", [("requeue", _b)], False),
    (60, 110): ("basic.recover", [("requeue", _b)], False),
    (60, 111): ("basic.recover_ok", [], False),
    (60, 120): ("basic.nack", [("delivery_tag", _L), ("multiple", _b), ("requeue", _b)], False),
    (85, 10): ("confirm.select", [("nowait", _b)], False),
    (85, 11): ("confirm.select_ok", [], False),
}
BY_NAME: Dict[str, Tuple[int, int]] = {v[0]: k for k, v in METHODS.items()}


class Method:
    """A decoded method frame: ``name``, ``class_id``, ``method_id`` and ``args`` (dict)."""

    __slots__ = ("class_id", "method_id", "name", "args")

    def __init__(self, class_id: int, method_id: int, args: Dict[str, Any]):
        self.class_id = class_id
        self.method_id = method_id
        self.name = METHODS[(class_id, method_id)][0]
        self.args = args

    def __getattr__(self, k):
        try:
            return self.args[k]
        except KeyError:
            raise AttributeError(k) from None

    @property
    def has_content(self) -> bool:
        return METHODS[(self.class_id, self.method_id)][2]

    def __repr__(self) -> str:
        return f"<{self.name} {self.args}>"


# ------------------------------------------------------------------ encoding --
def _enc_shortstr(s) -> bytes:
    b = s.encode("utf-8") if isinstance(s, str) else bytes(s or b"")
    if len(b) > 255:
        raise FrameError("shortstr longer than 255 bytes")
    return bytes([len(b)]) + b


def _enc_longstr(s) -> bytes:
    b = s.encode("utf-8") if isinstance(s, str) else bytes(s or b"")
    return struct.pack(">I", len(b)) + b


def _enc_field_value(v) -> bytes:
    if v is None:
        return b"V"
    if isinstance(v, bool):
        return b"t" + (b"\x01" if v else b"\x00")
    if isinstance(v, int):
        if -(2**31) <= v < 2**31:
            return b"I" + struct.pack(">i", v)
        return b"l" + struct.pack(">q", v)
    if isinstance(v, float):
        return b"d" + struct.pack(">d", v)
    if isinstance(v, decimal.Decimal):
        sign, digits, exp = v.as_tuple()
        places = max(0, -exp)
        raw = int(v.scaleb(places))
        return b"D" + struct.pack(">Bi", places, raw)
    if isinstance(v, str):
        return b"S" + _enc_longstr(v)
    if isinstance(v, (bytes, bytearray)):
        return b"x" + struct.pack(">I", len(v)) + bytes(v)
    if isinstance(v, datetime.datetime):
        return b"T" + struct.pack(">Q", int(v.timestamp()))
    if isinstance(v, dict):
        return b"F" + encode_table(v)
    if isinstance(v, (list, tuple)):
        body = b"".join(_enc_field_value(x) for x in v)
        return b"A" + struct.pack(">I", len(body)) + body
    raise FrameError(f"cannot encode field value of type {type(v).__name__}")


def encode_table(t: Optional[Dict[str, Any]]) -> bytes:
    if not t:
        return b"\x00\x00\x00\x00"
    body = b"".join(_enc_shortstr(k) + _enc_field_value(v) for k, v in t.items())
    return struct.pack(">I", len(body)) + body


def encode_args(spec: List[Tuple[str, str]], args: Dict[str, Any]) -> bytes:
    out = []
    bits: List[bool] = []

    def flush_bits():
        while bits:
            byte = 0
            for i, b in enumerate(bits[:8]):
                if b:
                    byte |= 1 << i
            out.append(bytes([byte]))
            del bits[:8]

    for name, typ in spec:
        v = args.get(name)
        if typ == "bit":
            bits.append(bool(v))
            continue
        flush_bits()
        if typ == "octet":
            out.append(struct.pack(">B", v or 0))
        elif typ == "short":
            out.append(struct.pack(">H", v or 0))
        elif typ == "long":
            out.append(struct.pack(">I", v or 0))
        elif typ in ("longlong", "timestamp"):
            out.append(struct.pack(">Q", v or 0))
        elif typ == "shortstr":
            out.append(_enc_shortstr(v or ""))
        elif typ == "longstr":
            out.append(_enc_longstr(v or b""))
        elif typ == "table":
            out.append(encode_table(v))
        else:  # pragma: no cover
            raise FrameError(f"unknown arg type {typ}")
    flush_bits()
    return b"".join(out)


def encode_method(channel: int, name: str, **args) -> bytes:
    cid, mid = BY_NAME[name]
    payload = struct.pack(">HH", cid, mid) + encode_args(METHODS[(cid, mid)][1], args)
    return struct.pack(">BHI", FRAME_METHOD, channel, len(payload)) + payload + b"\xce"


_ACK_FRAME = struct.Struct(">BHIHHQBB")  # method frame: basic.ack(delivery_tag, multiple)


def encode_ack(channel: int, delivery_tag: int, multiple: bool = False) -> bytes:
    """``basic.ack`` method frame (hot path: one per settled delivery or batch)."""
    return _ACK_FRAME.pack(FRAME_METHOD, channel, 13, 60, 80, delivery_tag, 1 if multiple else 0, 0xCE)


def encode_heartbeat() -> bytes:
    return b"\x08\x00\x00\x00\x00\x00\x00\xce"


# content header property flags (bit 15 first)
PROPS = [("content_type", "shortstr"), ("content_encoding", "shortstr"), ("headers", "table"),
         ("delivery_mode", "octet"), ("priority", "octet"), ("correlation_id", "shortstr"),
         ("reply_to", "shortstr"), ("expiration", "shortstr"), ("message_id", "shortstr"),
         ("timestamp", "timestamp"), ("type", "shortstr"), ("user_id", "shortstr"),
         ("app_id", "shortstr"), ("cluster_id", "shortstr")]


def encode_content(channel: int, class_id: int, body: bytes, properties: Optional[Dict[str, Any]],
                   frame_max: int) -> bytes:
    """Content header frame + body frames."""
    flags = 0
    parts = []
    props = properties or {}
    for i, (name, typ) in enumerate(PROPS):
        v = props.get(name)
        if v is None:
            continue
        flags |= 1 << (15 - i)
        parts.append(encode_args([(name, typ)], {name: v}))
    hdr = struct.pack(">HHQH", class_id, 0, len(body), flags) + b"".join(parts)
    out = [struct.pack(">BHI", FRAME_HEADER, channel, len(hdr)), hdr, b"\xce"]
    step = max(1, frame_max - 8)
    for off in range(0, len(body), step):
        chunk = body[off:off + step]
        out.append(struct.pack(">BHI", FRAME_BODY, channel, len(chunk)))
        out.append(chunk)
        out.append(b"\xce")
    return b"".join(out)


# ------------------------------------------------------------------ decoding --
class _Reader:
    __slots__ = ("b", "i")

    def __init__(self, b: bytes, i: int = 0):
        self.b = b
        self.i = i

    def take(self, n: int) -> bytes:
        j = self.i + n
        if j > len(self.b):
            raise FrameError("truncated method arguments", SYNTAX_ERROR)
        v = self.b[self.i:j]
        self.i = j
        return v

    def octet(self) -> int:
        return self.take(1)[0]

    def short(self) -> int:
        return struct.unpack(">H", self.take(2))[0]

    def long(self) -> int:
        return struct.unpack(">I", self.take(4))[0]

    def longlong(self) -> int:
        return struct.unpack(">Q", self.take(8))[0]

    def shortstr(self) -> str:
        n = self.octet()
        return self.take(n).decode("utf-8", "replace")

    def longstr(self) -> bytes:
        n = self.long()
        return self.take(n)

    def table(self) -> Dict[str, Any]:
        n = self.long()
        sub = _Reader(self.take(n))
        out = {}
        while sub.i < len(sub.b):
            k = sub.shortstr()
            out[k] = sub.field_value()
        return out

    def field_value(self):
        t = chr(self.octet())
        if t == "t":
            return self.octet() != 0
        if t == "b":
            return struct.unpack(">b", self.take(1))[0]
        if t == "B":
            return self.octet()
        if t == "s":
            return struct.unpack(">h", self.take(2))[0]
        if t == "u":
            return self.short()
        if t == "I":
            return struct.unpack(">i", self.take(4))[0]
        if t == "i":
            return self.long()
        if t == "l":
            return struct.unpack(">q", self.take(8))[0]
        if t == "L":
            return self.longlong()
        if t == "f":
            return struct.unpack(">f", self.take(4))[0]
        if t == "d":
            return struct.unpack(">d", self.take(8))[0]
        if t == "D":
            places = self.octet()
            raw = struct.unpack(">i", self.take(4))[0]
            return decimal.Decimal(raw).scaleb(-places)
        if t == "S":
            v = self.longstr()
            try:
                return v.decode("utf-8")
            except UnicodeDecodeError:
                return v
        if t == "x":
            return self.longstr()
        if t == "A":
            n = self.long()
            sub = _Reader(self.take(n))
            out = []
            while sub.i < len(sub.b):
                out.append(sub.field_value())
            return out
        if t == "T":
            return datetime.datetime.fromtimestamp(self.longlong(), datetime.timezone.utc)
        if t == "F":
            return self.table()
        if t == "V":
            return None
        raise FrameError(f"unknown field type {t!r}", SYNTAX_ERROR)


def decode_args(spec: List[Tuple[str, str]], payload: bytes, offset: int = 4) -> Dict[str, Any]:
    r = _Reader(payload, offset)
    out: Dict[str, Any] = {}
    bit_byte = 0
    bit_idx = 8
    for name, typ in spec:
        if typ == "bit":
            if bit_idx >= 8:
                bit_byte = r.octet()
                bit_idx = 0
            out[name] = bool(bit_byte & (1 << bit_idx))
            bit_idx += 1
            continue
        bit_idx = 8
        if typ == "octet":
            out[name] = r.octet()
        elif typ == "short":
            out[name] = r.short()
        elif typ == "long":
            out[name] = r.long()
        elif typ in ("longlong", "timestamp"):
            out[name] = r.longlong()
        elif typ == "shortstr":
            out[name] = r.shortstr()
        elif typ == "longstr":
            out[name] = r.longstr()
        elif typ == "table":
            out[name] = r.table()
    return out


def decode_method(payload: bytes) -> Method:
    if len(payload) < 4:
        raise FrameError("method frame too short", FRAME_ERROR)
    cid, mid = struct.unpack_from(">HH", payload)
    spec = METHODS.get((cid, mid))
    if spec is None:
        raise AmqpError(f"unknown method {cid}.{mid}", NOT_IMPLEMENTED, cid, mid)
    return Method(cid, mid, decode_args(spec[1], payload))


def decode_content_header(payload: bytes) -> Tuple[int, int, Dict[str, Any]]:
    """Returns ``(class_id, body_size, properties)``."""
    if len(payload) < 14:
        raise FrameError("content header too short", FRAME_ERROR)
    class_id, _weight, size, flags = struct.unpack_from(">HHQH", payload)
    r = _Reader(payload, 14)
    props: Dict[str, Any] = {}
    if flags:
        for i, (name, typ) in enumerate(PROPS):
            if flags & (1 << (15 - i)):
                if typ == "shortstr":
                    props[name] = r.shortstr()
                elif typ == "table":
                    props[name] = r.table()
                elif typ == "octet":
                    props[name] = r.octet()
                else:
                    props[name] = r.longlong()
    return class_id, size, props


class FrameParser:
    """Incremental frame splitter: ``feed(bytes)`` → list of ``(type, channel, payload)``."""

    def __init__(self, frame_max: int = 131072):
        self.buf = bytearray()
        self.frame_max = frame_max

    def feed(self, data: bytes) -> List[Tuple[int, int, bytes]]:
        buf = self.buf
        buf += data
        out = []
        i = 0
        n = len(buf)
        while n - i >= 7:
            ftype, ch, size = struct.unpack_from(">BHI", buf, i)
            if self.frame_max and size > self.frame_max:
                raise FrameError(f"frame of {size} bytes exceeds frame_max {self.frame_max}", FRAME_ERROR)
            end = i + 7 + size
            if end + 1 > n:
                break
            if buf[end] != FRAME_END:
                raise FrameError("missing frame-end octet", FRAME_ERROR)
            out.append((ftype, ch, bytes(buf[i + 7:end])))
            i = end + 1
        if i:
            del buf[:i]
        return out


def parse_url(url: str) -> Dict[str, Any]:
    """``amqp://user:pass@host:port/vhost?heartbeat=60&frame_max=131072``."""
    from urllib.parse import parse_qs, unquote, urlsplit
    u = urlsplit(url)
    if u.scheme not in ("amqp", "amqps"):
        raise ValueError(f"not an AMQP URL: {url!r}")
    vhost = unquote(u.path[1:]) if u.path and u.path != "/" else "/"
    q = {k: v[-1] for k, v in parse_qs(u.query).items()}
    return {
        "host": u.hostname or "localhost",
        "port": u.port or (5671 if u.scheme == "amqps" else 5672),
        "user": unquote(u.username) if u.username else "guest",
        "password": unquote(u.password) if u.password else "guest",
        "vhost": vhost,
        "heartbeat": int(q.get("heartbeat", 60)),
        "frame_max": int(q.get("frame_max", 131072)),
        "channel_max": int(q.get("channel_max", 2047)),
        "ssl": u.scheme == "amqps",
        # TLS options (amqps): ?cafile=/path/ca.pem&certfile=..&keyfile=..&verify=false&server_name=host
        "cafile": q.get("cafile"),
        "certfile": q.get("certfile"),
        "keyfile": q.get("keyfile"),
        "verify": q.get("verify", "true").lower() not in ("false", "0", "no"),
        "server_name": q.get("server_name"),
    }
