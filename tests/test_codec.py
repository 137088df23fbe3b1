"""Native protobuf codec vs the upb (google.protobuf) oracle.

The reference decodes with protobufjs via triton-core (index.js:63,129); our
hot path uses the native MessageCodec. It must agree with upb on every valid
input (same field values) and reject the same malformed inputs.
"""
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from beholder_amd.models import proto
from beholder_amd.models.proto import DecodeError
from beholder_amd.models.protoparse import parse_proto
from beholder_amd.ops import MessageCodec, codec_for, field_table

STATUS = proto.load("api.TelemetryStatus")
PROGRESS = proto.load("api.TelemetryProgress")
MEDIA = proto.load("api.Media")


def as_tuple(ptype, msg):
    return tuple(getattr(msg, f.name) for f in ptype.descriptor.fields)


def test_schema_field_numbers_pinned():
    """The documented wire contract (models/proto/api.proto)."""
    assert field_table(STATUS.descriptor) == [(1, "mediaId", 1), (2, "status", 10)]
    assert field_table(PROGRESS.descriptor) == [(1, "mediaId", 1), (2, "status", 10), (3, "progress", 3),
                                                (4, "host", 1)]
    assert [f.name for f in MEDIA.descriptor.fields][:4] == ["id", "name", "creator", "creatorId"]


def test_enum_semantics():
    """index.js:74,94,134,142: enumToString / stringToEnum; CreatorType.TRELLO == 1."""
    assert proto.enum_to_string(STATUS, "TelemetryStatusEntry", 4) == "DEPLOYED"
    assert proto.enumToString(PROGRESS, "TelemetryStatusEntry", 0) == "QUEUED"
    assert proto.enum_to_string(STATUS, "TelemetryStatusEntry", 99) is None  # undefined (Q6)
    assert proto.string_to_enum(STATUS, "TelemetryStatusEntry", "DEPLOYED") == 4
    assert proto.stringToEnum(MEDIA, "CreatorType", "TRELLO") == 1
    assert proto.string_to_enum(MEDIA, "CreatorType", "NOPE") is None


def test_proto3_defaults():
    for codec_dec in (codec_for(PROGRESS).decode, lambda b: proto.decode(PROGRESS, b)):
        m = codec_dec(b"")
        assert (m.mediaId, m.status, m.progress, m.host) == ("", 0, 0, "")


def test_roundtrip_matches_upb():
    c = codec_for(PROGRESS)
    for vals in [("m", 4, 45, "h"), ("", 0, 0, ""), ("é✓", 5, -7, "w" * 300), ("x" * 70000, 2, 2**31 - 1, "")]:
        native_bytes = c.encode(vals)
        upb_bytes = proto.encode(PROGRESS, dict(zip(("mediaId", "status", "progress", "host"), vals)))
        assert native_bytes == upb_bytes
        assert tuple(c.decode(upb_bytes)) == vals


def test_unknown_fields_and_wire_type_mismatch_skipped():
    c = codec_for(STATUS)
    # field 9 varint (unknown), field 2 as LEN (wrong wire type -> unknown), then real status
    data = b"\x48\x05" + b"\x12\x01x" + b"\x0a\x02ab" + b"\x10\x03"
    assert tuple(c.decode(data)) == ("ab", 3)
    assert as_tuple(STATUS, proto.decode(STATUS, data)) == ("ab", 3)


def test_last_value_wins():
    c = codec_for(STATUS)
    data = b"\x0a\x01a\x10\x01\x0a\x01b\x10\x02"
    assert tuple(c.decode(data)) == ("b", 2) == as_tuple(STATUS, proto.decode(STATUS, data))


def test_group_skipping():
    c = codec_for(STATUS)
    # unknown group field 5 containing a varint field 1, then mediaId
    data = b"\x2b\x08\x01\x2c" + b"\x0a\x01z"
    assert tuple(c.decode(data)) == ("z", 0)
    assert as_tuple(STATUS, proto.decode(STATUS, data)) == ("z", 0)


@pytest.mark.parametrize("bad", [
    b"\x0a\x05ab",            # truncated string
    b"\x0a",                  # truncated length
    b"\x10",                  # truncated varint
    b"\x10\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\x01",  # > 10-byte varint
    b"\x00\x01",              # field number 0
    b"\x0e\x01",              # wire type 6
    b"\x0c",                  # stray end-group
    b"\x0a\x02\xff\xfe",      # invalid UTF-8 in a proto3 string
    b"\x2b\x08\x01",          # unterminated group
])
def test_malformed_rejected_by_both(bad):
    with pytest.raises(DecodeError):
        codec_for(STATUS).decode(bad)
    with pytest.raises(DecodeError):
        proto.decode(STATUS, bad)


def test_negative_int32_is_10_byte_varint():
    c = codec_for(PROGRESS)
    b = c.encode({"progress": -1})
    assert b == b"\x18" + b"\xff" * 9 + b"\x01"
    assert c.decode(b).progress == -1 == proto.decode(PROGRESS, b).progress


def test_int32_truncation_of_large_varint():
    """A 64-bit varint on an int32 field keeps the low 32 bits (upb semantics)."""
    data = b"\x18\x80\x80\x80\x80\x10"  # 2**32 -> low 32 bits = 0
    assert codec_for(PROGRESS).decode(data).progress == proto.decode(PROGRESS, data).progress == 0


def test_all_scalar_kinds_against_upb():
    src = """
    syntax = "proto3";
    package t;
    enum E { A = 0; B = 1; }
    message All {
      string s = 1; bytes b = 2; int32 i32 = 3; int64 i64 = 4; uint32 u32 = 5; uint64 u64 = 6;
      sint32 s32 = 7; sint64 s64 = 8; bool bo = 9; E e = 10; float f = 11; double d = 12;
      fixed32 f32 = 13; fixed64 f64 = 14; sfixed32 sf32 = 15; sfixed64 sf64 = 16;
    }
    """
    from google.protobuf import descriptor_pool, message_factory
    pool = descriptor_pool.DescriptorPool()
    pool.Add(parse_proto(src, "t.proto"))
    desc = pool.FindMessageTypeByName("t.All")
    cls = message_factory.GetMessageClass(desc)
    codec = MessageCodec("t.All", field_table(desc))
    vals = dict(s="héllo", b=b"\x00\xff", i32=-5, i64=-(2**40), u32=2**32 - 1, u64=2**64 - 1, s32=-77,
                s64=-(2**50), bo=True, e=1, f=1.5, d=-2.25, f32=7, f64=2**63, sf32=-8, sf64=-(2**62))
    upb = cls(**vals).SerializeToString()
    dec = codec.decode(upb)
    for k, v in vals.items():
        assert getattr(dec, k) == v, k
    assert codec.encode(vals) == upb
    # the reference's reader (protobufjs 6.8.8 dialect, ops/csrc/pbjs.hpp) reads the kinds it models
    # alike: length-delimited bytes, fixed32 / float, fixed64 / double (64-bit integers it refuses)
    with pytest.raises(ValueError, match="64-bit integer"):
        MessageCodec("t.All", field_table(desc), "protobufjs")
    keep = [f for f in field_table(desc) if f[1] in ("s", "b", "i32", "u32", "s32", "bo", "e", "f", "d", "f32", "sf32")]
    pbjs = MessageCodec("t.All", keep, "protobufjs")
    assert pbjs.dialect == "protobufjs" and pbjs.type_name == "t.All" and codec.type_name == "t.All"
    small = {k: vals[k] for k in ("s", "b", "i32", "u32", "s32", "bo", "e", "f", "d", "f32", "sf32")}
    data = cls(**small).SerializeToString()
    dec = pbjs.decode(data)
    for k, v in small.items():
        assert getattr(dec, k) == v, k
    for bad in (b"\x6d\x01\x02", b"\x61\x01\x02\x03", b"\x12\x05ab"):  # fixed32 / double / bytes cut short
        with pytest.raises(Exception):
            pbjs.decode(bad)


# ------------------------------------------------------------- fuzzing ----
int32s = st.integers(min_value=-(2**31), max_value=2**31 - 1)


@settings(max_examples=300, deadline=None)
@given(st.text(max_size=64), int32s, int32s, st.text(max_size=16))
def test_fuzz_roundtrip(mid, status, prog, host):
    c = codec_for(PROGRESS)
    b = proto.encode(PROGRESS, {"mediaId": mid, "status": status, "progress": prog, "host": host})
    assert tuple(c.decode(b)) == (mid, status, prog, host)
    assert c.encode((mid, status, prog, host)) == b


@settings(max_examples=1500, deadline=None)
@given(st.binary(max_size=48))
def test_fuzz_arbitrary_bytes_agree_with_upb(data):
    """On random bytes the native codec accepts exactly what upb accepts, with equal values."""
    c = codec_for(PROGRESS)
    try:
        want = as_tuple(PROGRESS, proto.decode(PROGRESS, data))
    except DecodeError:
        want = None
    try:
        got = tuple(c.decode(data))
    except DecodeError:
        got = None
    assert got == want


@pytest.mark.parametrize("data", [
    b"\x60" + b"\x80" * 9 + b"\x02",          # unknown varint, overflow bits in the 10th byte
    b"\x60" + b"\x80" * 9 + b"\x7f",
    b"\x18" + b"\x80" * 9 + b"\x02",          # known int32 field, same
    b"\x18" + b"\xff" * 9 + b"\x01",
    b"\xe0\x80\x80\x80\x80\x00\x00",          # 6-byte encoding of a small tag
    b"\xe0\x80\x80\x80\x00\x00",              # 5-byte encoding of a small tag
    b"\x80\x80\x80\x80\x10\x00",              # tag wider than 32 bits
    b"\xe0\x00\x80\x80\x80\x80\x80\x80\x80\x80\x80\x02\x08\x00\x08\x00\r\x00\x00\x00\x00",  # fuzz find
    bytes.fromhex("3b003a983f2e3c"),          # field number 0 inside a skipped group: tolerated
    bytes.fromhex("3b03043c"),                # nested group with field number 0
    bytes.fromhex("3b1b0c3c"),                # mismatched nested end group
])
def test_varint_edge_cases_agree_with_upb(data):
    """Fuzzing found that upb keeps only bit 63 of a 10-byte varint (no error) and caps tags
    at 5 bytes; the native reader follows both rules."""
    c = codec_for(PROGRESS)
    try:
        m = proto.decode(PROGRESS, data)
        want = (m.mediaId, m.status, m.progress, m.host)
    except DecodeError:
        want = None
    try:
        got = tuple(c.decode(data))
    except DecodeError:
        got = None
    assert got == want


# protobufjs 6.8.8 dialect (ops/csrc/pbjs.hpp): what the reference's reader does with malformed input.
# Each vector is worked by hand from protobufjs's reader.js / reader_buffer.js; the node oracle
# (tests/test_reference_oracle.py) checks the same reader against a JS re-implementation.
PBJS_VECTORS = [
    (b"\x0a\x03abc\x10\x04\x18\x05", ("abc", 4, 5, "")),
    (b"\x80", "index out of range: 1 + 10 > 1"),             # uint32 reads past the end, then +5
    (b"\x0a\x05ab", ("ab", 0, 0, "")),                       # BufferReader.string clamps
    (b"\x0c", "index out of range: 1 + 10 > 1"),             # known field: no wire-type check
    (b"\x11ab", "index out of range: 3 + 10 > 3"),           # status read as varint, 'b' is a tag
    (b"\x1d\x01", ("", 0, 1, "")),                           # progress (int32) despite wire type 5
    (b"\x0a\x03\xff\xfeA", ("��A", 0, 0, "")),     # no UTF-8 validation
    (b"\x10\xff\xff\xff\xff\xff\x00\x00\x00\x00\x00", ("", -1, 0, "")),
    (b"\x10\xff\xff\xff\xff\xff\x00\x00", "index out of range: 8 + 10 > 8"),
    (b"\x00\x00\x18\x02", ("", 0, 2, "")),                   # field 0 skipped like any unknown field
    (b"\x2c", "invalid wire type 4 at offset 1"),            # stray end group
    (b"\x2e", "invalid wire type 6 at offset 1"),
    (b"\x2b\x33\x08\x01\x34\x3c\x18\x09", ("", 0, 9, "")),  # nested groups end on any end-group tag
    (b"\x2b\x33\x08\x01\x34", "index out of range: 5 + 10 > 5"),
    (b"\x29\x01\x02", "index out of range: 1 + 8 > 3"),      # unknown fixed64: skip(8)
    (b"\x2a\x05ab", "index out of range: 2 + 5 > 4"),        # unknown bytes: skip(n)
    (b"\x28\x80", "index out of range: 2 + 1 > 2"),          # unknown varint: skip()
]


@pytest.mark.parametrize("data,want", PBJS_VECTORS)
def test_protobufjs_dialect_vectors(data, want):
    c = codec_for(PROGRESS, "protobufjs")
    assert c.dialect == "protobufjs"
    if isinstance(want, str):
        with pytest.raises(DecodeError) as ei:
            c.decode(data)
        assert str(ei.value) == want
    else:
        assert tuple(c.decode(data)) == want


@settings(max_examples=300, deadline=None)
@given(st.text(max_size=40), st.integers(-2**31, 2**31 - 1), st.integers(-2**31, 2**31 - 1), st.text(max_size=20))
def test_protobufjs_dialect_agrees_with_upb_on_valid_input(mid, status, progress, host):
    data = codec_for(PROGRESS).encode((mid, status, progress, host))
    assert tuple(codec_for(PROGRESS, "protobufjs").decode(data)) == tuple(codec_for(PROGRESS).decode(data))


def test_handlers_decode_with_the_configured_dialect():
    import helpers
    r = helpers.Rig()
    assert r.h.decode_status.__self__.dialect == "protobufjs"
    r2 = helpers.Rig(config=helpers.cfg({"service": {"proto": {"dialect": "upb"}}}))
    assert r2.h.decode_status.__self__.dialect == "upb"


def test_decoded_messages_release_their_type_and_fields():
    """Decoded messages are made without CPython's per-object struct-sequence size lookups
    (py_codec.cpp new_result / result_dealloc): every one still holds and releases one
    reference to its type and its fields, and behaves as the struct sequence it is."""
    import gc
    import sys
    for dialect in ("upb", "protobufjs"):
        c = codec_for(PROGRESS, dialect)
        body = proto.encode(PROGRESS, {"mediaId": "m-1", "status": 2, "progress": 7, "host": "worker-1"})
        tp = type(c.decode(body))
        r0 = sys.getrefcount(tp)
        ms = [c.decode(body) for _ in range(500)]
        assert sys.getrefcount(tp) == r0 + 500
        host = ms[0].host
        hr = sys.getrefcount(host)
        del ms
        assert sys.getrefcount(tp) == r0
        assert sys.getrefcount(host) == hr - 1  # the last message holding it is gone
        m = c.decode(body)
        assert not gc.is_tracked(m)  # as PyStructSequence_New leaves it (atoms only)
        assert m == ("m-1", 2, 7, "worker-1") and tuple(m) == ("m-1", 2, 7, "worker-1") and len(m) == 4
        assert (m.mediaId, m[1], m.progress, m[-1]) == ("m-1", 2, 7, "worker-1")
        assert repr(m) == "api.TelemetryProgress(mediaId='m-1', status=2, progress=7, host='worker-1')"
