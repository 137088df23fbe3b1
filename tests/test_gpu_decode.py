"""The HIP batched decode (ops/hip/telemetry_decode.hip, ops/gpu_decode.py), the GPU-offload probe.

CPU tests pin the plain-Python row definitions to the service's own codecs: ``reference_decode``
to the upb codec on valid messages, ``reference_decode_pbjs`` to the protobufjs codec (the one
the service runs, handlers._dialect) on valid AND malformed messages. GPU tests compare the
kernel's table against both references and, in the protobufjs dialect, against the service's
codec itself on a corpus of valid, truncated, wrong-wire-type, field-0 and random bodies."""
from __future__ import annotations

import random

import pytest
from hypothesis import given, settings, strategies as st

from beholder_amd import ops
from beholder_amd.bench.generator import Workload
from beholder_amd.models import proto

np = pytest.importorskip("numpy")  # the probe's host tables are numpy; the service never imports it
from beholder_amd.ops import gpu_decode as gd  # noqa: E402

PROGRESS = ops.codec_for(proto.load("api.TelemetryProgress"))
STATUS = ops.codec_for(proto.load("api.TelemetryStatus"))
PROGRESS_PBJS = ops.codec_for(proto.load("api.TelemetryProgress"), "protobufjs")


def _pbjs_values(bodies) -> list:
    """The service's decode of each body: (mediaId, status, progress, host), None on DecodeError."""
    out = []
    for b in bodies:
        try:
            m = PROGRESS_PBJS.decode(b)
        except proto.DecodeError:
            out.append(None)
        else:
            out.append((m.mediaId, m.status, m.progress, m.host))
    return out


messages = st.builds(
    lambda mid, status, progress, host: PROGRESS.encode(
        {"mediaId": mid, "status": status, "progress": progress, "host": host}),
    st.text(max_size=40), st.integers(0, 5), st.integers(-2 ** 31, 2 ** 31 - 1), st.text(max_size=12))


def _fields(buf: bytes, row) -> tuple:
    io, il, status, progress, ho, hl, ok, _ = (int(x) for x in row)
    return buf[io:io + il].decode(), status, progress, buf[ho:ho + hl].decode(), ok


@settings(max_examples=300, deadline=None)
@given(st.lists(messages, min_size=1, max_size=6))
def test_reference_row_matches_the_service_codec(bodies):
    buf, offs = gd.pack(bodies)
    for k, b in enumerate(bodies):
        m = PROGRESS.decode(b)
        row = gd.reference_decode(buf, int(offs[k]), int(offs[k + 1]))
        assert _fields(buf, row) == (m.mediaId, m.status, m.progress, m.host, 1)


@settings(max_examples=300, deadline=None)
@given(st.lists(st.binary(max_size=24), max_size=6))
def test_reference_never_reads_past_its_message(bodies):
    buf, offs = gd.pack(bodies)
    for k in range(len(bodies)):
        io, il, _, _, ho, hl, _, _ = gd.reference_decode(buf, int(offs[k]), int(offs[k + 1]))
        for off, ln in ((io, il), (ho, hl)):
            assert ln == 0 or offs[k] <= off and off + ln <= offs[k + 1]


def test_native_materialise_gives_the_codec_values():
    bodies = [b for _, b in Workload(n_media=8, seed=2).events(200)] + [b"\xff", b""]
    buf, _ = gd.pack(bodies)
    got = gd.materialise(buf, gd.reference_table(bodies))
    for b, row in zip(bodies[:200], got):
        m = PROGRESS.decode(b)
        assert row == (m.mediaId, m.status, m.progress, m.host)
    assert got[200] is None and got[201] == ("", 0, 0, "")
    bad = gd.reference_table(bodies[:1])
    bad[0, 1] = len(buf) + 1
    with pytest.raises(ValueError, match="outside"):
        gd.materialise(buf, bad)


def test_layout_guards_and_loud_missing_library(monkeypatch):
    buf, offs = gd.pack([b"\n\x01a", b""])
    gd.check_layout(len(buf), offs)
    for bad in (np.array([1, 3, 3], np.int32), np.array([0, 3, 2], np.int32), np.array([0, 2, 2], np.int32),
                np.array([0, 3, 3], np.int64)):
        with pytest.raises(ValueError):
            gd.check_layout(len(buf), bad)
    monkeypatch.setattr(gd, "LIB_PATH", "/nonexistent/libbeholder_hip.so")
    monkeypatch.setattr(gd, "_lib", None)
    with pytest.raises(RuntimeError, match="missing"):
        gd.lib()


def _corpus(rng: random.Random) -> list:
    w = Workload(n_media=64, seed=5)
    bodies = [b for _, b in w.events(3000)]
    bodies += [STATUS.encode({"mediaId": f"m{i}", "status": i % 7}) for i in range(200)]
    for _ in range(500):  # truncations, garbage, unknown fields, empty
        b = rng.choice(bodies)
        bodies.append(b[:rng.randrange(len(b) + 1)])
        bodies.append(bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 30))))
        bodies.append(b + bytes([0x28, rng.randrange(128), 0x35, 1, 2, 3, 4, 0x39]) + bytes(8))
    bodies += _malformed(rng)
    bodies.append(b"")
    return bodies


def _malformed(rng: random.Random) -> list:
    """Where protobufjs and upb disagree: field 0, known fields with the wrong wire type, strings
    running past the end (clamped by protobufjs), 5-byte and overlong varints, groups, invalid
    UTF-8, and a tag varint truncated in its 5th byte."""
    out = [
        b"\x00\x05",                         # field 0 (varint): skipped by protobufjs, an error for upb
        b"\x02\x01x\x0a\x02ok",             # field 0 length-delimited, then mediaId
        b"\x08\x07",                         # mediaId tagged as a varint: read as a string of length 7
        b"\x10\x03abc",                      # ... status tagged fine
        b"\x15\x05\x00\x00\x00",           # status with wire type 5: read as a varint anyway
        b"\x1a\x2a",                         # progress with wire type 2: varint 42
        b"\x0a\x7fabc",                      # mediaId of 127 bytes in a 5-byte body: clamped
        b"\x22\xff\xff\xff\xff\x0fhost",  # host length 2^32-1: clamped
        b"\x18\xff\xff\xff\xff\xff\x01\x00\x00\x00\x00",  # 10-byte progress varint
        b"\x18\xff\xff\xff\xff\xff",       # ... truncated inside the unchecked tail
        b"\x80\x80\x80\x80\x80",           # 5-byte tag with continuation: tail past the end
        b"\x2b\x08\x01\x2c\x0a\x01z",     # a group (field 5) around a varint, then mediaId
        b"\x2b\x33\x08\x01\x34\x2c",      # nested groups
        b"\x2c",                              # end-group with nothing open
        b"\x2e", b"\x2f\x00",                # wire types 6 / 7
        b"\x0a\x03\xff\xfe\xfd",           # invalid UTF-8 (protobufjs: U+FFFD)
        b"\x0a\x02ab\x0a\x01c\x10\x01\x10\x02",  # repeated scalars: last wins
        b"\x39" + bytes(7),                   # unknown fixed64 one byte short
        b"\x3d\x01\x02\x03",                # unknown fixed32 one byte short
    ]
    for _ in range(400):  # random bodies built from tags of every field number 0-6 and wire type
        b = bytearray()
        for _ in range(rng.randrange(1, 6)):
            b.append((rng.randrange(7) << 3) | rng.randrange(8))
            b += bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 6)))
        out.append(bytes(b))
    return out


def test_pbjs_reference_row_matches_the_service_codec():
    """reference_decode_pbjs (the kernel's protobufjs dialect, in Python) gives exactly what the
    service's protobufjs codec gives, malformed input included: ok == 0 where it raises."""
    bodies = _corpus(random.Random(11))
    buf, _ = gd.pack(bodies)
    got = gd.materialise(buf, gd.reference_table(bodies, dialect="protobufjs"))
    want = _pbjs_values(bodies)
    diffs = [(bodies[i], got[i], want[i]) for i in range(len(bodies)) if got[i] != want[i]]
    assert not diffs, diffs[:5]
    assert sum(v is None for v in want) > 100  # the corpus does reach the error branches
    # and the two dialects really do differ on this corpus
    assert np.any(gd.reference_table(bodies, "upb")[:, 6] != gd.reference_table(bodies, "protobufjs")[:, 6])


@pytest.mark.gpu
def test_kernel_pbjs_matches_the_service_codec_on_malformed_input():
    """The kernel's default dialect is the service's: on valid, truncated, wrong-wire-type, field-0
    and random bodies its rows materialise to exactly what codec_for(..., "protobufjs") decodes,
    None exactly where that codec raises DecodeError."""
    bodies = _corpus(random.Random(11))
    got = gd.decode_bodies(bodies)  # default dialect: protobufjs
    want = gd.reference_table(bodies, "protobufjs")
    bad = np.nonzero(np.any(got != want, axis=1))[0]
    assert len(bad) == 0, [(bodies[i], got[i].tolist(), want[i].tolist()) for i in bad[:5]]
    buf, _ = gd.pack(bodies)
    rows = gd.materialise(buf, got)
    values = _pbjs_values(bodies)
    diffs = [(bodies[i], rows[i], values[i]) for i in range(len(bodies)) if rows[i] != values[i]]
    assert not diffs, diffs[:5]


@pytest.mark.gpu
def test_kernel_matches_reference_on_valid_random_and_truncated_messages():
    bodies = _corpus(random.Random(11))
    got = gd.decode_bodies(bodies, dialect="upb")
    want = gd.reference_table(bodies)
    assert got.shape == want.shape == (len(bodies), 8)
    bad = np.nonzero(np.any(got != want, axis=1))[0]
    assert len(bad) == 0, [(bodies[i], got[i].tolist(), want[i].tolist()) for i in bad[:5]]
    assert want[:3000, 6].all()  # the workload's messages all decode


@pytest.mark.gpu
def test_kernel_large_batch_and_argument_checks():
    import torch
    w = Workload(n_media=256, seed=9)
    bodies = [b for _, b in w.events(200_000)]
    got = gd.decode_bodies(bodies)
    buf, offs = gd.pack(bodies)
    sample = range(0, len(bodies), 997)
    for k in sample:
        assert got[k].tolist() == gd.reference_decode_pbjs(buf, int(offs[k]), int(offs[k + 1]))
    assert np.array_equal(got, gd.decode_bodies(bodies, dialect="upb"))  # valid input: dialects agree
    assert got[:, 6].all()
    dev = torch.zeros(4, dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        gd.decode_batch(dev, torch.zeros(3, dtype=torch.int64, device="cuda"), 2)
    with pytest.raises(ValueError):
        gd.decode_batch(dev.cpu(), torch.zeros(3, dtype=torch.int32), 2)
    assert gd.decode_batch(dev, torch.zeros(1, dtype=torch.int32, device="cuda"), 0).shape == (0, 8)
    with pytest.raises(ValueError):
        gd.decode_batch(dev, torch.zeros(1, dtype=torch.int32, device="cuda"), 0, dialect="proto2")


@pytest.mark.gpu
def test_kernel_long_fields_and_mixed_sizes():
    """Multi-byte length varints (fields of 128 bytes and up, one of 40,000) at every alignment."""
    rng = random.Random(3)
    bodies = [PROGRESS.encode({"mediaId": "x" * rng.randrange(0, 400), "status": 2, "progress": k,
                               "host": "h" * rng.randrange(0, 40)}) for k in range(3000)]
    bodies[700] = PROGRESS.encode({"mediaId": "y" * 40000, "status": 4})
    got = gd.decode_bodies(bodies)
    assert np.array_equal(got, gd.reference_table(bodies, "protobufjs"))
    assert np.array_equal(got, gd.reference_table(bodies))
