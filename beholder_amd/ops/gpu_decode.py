"""Batched telemetry decode on the GPU (``ops/hip/telemetry_decode.hip``): the offload probe.

The service decodes each event on the CPU as it arrives (``ops/csrc/py_codec.cpp``; the
``decode`` of index.js:63,129). This module is the measured alternative. It packs a batch of
message bodies, copies it to the device, decodes every message in one kernel (one lane per
message) and returns an ``(n, 8)`` int32 table:
``[id_off, id_len, status, progress, host_off, host_len, ok, fields_seen]``.

The kernel reads in either of the CPU codec's dialects (``ops.DIALECTS``). The default is
``protobufjs``, the reader the service itself runs (``handlers._dialect``, ``csrc/pbjs.hpp``), so
on malformed input the kernel agrees with production: ``ok == 0`` exactly where
``codec_for(ptype, "protobufjs").decode`` raises, and the same field values everywhere else.

``scripts/gpu_offload_probe.py`` prices this path against the CPU decode; docs/DESIGN.md
("Why there are no HIP kernels") cites the result. :func:`reference_decode` (upb) and
:func:`reference_decode_pbjs` are plain-Python definitions of the table; the GPU tests compare
the kernel against them and against the service's own protobufjs codec.

The extension is built in-tree by ``beholder_amd._build.build_hip`` (hipcc, gfx950) and loaded
with ctypes after ``import torch``. torch's HIP runtime has the same soname, so the kernel
launches on torch's runtime and stream. A missing library raises; there is no CPU fallback
behind :func:`decode_batch`.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence, Tuple

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hip", "libbeholder_hip.so")
FIELDS = ("id_off", "id_len", "status", "progress", "host_off", "host_len", "ok", "seen")
DIALECT_IDS = {"upb": 0, "protobufjs": 1}  # the kernel's DIALECT_* constants
_lib = None


def lib() -> ctypes.CDLL:
    """The HIP extension (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m beholder_amd.ops.build`")
        import torch  # noqa: F401  load torch's libamdhip64 first so the kernel shares its runtime
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.bh_decode_telemetry.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_int]
        _lib.bh_decode_telemetry.restype = ctypes.c_int
    return _lib


def pack(bodies: Sequence[bytes]) -> Tuple[bytes, np.ndarray]:
    """Concatenated bodies and their ``n + 1`` int32 boundaries."""
    offs = np.zeros(len(bodies) + 1, dtype=np.int32)
    np.cumsum([len(b) for b in bodies], out=offs[1:])
    return b"".join(bodies), offs


def check_layout(nbytes: int, offs: np.ndarray) -> None:
    """The kernel trusts ``offs``: validate it on the host before any launch."""
    if offs.ndim != 1 or offs.dtype != np.int32 or len(offs) < 1:
        raise ValueError("offs must be a 1-D int32 array of n + 1 boundaries")
    if offs[0] != 0 or offs[-1] != nbytes or (len(offs) > 1 and np.any(np.diff(offs) < 0)):
        raise ValueError("offs must start at 0, never decrease and end at len(buf)")
    if nbytes >= 2 ** 31:
        raise ValueError("batch too large for int32 offsets")


def decode_batch(buf_dev, offs_dev, n: int, out_dev=None, dialect: str = "protobufjs"):
    """Decode ``n`` messages already on the device (uint8 ``buf_dev``, int32 ``offs_dev`` of
    ``n + 1`` host-checked boundaries) on the current torch stream, in ``dialect``. Returns the
    ``(n, 8)`` int32 table (``out_dev`` if given)."""
    import torch
    if dialect not in DIALECT_IDS:
        raise ValueError(f"unknown dialect {dialect!r} ({'|'.join(DIALECT_IDS)})")
    if buf_dev.dtype != torch.uint8 or offs_dev.dtype != torch.int32 or offs_dev.numel() != n + 1:
        raise ValueError("decode_batch needs uint8 buf, int32 offs of n + 1")
    if not (buf_dev.is_cuda and offs_dev.is_cuda and buf_dev.is_contiguous() and offs_dev.is_contiguous()):
        raise ValueError("decode_batch needs contiguous device tensors")
    if out_dev is None:
        out_dev = torch.empty((n, 8), dtype=torch.int32, device=buf_dev.device)
    elif out_dev.shape != (n, 8) or out_dev.dtype != torch.int32 or not out_dev.is_contiguous():
        raise ValueError("out must be a contiguous (n, 8) int32 tensor")
    if n == 0:
        return out_dev
    stream = torch.cuda.current_stream(buf_dev.device).cuda_stream
    err = lib().bh_decode_telemetry(buf_dev.data_ptr(), offs_dev.data_ptr(), n, out_dev.data_ptr(), stream,
                                    DIALECT_IDS[dialect])
    if err:
        raise RuntimeError(f"bh_decode_telemetry launch failed: hipError {err}")
    return out_dev


def decode_bodies(bodies: Sequence[bytes], device="cuda", dialect: str = "protobufjs"):
    """Host bodies → host ``(n, 8)`` numpy table through the GPU (tests; the probe times the steps)."""
    import torch
    buf, offs = pack(bodies)
    check_layout(len(buf), offs)
    b = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(device) if buf else \
        torch.zeros(1, dtype=torch.uint8, device=device)
    o = torch.from_numpy(offs).to(device)
    out = decode_batch(b, o, len(bodies), dialect=dialect)
    return out.cpu().numpy()


def materialise(buf: bytes, table) -> list:
    """Table rows → ``(mediaId, status, progress, host)`` tuples (None for ok == 0), in C
    (``materialise_table``, ops/csrc/py_codec.cpp): the host work any offload still has to do."""
    from . import native
    return native.materialise_table(buf, np.ascontiguousarray(table, dtype=np.int32))


def _varint(p: bytes, i: int, end: int):
    v = 0
    for shift in range(0, 70, 7):
        if i >= end:
            return None, i
        b = p[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v & 0xFFFFFFFFFFFFFFFF, i  # the kernel's uint64 keeps the low 64 bits
    return None, i


def _i32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def reference_decode(buf: bytes, start: int, end: int) -> List[int]:
    """Plain-Python definition of one kernel output row (same rules as the kernel's header)."""
    i = start
    r = [0, 0, 0, 0, 0, 0, 1, 0]
    while i < end:
        key, i = _varint(buf, i, end)
        if key is None or key >> 3 == 0:
            r[6] = 0
            break
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i, end)
            if v is None:
                r[6] = 0
                break
            if field == 2:
                r[2] = _i32(v)
                r[7] |= 2
            elif field == 3:
                r[3] = _i32(v)
                r[7] |= 4
        elif wt == 2:
            n, i = _varint(buf, i, end)
            if n is None or n > end - i:
                r[6] = 0
                break
            if field == 1:
                r[0], r[1] = i, n
                r[7] |= 1
            elif field == 4:
                r[4], r[5] = i, n
                r[7] |= 8
            i += n
        elif wt in (1, 5):
            w = 8 if wt == 1 else 4
            if end - i < w:
                r[6] = 0
                break
            i += w
        else:
            r[6] = 0
            break
    return r


class _PbjsOverrun(Exception):
    pass


class _PbjsReader:
    """protobufjs 6.8.8 BufferReader over ``buf[start:end]`` (csrc/pbjs.hpp, in Python)."""

    def __init__(self, buf: bytes, start: int, end: int):
        self.b, self.base, self.len, self.pos = buf, start, end - start, 0

    def at(self, i: int) -> int:
        return self.b[self.base + i] if i < self.len else -1

    def uint32(self) -> int:
        v = 0
        for k in range(4):
            b = self.at(self.pos)
            v |= (0 if b < 0 else b & 127) << (7 * k)
            self.pos += 1
            if 0 <= b < 128:
                return v
        b = self.at(self.pos)
        v |= (0 if b < 0 else b & 15) << 28
        self.pos += 1
        if 0 <= b < 128:
            return v & 0xFFFFFFFF
        self.pos += 5
        if self.pos > self.len:
            raise _PbjsOverrun
        return v & 0xFFFFFFFF

    def skip_n(self, n: int) -> None:
        if self.pos + n > self.len:
            raise _PbjsOverrun
        self.pos += n

    def skip_type(self, wt: int) -> None:
        depth = 0
        while True:
            if wt == 0:
                while True:
                    if self.pos >= self.len:
                        raise _PbjsOverrun
                    b = self.b[self.base + self.pos]
                    self.pos += 1
                    if not b & 128:
                        break
            elif wt == 1:
                self.skip_n(8)
            elif wt == 2:
                self.skip_n(self.uint32())
            elif wt == 3:
                depth += 1
            elif wt == 5:
                self.skip_n(4)
            elif wt == 4 and depth > 0:
                depth -= 1
            else:
                raise _PbjsOverrun
            if depth == 0:
                return
            wt = self.uint32() & 7

    def string(self) -> Tuple[int, int]:
        n = self.uint32()
        e = min(self.pos + n, self.len)
        off, self.pos = self.pos, e
        return self.base + off, e - off


def reference_decode_pbjs(buf: bytes, start: int, end: int) -> List[int]:
    """Plain-Python definition of one kernel output row in the protobufjs dialect."""
    r = [0, 0, 0, 0, 0, 0, 1, 0]
    rd = _PbjsReader(buf, start, end)
    try:
        while rd.pos < rd.len:
            t = rd.uint32()
            field = t >> 3
            if field in (1, 4):
                k = 0 if field == 1 else 4
                r[k], r[k + 1] = rd.string()
                r[7] |= 1 if field == 1 else 8
            elif field in (2, 3):
                r[field] = _i32(rd.uint32())
                r[7] |= 2 if field == 2 else 4
            else:
                rd.skip_type(t & 7)
    except _PbjsOverrun:
        r[6] = 0
    return r


def reference_table(bodies: Sequence[bytes], dialect: str = "upb") -> np.ndarray:
    buf, offs = pack(bodies)
    row = reference_decode_pbjs if dialect == "protobufjs" else reference_decode
    return np.array([row(buf, int(offs[k]), int(offs[k + 1])) for k in range(len(bodies))],
                    dtype=np.int32).reshape(len(bodies), 8)
