"""Native runtime (``_native`` C++ extension) — loader and schema bridge.

The extension is built in-tree by :mod:`beholder_amd.ops.build` (called from
``__graft_entry__.build()``). Importing this package loads it; if the shared
object is missing it is built on the spot when a C++ compiler is available,
otherwise the import fails loudly — the ingest runtime has no silent Python
fallback (set ``BEHOLDER_ALLOW_BUILD=0`` to forbid the on-import build).

Exports: ``MessageCodec``, ``Ingest``, ``Delivery``, ``Settler``, ``Counter``,
``Histogram``, ``frame``, ``frames``, ``mono_ns`` and :func:`codec_for`, which
derives a native codec from a runtime protobuf descriptor. Bench and diagnostic
natives are a separate module (:mod:`beholder_amd.ops.bench_native`).
"""
from __future__ import annotations

import importlib
import os
import subprocess
import threading
from typing import Dict, Optional

from google.protobuf.descriptor import FieldDescriptor as _FD

from ..topics import TOPIC_NAMES_BY_ID

_native = None
_lock = threading.Lock()


def _load():
    global _native
    if _native is not None:
        return _native
    with _lock:
        if _native is not None:
            return _native
        if os.environ.get("BEHOLDER_ALLOW_BUILD", "1") != "0":
            # no-op when the in-tree .so matches the sources (hash stamp); rebuilds a stale one
            from .. import _build
            try:
                _build.build()
            except (OSError, subprocess.CalledProcessError) as e:  # no compiler: use what is there
                if not os.path.exists(_build.TARGET):
                    raise ImportError(f"cannot build the beholder native runtime: {e}") from e
        try:
            mod = importlib.import_module("beholder_amd.ops._native")
        except ImportError as first:
            raise ImportError(
                "beholder native runtime is not built; run `python -m beholder_amd.ops.build`") from first
        from ..models.proto import DecodeError
        mod.configure(decode_error=DecodeError, topics=TOPIC_NAMES_BY_ID)
        _native = mod
        return mod


native = _load()

MessageCodec = native.MessageCodec
Ingest = native.Ingest
Delivery = native.Delivery
Settler = native.Settler
Counter = native.Counter
Histogram = native.Histogram
AmqpDemux = native.AmqpDemux
H1Parser = native.H1Parser
PgReader = native.PgReader
Driver = native.Driver
Window = native.Window
IOFuture = native.IOFuture
if os.environ.get("BEHOLDER_NATIVE_IO", "1") == "0":  # all native I/O off: plain asyncio futures for replies
    import asyncio as _asyncio

    class IOFuture(_asyncio.Future):  # type: ignore[no-redef]
        def __init__(self, loop=None):
            super().__init__(loop=loop)

        resolve = _asyncio.Future.set_result
        reject = _asyncio.Future.set_exception
AckBatcher = native.AckBatcher
SinkStats = native.SinkStats
NativeHandlers = native.NativeHandlers
dispatch_batch = native.dispatch_batch
frame = native.frame
frames = native.frames
mono_ns = native.mono_ns
format_line = native.format_line
quick_format = native.quick_format
js_str = native.js_str
js_number = native.js_number
encode_query = native.encode_query
quote_component = native.quote_component

# Field kinds (csrc/wire.hpp `Kind`)
K_STRING, K_BYTES, K_INT32, K_INT64, K_UINT32, K_UINT64, K_SINT32, K_SINT64 = 1, 2, 3, 4, 5, 6, 7, 8
K_BOOL, K_ENUM, K_FLOAT, K_DOUBLE, K_FIXED32, K_FIXED64, K_SFIXED32, K_SFIXED64 = 9, 10, 11, 12, 13, 14, 15, 16

_KIND_OF = {
    _FD.TYPE_STRING: K_STRING, _FD.TYPE_BYTES: K_BYTES, _FD.TYPE_INT32: K_INT32,
    _FD.TYPE_INT64: K_INT64, _FD.TYPE_UINT32: K_UINT32, _FD.TYPE_UINT64: K_UINT64,
    _FD.TYPE_SINT32: K_SINT32, _FD.TYPE_SINT64: K_SINT64, _FD.TYPE_BOOL: K_BOOL,
    _FD.TYPE_ENUM: K_ENUM, _FD.TYPE_FLOAT: K_FLOAT, _FD.TYPE_DOUBLE: K_DOUBLE,
    _FD.TYPE_FIXED32: K_FIXED32, _FD.TYPE_FIXED64: K_FIXED64,
    _FD.TYPE_SFIXED32: K_SFIXED32, _FD.TYPE_SFIXED64: K_SFIXED64,
}

_codecs: Dict[tuple, Optional[object]] = {}


def field_table(descriptor):
    """``[(number, name, kind), ...]`` for a flat descriptor, or ``None`` if the
    message has repeated / sub-message / proto2-required fields (upb handles those)."""
    out = []
    for f in descriptor.fields:
        if f.is_repeated or f.is_required or f.type in (_FD.TYPE_MESSAGE, _FD.TYPE_GROUP):
            return None
        if getattr(f, "has_presence", False) and f.containing_oneof is not None:
            return None  # oneof / proto3 optional: presence semantics not modelled natively
        kind = _KIND_OF.get(f.type)
        if kind is None:
            return None
        out.append((f.number, f.name, kind))
    return out or None


DIALECTS = ("upb", "protobufjs")


def codec_for(ptype, dialect: str = "upb") -> Optional[object]:
    """Native ``MessageCodec`` for a :class:`~beholder_amd.models.proto.ProtoType` (cached).

    ``dialect`` picks how malformed input is read: ``upb`` (google.protobuf's rules, the test
    oracle for tooling) or ``protobufjs`` (the reference's reader, ``csrc/pbjs.hpp``). Valid
    input decodes identically. None when the schema is not flat, or when the protobufjs
    dialect is asked for a 64-bit integer field it does not model."""
    key = (ptype.full_name, dialect)
    if key in _codecs:
        return _codecs[key]
    table = field_table(ptype.descriptor)
    codec = None
    if table:
        try:
            codec = MessageCodec(ptype.full_name, table, dialect)
        except ValueError:
            if dialect not in DIALECTS:
                raise
    _codecs[key] = codec
    return codec


__all__ = [
    "native", "NativeHandlers", "SinkStats", "AckBatcher", "AmqpDemux", "Driver", "Window", "IOFuture", "H1Parser", "PgReader", "MessageCodec", "Ingest", "Delivery", "Settler", "Counter", "Histogram",
    "frame", "frames", "mono_ns", "codec_for", "field_table", "format_line", "quick_format", "js_str",
    "js_number", "encode_query", "quote_component",
]

# JS-semantics fallbacks for the native text helpers (lists, dicts, %j) live in
# utils.log, which imports this package; importing it last avoids a cycle.
from ..utils import log as _log  # noqa: E402,F401
