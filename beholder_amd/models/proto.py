"""Schema registry and codec API — parity with ``triton-core/proto``.

Reference call sites (``/root/reference/index.js``):

* ``proto.load('api.TelemetryProgress')`` etc. — index.js:46-48
* ``proto.decode(type, rmsg.message.content)`` — index.js:63 (sync), :129 (awaited)
* ``proto.enumToString(type, 'TelemetryStatusEntry', status)`` — index.js:74, :134
* ``proto.stringToEnum(type, 'TelemetryStatusEntry', 'DEPLOYED')`` — index.js:94
* ``proto.stringToEnum(mediaProto, 'CreatorType', 'TRELLO')`` — index.js:142

Semantics reproduced from protobufjs (the library triton-core wraps):

* ``decode`` of proto3 fills absent scalars with defaults (``""`` / ``0``) and
  raises on truncated / malformed input;
* ``enumToString`` of an unknown number returns ``None`` (JS ``undefined``);
* ``stringToEnum`` of an unknown name returns ``None``.

Message *classes* come from ``google.protobuf`` (upb) built at runtime from
the ``.proto`` files — the reference-quality codec used for encoding, tooling
and as the oracle in tests. The hot ingest path decodes with the native C++
codec (``beholder_amd.ops``), which is tested field-for-field against it.
"""
from __future__ import annotations

import glob
import os
import threading
from typing import Dict, Optional

from google.protobuf import descriptor_pool, message_factory
from google.protobuf.message import DecodeError as _PbDecodeError

from .protoparse import parse_proto

PROTO_DIR = os.environ.get("BEHOLDER_PROTO_PATH") or os.path.join(os.path.dirname(__file__), "proto")


class DecodeError(ValueError):
    """Raised when bytes are not a valid encoding of the requested type."""


class ProtoType:
    """Handle returned by :func:`load` (the ``telemetryStatusProto`` of index.js:47)."""

    __slots__ = ("full_name", "package", "descriptor", "cls", "_enum_cache", "registry")

    def __init__(self, full_name: str, descriptor, cls, registry: "Registry"):
        self.full_name = full_name
        self.package = full_name.rsplit(".", 1)[0] if "." in full_name else ""
        self.descriptor = descriptor
        self.cls = cls
        self.registry = registry
        self._enum_cache: Dict[str, tuple] = {}

    @property
    def name(self) -> str:
        return self.descriptor.name

    def enum(self, enum_name: str):
        """Resolve ``enum_name`` relative to this type (nested first, then package)."""
        hit = self._enum_cache.get(enum_name)
        if hit is not None:
            return hit
        ed = None
        for cand in (f"{self.full_name}.{enum_name}",
                     f"{self.package}.{enum_name}" if self.package else enum_name,
                     enum_name):
            try:
                ed = self.registry.pool.FindEnumTypeByName(cand)
                break
            except KeyError:
                continue
        if ed is None:
            raise KeyError(f"no enum {enum_name!r} visible from {self.full_name}")
        by_num: Dict[int, str] = {}
        for v in ed.values:
            by_num.setdefault(v.number, v.name)  # first name wins on aliases (protobufjs)
        by_name = {v.name: v.number for v in ed.values}
        hit = (by_num, by_name)
        self._enum_cache[enum_name] = hit
        return hit

    def __repr__(self) -> str:
        return f"ProtoType({self.full_name})"


class Registry:
    """A descriptor pool populated from a directory of ``.proto`` files."""

    def __init__(self, proto_dir: str = PROTO_DIR):
        self.proto_dir = proto_dir
        self.pool = descriptor_pool.DescriptorPool()
        self._types: Dict[str, ProtoType] = {}
        self._lock = threading.Lock()
        self._loaded = False

    def _load_files(self) -> None:
        files = sorted(glob.glob(os.path.join(self.proto_dir, "**", "*.proto"), recursive=True))
        if not files:
            raise FileNotFoundError(f"no .proto files under {self.proto_dir}")
        known: dict = {}
        fds = []
        for path in files:
            with open(path, "r", encoding="utf-8") as f:
                src = f.read()
            rel = os.path.relpath(path, self.proto_dir)
            fds.append(parse_proto(src, rel, known))
        # Add in dependency order (files only depend on files in this dir).
        added = set()
        pending = list(fds)
        while pending:
            progressed = False
            for fd in list(pending):
                if all(d in added for d in fd.dependency):
                    self.pool.Add(fd)
                    added.add(fd.name)
                    pending.remove(fd)
                    progressed = True
            if not progressed:
                raise ValueError("unresolvable .proto imports: " + ", ".join(f.name for f in pending))
        self._loaded = True

    def load(self, full_name: str) -> ProtoType:
        with self._lock:
            t = self._types.get(full_name)
            if t is not None:
                return t
            if not self._loaded:
                self._load_files()
            try:
                desc = self.pool.FindMessageTypeByName(full_name)
            except KeyError:
                raise KeyError(f"no such message type: {full_name}") from None
            cls = message_factory.GetMessageClass(desc)
            t = ProtoType(full_name, desc, cls, self)
            self._types[full_name] = t
            return t


_default: Optional[Registry] = None
_default_lock = threading.Lock()


def default_registry() -> Registry:
    global _default
    with _default_lock:
        if _default is None:
            _default = Registry()
        return _default


def load(full_name: str) -> ProtoType:
    """``proto.load('api.TelemetryStatus')`` (index.js:46-48)."""
    return default_registry().load(full_name)


def decode(ptype: ProtoType, data: bytes):
    """``proto.decode(type, buf)`` (index.js:63,129) → message object (fields by proto name)."""
    if not isinstance(data, (bytes, bytearray, memoryview)):
        raise DecodeError(f"illegal buffer: expected bytes, got {type(data).__name__}")
    msg = ptype.cls()
    try:
        msg.ParseFromString(bytes(data))
    except _PbDecodeError as e:
        raise DecodeError(str(e)) from None
    return msg


def encode(ptype: ProtoType, obj) -> bytes:
    """Encode a dict (proto field names) or a message instance."""
    if isinstance(obj, dict):
        msg = ptype.cls(**obj)
    else:
        msg = obj
    return msg.SerializeToString()


def enum_to_string(ptype: ProtoType, enum_name: str, value) -> Optional[str]:
    """``proto.enumToString`` — unknown numbers give ``None`` (index.js:74,134; quirk Q6)."""
    by_num, _ = ptype.enum(enum_name)
    try:
        return by_num.get(int(value))
    except (TypeError, ValueError):
        return None


def string_to_enum(ptype: ProtoType, enum_name: str, name: str) -> Optional[int]:
    """``proto.stringToEnum`` (index.js:94,142)."""
    _, by_name = ptype.enum(enum_name)
    return by_name.get(name)


# camelCase aliases matching the triton-core API names
enumToString = enum_to_string
stringToEnum = string_to_enum
