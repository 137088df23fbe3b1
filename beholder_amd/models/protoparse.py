"""Tiny ``.proto`` (proto3 subset) parser → ``FileDescriptorProto``.

There is no ``protoc`` / ``grpc_tools`` in the image, but
``google.protobuf`` (upb backend) is importable, and it can build message
classes from descriptors at runtime. This parser turns our ``.proto`` source
into a ``FileDescriptorProto`` so the ``.proto`` file stays the single source
of truth for the schema — the same way triton-core's ``proto.load`` reads
``.proto`` files at runtime (index.js:46-48).

Supported: ``syntax``, ``package``, ``import`` (recorded as a dependency),
``option`` (ignored), ``enum`` (incl. ``option allow_alias``), ``message``
(nested messages/enums), field labels ``optional`` / ``repeated``, scalar,
enum and message field types, ``map<K,V>``, ``oneof`` and ``reserved``.
Services / extensions are not supported (beholder has none).
"""
from __future__ import annotations

import re
from typing import List, Optional, Tuple

from google.protobuf import descriptor_pb2

FDP = descriptor_pb2.FieldDescriptorProto

SCALARS = {
    "double": FDP.TYPE_DOUBLE, "float": FDP.TYPE_FLOAT,
    "int64": FDP.TYPE_INT64, "uint64": FDP.TYPE_UINT64, "int32": FDP.TYPE_INT32,
    "fixed64": FDP.TYPE_FIXED64, "fixed32": FDP.TYPE_FIXED32, "bool": FDP.TYPE_BOOL,
    "string": FDP.TYPE_STRING, "bytes": FDP.TYPE_BYTES, "uint32": FDP.TYPE_UINT32,
    "sfixed32": FDP.TYPE_SFIXED32, "sfixed64": FDP.TYPE_SFIXED64,
    "sint32": FDP.TYPE_SINT32, "sint64": FDP.TYPE_SINT64,
}

_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<lc>//[^\n]*)
  | (?P<bc>/\*.*?\*/)
  | (?P<str>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*')
  | (?P<num>-?(?:0[xX][0-9a-fA-F]+|\d+(?:\.\d*)?(?:[eE][+-]?\d+)?))
  | (?P<id>[A-Za-z_][A-Za-z0-9_.]*)
  | (?P<sym>[{}\[\]()<>;=,])
""", re.S | re.X)


class ProtoSyntaxError(ValueError):
    pass


def tokenize(src: str) -> List[Tuple[str, str, int]]:
    toks = []
    pos = 0
    line = 1
    while pos < len(src):
        m = _TOKEN.match(src, pos)
        if not m:
            raise ProtoSyntaxError(f"line {line}: unexpected character {src[pos]!r}")
        kind = m.lastgroup
        text = m.group()
        if kind in ("str", "num", "id", "sym"):
            toks.append((kind, text, line))
        line += text.count("\n")
        pos = m.end()
    return toks


def _camel_json(name: str) -> str:
    out, up = [], False
    for ch in name:
        if ch == "_":
            up = True
        elif up:
            out.append(ch.upper())
            up = False
        else:
            out.append(ch)
    return "".join(out)


class _Parser:
    def __init__(self, src: str, filename: str):
        self.toks = tokenize(src)
        self.i = 0
        self.fd = descriptor_pb2.FileDescriptorProto(name=filename)
        self.syntax = "proto2"

    # token helpers
    def peek(self, k: int = 0) -> Optional[str]:
        j = self.i + k
        return self.toks[j][1] if j < len(self.toks) else None

    def next(self) -> str:
        if self.i >= len(self.toks):
            raise ProtoSyntaxError("unexpected end of file")
        t = self.toks[self.i]
        self.i += 1
        return t[1]

    def expect(self, text: str) -> None:
        line = self.toks[self.i][2] if self.i < len(self.toks) else -1
        got = self.next()
        if got != text:
            raise ProtoSyntaxError(f"line {line}: expected {text!r}, got {got!r}")

    def skip_statement(self) -> None:
        depth = 0
        while True:
            t = self.next()
            if t in "{[(" and len(t) == 1:
                depth += 1
            elif t in "}])" and len(t) == 1:
                depth -= 1
                if depth == 0 and t == "}":
                    return
            elif t == ";" and depth == 0:
                return

    # grammar
    def parse(self) -> descriptor_pb2.FileDescriptorProto:
        while self.i < len(self.toks):
            t = self.peek()
            if t == "syntax":
                self.next(); self.expect("=")
                self.syntax = self.next().strip("\"'")
                self.expect(";")
                if self.syntax == "proto3":
                    self.fd.syntax = "proto3"
            elif t == "package":
                self.next(); self.fd.package = self.next(); self.expect(";")
            elif t == "import":
                self.next()
                if self.peek() in ("public", "weak"):
                    self.next()
                self.fd.dependency.append(self.next().strip("\"'"))
                self.expect(";")
            elif t == "option":
                self.skip_statement()
            elif t == "enum":
                self.parse_enum(self.fd.enum_type.add())
            elif t == "message":
                self.parse_message(self.fd.message_type.add())
            elif t == ";":
                self.next()
            else:
                raise ProtoSyntaxError(f"line {self.toks[self.i][2]}: unsupported top-level {t!r}")
        return self.fd

    def parse_enum(self, ed) -> None:
        self.expect("enum")
        ed.name = self.next()
        self.expect("{")
        while self.peek() != "}":
            t = self.peek()
            if t == "option":
                self.next()
                oname = self.next(); self.expect("="); oval = self.next(); self.expect(";")
                if oname == "allow_alias":
                    ed.options.allow_alias = oval == "true"
            elif t == "reserved":
                self.skip_statement()
            elif t == ";":
                self.next()
            else:
                v = ed.value.add()
                v.name = self.next()
                self.expect("=")
                v.number = int(self.next(), 0)
                if self.peek() == "[":
                    self.skip_statement()
                else:
                    self.expect(";")
        self.expect("}")

    def parse_message(self, md) -> None:
        self.expect("message")
        md.name = self.next()
        self.parse_message_body(md)

    def parse_message_body(self, md, oneof_index: Optional[int] = None) -> None:
        self.expect("{")
        while self.peek() != "}":
            t = self.peek()
            if t == "message":
                self.parse_message(md.nested_type.add())
            elif t == "enum":
                self.parse_enum(md.enum_type.add())
            elif t in ("option", "reserved", "extensions"):
                self.skip_statement()
            elif t == "oneof":
                self.next()
                od = md.oneof_decl.add()
                od.name = self.next()
                self.parse_oneof(md, len(md.oneof_decl) - 1)
            elif t == "map":
                self.parse_map(md)
            elif t == ";":
                self.next()
            else:
                self.parse_field(md, oneof_index)
        self.expect("}")

    def parse_oneof(self, md, idx: int) -> None:
        self.expect("{")
        while self.peek() != "}":
            if self.peek() == "option":
                self.skip_statement()
                continue
            self.parse_field(md, idx)
        self.expect("}")

    def parse_field(self, md, oneof_index: Optional[int]) -> None:
        label = FDP.LABEL_OPTIONAL
        proto3_optional = False
        if self.peek() in ("optional", "repeated", "required"):
            lab = self.next()
            if lab == "repeated":
                label = FDP.LABEL_REPEATED
            elif lab == "required":
                label = FDP.LABEL_REQUIRED
            elif self.syntax == "proto3":
                proto3_optional = True
        ftype = self.next()
        f = md.field.add()
        f.name = self.next()
        self.expect("=")
        f.number = int(self.next(), 0)
        f.label = label
        f.json_name = _camel_json(f.name)
        if ftype in SCALARS:
            f.type = SCALARS[ftype]
        else:
            f.type_name = ftype  # resolved after the whole file is parsed
        if oneof_index is not None:
            f.oneof_index = oneof_index
        if proto3_optional:
            f.proto3_optional = True
            od = md.oneof_decl.add()
            od.name = "_" + f.name
            f.oneof_index = len(md.oneof_decl) - 1
        if self.peek() == "[":
            depth = 0
            while True:
                t = self.next()
                if t == "[":
                    depth += 1
                elif t == "]":
                    depth -= 1
                    if depth == 0:
                        break
                elif t == "packed" and self.peek() == "=":
                    self.next()
                    f.options.packed = self.next() == "true"
        self.expect(";")

    def parse_map(self, md) -> None:
        self.expect("map"); self.expect("<")
        ktype = self.next(); self.expect(","); vtype = self.next(); self.expect(">")
        name = self.next(); self.expect("="); number = int(self.next(), 0)
        if self.peek() == "[":
            self.skip_statement()
        else:
            self.expect(";")
        entry = md.nested_type.add()
        entry.name = "".join(p[:1].upper() + p[1:] for p in name.split("_")) + "Entry"
        entry.options.map_entry = True
        for fname, ft, num in (("key", ktype, 1), ("value", vtype, 2)):
            ef = entry.field.add(name=fname, number=num, label=FDP.LABEL_OPTIONAL, json_name=fname)
            if ft in SCALARS:
                ef.type = SCALARS[ft]
            else:
                ef.type_name = ft
        f = md.field.add(name=name, number=number, label=FDP.LABEL_REPEATED,
                         type=FDP.TYPE_MESSAGE, type_name=entry.name, json_name=_camel_json(name))
        del f


def _resolve(fd: descriptor_pb2.FileDescriptorProto, known: dict) -> None:
    """Resolve relative type names to fully-qualified ``.pkg.Type`` and set MESSAGE/ENUM."""
    pkg = fd.package

    def collect(prefix: str, msgs, enums):
        for e in enums:
            known[f"{prefix}.{e.name}"] = "enum"
        for m in msgs:
            known[f"{prefix}.{m.name}"] = "message"
            collect(f"{prefix}.{m.name}", m.nested_type, m.enum_type)

    root = "." + pkg if pkg else ""
    collect(root, fd.message_type, fd.enum_type)

    def lookup(scope: str, name: str) -> str:
        if name.startswith("."):
            if name in known:
                return name
            raise ProtoSyntaxError(f"unknown type {name!r}")
        parts = scope.split(".")
        while parts:
            cand = ".".join(parts + [name])
            cand = cand if cand.startswith(".") else "." + cand
            if cand in known:
                return cand
            parts = parts[:-1]
        raise ProtoSyntaxError(f"unknown type {name!r} referenced in scope {scope!r}")

    def fix(scope: str, msgs):
        for m in msgs:
            here = f"{scope}.{m.name}"
            for f in m.field:
                if f.type_name:
                    full = lookup(here, f.type_name)
                    f.type_name = full
                    f.type = FDP.TYPE_MESSAGE if known[full] == "message" else FDP.TYPE_ENUM
            fix(here, m.nested_type)

    fix(root, fd.message_type)


def parse_proto(src: str, filename: str = "api.proto", known: Optional[dict] = None) -> descriptor_pb2.FileDescriptorProto:
    """Parse ``src`` into a resolved ``FileDescriptorProto``."""
    fd = _Parser(src, filename).parse()
    _resolve(fd, known if known is not None else {})
    return fd
