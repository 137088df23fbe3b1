"""Stdin / file frame formats.

Binary (default, what the native reader thread parses)::

    u32 little-endian L (= 1 + len(payload)) | u8 topic_id | payload[L-1]

``topic_id``: 1 = ``v1.telemetry.status``, 2 = ``v1.telemetry.progress``
(:mod:`beholder_amd.topics`). ``payload`` is the protobuf message body (the
AMQP message content in the reference).

NDJSON (human-friendly; parsed in Python, then fed to the same ring)::

    {"topic": "v1.telemetry.progress", "b64": "<base64 protobuf>"}
    {"topic": "v1.telemetry.progress", "json": {"mediaId": "m1", "status": "CONVERTING", "progress": 40}}

In ``json`` form enum fields may be given by name or number.
"""
from __future__ import annotations

import base64
import json
import struct
from typing import Iterable, Iterator, Tuple

from ..ops import frame, frames  # noqa: F401  (re-exported)
from ..topics import PROGRESS, STATUS, TOPIC_IDS, topic_id

_TYPES = {STATUS: "api.TelemetryStatus", PROGRESS: "api.TelemetryProgress"}


def iter_frames(buf: bytes) -> Iterator[Tuple[int, bytes]]:
    """Pure-Python splitter (tests / tools)."""
    i, n = 0, len(buf)
    while i < n:
        if n - i < 4:
            raise ValueError("truncated frame header")
        (L,) = struct.unpack_from("<I", buf, i)
        if L == 0 or n - i - 4 < L:
            raise ValueError("truncated or empty frame")
        yield buf[i + 4], bytes(buf[i + 5:i + 4 + L])
        i += 4 + L


def _encode_json_obj(topic: str, obj: dict) -> bytes:
    from ..models import proto
    pt = proto.load(_TYPES[topic])
    fields = {}
    for k, v in obj.items():
        if k == "status" and isinstance(v, str):
            num = proto.string_to_enum(pt, "TelemetryStatusEntry", v.upper())
            if num is None:
                raise ValueError(f"unknown status {v!r}")
            v = num
        fields[k] = v
    return proto.encode(pt, fields)


def ndjson_line_to_frame(line: str) -> Tuple[int, bytes]:
    rec = json.loads(line)
    topic = rec.get("topic")
    if topic not in TOPIC_IDS:
        raise ValueError(f"unknown topic {topic!r}")
    if "b64" in rec:
        payload = base64.b64decode(rec["b64"])
    elif "json" in rec:
        payload = _encode_json_obj(topic, rec["json"])
    else:
        raise ValueError("ndjson record needs 'b64' or 'json'")
    return topic_id(topic), payload


def ndjson_to_frames(lines: Iterable[str]) -> bytes:
    out = []
    for line in lines:
        line = line.strip()
        if line:
            out.append(ndjson_line_to_frame(line))
    return frames(out)
