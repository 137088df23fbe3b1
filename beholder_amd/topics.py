"""Queue / topic names and their compact ids.

The reference listens on two queues (``index.js:62`` and ``index.js:127``).
The native ingest frame format carries a one-byte topic id; these are the ids.
"""
from __future__ import annotations

STATUS = "v1.telemetry.status"      # index.js:62
PROGRESS = "v1.telemetry.progress"  # index.js:127

STATUS_ID = 1
PROGRESS_ID = 2

TOPIC_IDS = {STATUS: STATUS_ID, PROGRESS: PROGRESS_ID}
# index -> name (index 0 is reserved / unknown)
TOPIC_NAMES_BY_ID = (None, STATUS, PROGRESS)


def topic_id(name: str) -> int:
    try:
        return TOPIC_IDS[name]
    except KeyError:
        raise KeyError(f"unknown topic {name!r} (known: {', '.join(TOPIC_IDS)})") from None


def topic_name(tid: int):
    return TOPIC_NAMES_BY_ID[tid] if 0 <= tid < len(TOPIC_NAMES_BY_ID) else None
