"""Structured differential fuzz of the native protobuf codec against upb (long run, seeded):

    python scripts/fuzz_codec.py SEED

Generates plausible field encodings (all wire types, over-long tags and varints, groups) for
every schema message and reports any input the two decoders disagree on."""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beholder_amd.models import proto  # noqa: E402
from beholder_amd.models.proto import DecodeError  # noqa: E402
from beholder_amd.ops import codec_for  # noqa: E402

rng = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
bad = 0
for T in ("api.TelemetryProgress", "api.TelemetryStatus", "api.Media"):
    P = proto.load(T); c = codec_for(P)
    if c is None: print("no native codec for", T); continue
    fields = [f.name for f in P.descriptor.fields]
    for it in range(60000):
        parts = []
        for _ in range(rng.randint(0, 6)):
            kind = rng.random()
            if kind < 0.5:  # plausible field
                fn = rng.randint(1, 14); wt = rng.choice([0, 0, 2, 2, 1, 5, 3, 4, 6, 7])
                tag = (fn << 3) | wt
                tb = bytearray()
                v = tag
                while True:
                    b = v & 0x7f; v >>= 7
                    tb.append(b | (0x80 if v else 0))
                    if not v: break
                if rng.random() < 0.1: tb[-1] |= 0x80; tb.append(0)  # over-long tag
                parts.append(bytes(tb))
                if wt == 0:
                    n = rng.randint(1, 11)
                    parts.append(bytes(rng.randint(0x80, 0xff) for _ in range(n - 1)) + bytes([rng.randint(0, 0x7f)]))
                elif wt == 2:
                    ln = rng.randint(0, 8)
                    parts.append(bytes([ln]) + bytes(rng.randint(0, 255) for _ in range(rng.randint(0, 9))))
                elif wt == 1:
                    parts.append(bytes(rng.randint(0, 255) for _ in range(rng.randint(6, 9))))
                elif wt == 5:
                    parts.append(bytes(rng.randint(0, 255) for _ in range(rng.randint(3, 5))))
            else:
                parts.append(bytes(rng.randint(0, 255) for _ in range(rng.randint(1, 4))))
        data = b"".join(parts)
        try:
            m = proto.decode(P, data); want = tuple(getattr(m, f) for f in fields)
        except DecodeError:
            want = None
        try:
            got = tuple(c.decode(data))
        except DecodeError:
            got = None
        if got != want:
            bad += 1
            if bad <= 5: print(T, data.hex(), "upb", want, "native", got)
print("mismatches", bad)
