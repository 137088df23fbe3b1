"""Native log-linear histogram vs exact percentiles."""
import random

from beholder_amd.ops import Histogram


def exact_pct(vals, p):
    s = sorted(vals)
    import math
    rank = max(1, math.ceil(p / 100 * len(s)))
    return s[rank - 1]


def test_percentiles_within_relative_error():
    rng = random.Random(0)
    vals = [int(rng.lognormvariate(10, 2)) for _ in range(50000)]
    h = Histogram()
    h.record_many(vals)
    assert h.count == len(vals) and h.min == min(vals) and h.max == max(vals)
    for p in (1, 10, 50, 90, 99, 99.9):
        want = exact_pct(vals, p)
        got = h.percentile(p)
        assert abs(got - want) <= max(1, 0.008 * want), (p, got, want)


def test_small_values_exact():
    h = Histogram()
    for v in range(256):
        h.record(v)
    assert h.percentile(50) == 127 and h.count_le(99) == 100


def test_merge_and_bytes_roundtrip():
    a, b = Histogram(), Histogram()
    a.record_many(range(1000))
    b.record_many(range(1000, 5000, 3))
    m = Histogram()
    m.merge_bytes(a.to_bytes())
    m.merge_bytes(b.to_bytes())
    a.merge(b)
    assert m.summary() == a.summary()
    assert m.count == 1000 + len(range(1000, 5000, 3))


def test_empty():
    h = Histogram()
    assert h.percentile(50) == 0 and h.count == 0 and h.summary()["count"] == 0
