"""Prometheus exposition parity with prom-client 11 (index.js:27-40,57,136-138)."""
import pytest

from beholder_amd.metrics import Registry, parse_exposition
from beholder_amd.metrics.registry import Histogram
from beholder_amd.utils.log import Logger


def reference_registry():
    r = Registry("beholder")
    p = r.counter("beholder_progress_updates_total", "Total number of messages processed in this processes lifetime",
                  ["status"])
    t = r.counter("beholder_trello_comments", "Total trello comments crreated in this processes lifetime")
    return r, p, t


def test_exact_initial_exposition():
    r, _, _ = reference_registry()
    assert r.render() == (
        "# HELP beholder_progress_updates_total Total number of messages processed in this processes lifetime\n"
        "# TYPE beholder_progress_updates_total counter\n"
        "\n"
        "# HELP beholder_trello_comments Total trello comments crreated in this processes lifetime\n"
        "# TYPE beholder_trello_comments counter\n"
        "beholder_trello_comments 0\n")


def test_counter_api_variants():
    r, p, t = reference_registry()
    p.inc({"status": "deployed"})
    p.inc({"status": "deployed"}, 2)
    p.labels(status="queued").inc()
    p.child_for("queued").inc(0.5)
    t.inc()
    t.inc(3)
    m = parse_exposition(r.render())
    assert m['beholder_progress_updates_total{status="deployed"}'] == 3
    assert m['beholder_progress_updates_total{status="queued"}'] == 1.5
    assert m["beholder_trello_comments"] == 4


def test_counter_rejects_decrease_and_bad_labels():
    r, p, t = reference_registry()
    with pytest.raises(ValueError):
        t.inc(-1)
    with pytest.raises(ValueError):
        p.inc({"nope": "x"})
    with pytest.raises(ValueError):
        t.inc({"status": "x"})
    with pytest.raises(ValueError):
        r.counter("beholder_trello_comments", "dup")


def test_label_escaping():
    r = Registry()
    c = r.counter("x_total", "help with \\ and\nnewline", ["l"])
    c.inc({"l": 'a"b\\c\nd'})
    out = r.render()
    assert '# HELP x_total help with \\\\ and\\nnewline' in out
    assert 'x_total{l="a\\"b\\\\c\\nd"} 1' in out


def test_histogram_and_gauge():
    r = Registry()
    h = r.histogram("lat_seconds", "latency", buckets=[0.1, 1])
    for v in (0.05, 0.5, 5):
        h.observe(v)
    g = r.gauge("depth", "queue depth", ["q"])
    g.set({"q": "a"}, 3)
    g.inc({"q": "a"})
    m = parse_exposition(r.render())
    assert m['lat_seconds_bucket{le="0.1"}'] == 1 and m['lat_seconds_bucket{le="1"}'] == 2
    assert m['lat_seconds_bucket{le="+Inf"}'] == 3 and m["lat_seconds_count"] == 3
    assert m["lat_seconds_sum"] == pytest.approx(5.55)
    assert m['depth{q="a"}'] == 4
    with pytest.raises(ValueError):
        Histogram("h", "x", ["le"])


def test_invalid_names():
    r = Registry()
    with pytest.raises(ValueError):
        r.counter("bad-name", "x")
    with pytest.raises(ValueError):
        r.counter("ok", "x", ["__reserved"])


def test_native_buckets_match_bisect_reference():
    """Histogram cells are native (ops.Buckets); pinned to the prom-client `le` rule."""
    import bisect
    import math

    from hypothesis import given, settings, strategies as st

    from beholder_amd.ops import native

    @settings(max_examples=200, deadline=None)
    @given(st.lists(st.floats(-1e3, 1e3, allow_nan=False), min_size=1, max_size=12, unique=True),
           st.lists(st.floats(allow_nan=False, allow_infinity=True, width=64), max_size=50))
    def check(bounds, values):
        bounds = sorted(bounds)
        cell = native.Buckets(bounds)
        ref = [0] * len(bounds)
        for v in values:
            cell.observe(v)
            i = bisect.bisect_left(bounds, v)
            if i < len(bounds):
                ref[i] += 1
        counts, total, n = cell.snapshot()
        assert counts == ref and n == len(values)
        s = 0.0
        for v in values:  # same summation order as the native cell
            s += v
        assert (math.isnan(total) and math.isnan(s)) or total == s
    check()
    with pytest.raises(ValueError):
        native.Buckets([1, 1])


def test_cluster_metrics_serve_a_missed_worker_from_its_last_exposition(monkeypatch):
    """A worker that misses a scrape is summed from its last good exposition, so the merged
    counters never step back, and beholder_cluster_worker_up / _scrape_failures_total say so."""
    from beholder_amd.metrics import aggregate as agg
    answers = {1: ["c_total 5\n", None, "c_total 7\n"], 2: ["c_total 1\n", "c_total 2\n", "c_total 3\n"]}

    def fake_fetch(url, timeout=2.0):
        port = int(url.split(":")[2].split("/")[0])
        return answers[port].pop(0)
    monkeypatch.setattr(agg, "fetch", fake_fetch)
    srv = agg.ClusterMetricsServer("127.0.0.1", 0, lambda: [(0, 1), (1, 2)], lambda: True)
    first, second, third = srv.merged_metrics(), srv.merged_metrics(), srv.merged_metrics()

    def val(text, key):
        return float([ln for ln in text.splitlines() if ln.startswith(key + " ")][0].split()[-1])
    assert val(first, "c_total") == 6 and val(second, "c_total") == 7 and val(third, "c_total") == 10
    assert val(second, 'beholder_cluster_worker_up{worker="0"}') == 0
    assert val(second, 'beholder_cluster_worker_up{worker="1"}') == 1
    assert val(third, 'beholder_cluster_scrape_failures_total{worker="0"}') == 1


def test_cluster_metrics_stop_serving_a_worker_that_keeps_failing(monkeypatch):
    """a dead or wedged worker's last exposition is served for at most `stale_after`
    consecutive failed scrapes (or `stale_s` seconds); a worker no longer in the supervisor's
    list is forgotten at once."""
    from beholder_amd.metrics import aggregate as agg
    answers = {1: ["c_total 5\n"] + [None] * 4, 2: ["c_total 1\n"] * 5}
    workers = [(0, 1), (1, 2)]

    def fake_fetch(url, timeout=2.0):
        port = int(url.split(":")[2].split("/")[0])
        return answers[port].pop(0)
    monkeypatch.setattr(agg, "fetch", fake_fetch)
    srv = agg.ClusterMetricsServer("127.0.0.1", 0, lambda: list(workers), lambda: True, stale_after=2)

    def val(text):
        return float([ln for ln in text.splitlines() if ln.startswith("c_total ")][0].split()[-1])
    got = [val(srv.merged_metrics()) for _ in range(4)]
    assert got == [6, 6, 6, 1]  # scrape ok, 2 failures served stale, the 3rd drops it
    srv2 = agg.ClusterMetricsServer("127.0.0.1", 0, lambda: list(workers), lambda: True, stale_s=0.0)
    answers[1] = ["c_total 5\n", None]
    answers[2] = ["c_total 1\n"] * 2
    assert val(srv2.merged_metrics()) == 6
    import time as _t
    _t.sleep(0.01)
    assert val(srv2.merged_metrics()) == 1  # older than stale_s: not served
    answers[2] = ["c_total 1\n"]
    workers[:] = [(1, 2)]
    srv2.merged_metrics()
    assert 0 not in srv2._last


def test_line_splitting_keeps_unicode_line_separators_in_values():
    """Exposition and log lines end in "\\n" only: a label value or log message holding U+0085,
    U+2028 or U+001E (all line breaks to str.splitlines) stays inside its line."""
    from beholder_amd.metrics.aggregate import aggregate
    from beholder_amd.utils.log import MemoryStream
    odd = "a\x85b c\x1ed"
    r = Registry()
    c = r.counter("odd_total", "x", ["status"])
    c.labels(status=odd).inc(2)
    text = r.render()
    merged = parse_exposition(aggregate([text, text]))
    assert merged == {f'odd_total{{status="{odd}"}}': 4.0}
    s = MemoryStream()
    Logger(stream=s).info("media " + odd)
    assert [rec["msg"] for rec in s.records()] == ["media " + odd]
