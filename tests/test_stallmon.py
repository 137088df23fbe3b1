"""bench/stallmon.py: stall intervals and the attribution of slow deliveries to processes."""
import asyncio
import time

from beholder_amd.bench.stallmon import StallMonitor, _overlap, attribute, parse_stall_lines


def test_overlap_merges_overlapping_intervals():
    ivs = sorted([(0, 10), (5, 20), (30, 40), (100, 200)])
    starts = [a for a, _ in ivs]
    assert _overlap(0, 50, ivs, starts) == 30  # [0,20) + [30,40)
    assert _overlap(15, 35, ivs, starts) == 10  # [15,20) + [30,35)
    assert _overlap(50, 90, ivs, starts) == 0
    assert _overlap(150, 400, ivs, starts) == 50


def test_attribute_blames_the_process_that_stalled_under_each_delivery():
    slow = [(0, 100, 1100),      # 1 ms; pg stalled 100..900
            (0, 2000, 3000),     # 1 ms; consumer stalled 2000..2900, pg a little
            (0, 5000, 6000)]     # 1 ms; nothing stalled: queueing
    sources = {"consumer": [(2000, 2900)], "pg": [(100, 900), (2950, 3000)], "http": []}
    r = attribute(slow, sources)
    assert r["deliveries"] == 3
    assert r["blamed"] == {"consumer": 1, "pg": 1, "http": 0, "none": 1}
    assert r["time_share"]["pg"] == round((800 + 50) / 3000, 3)
    # under min_share: a 10% overlap is not enough to blame
    assert attribute([(0, 0, 1000)], {"pg": [(0, 100)]})["blamed"] == {"pg": 0, "none": 1}


def test_monitor_records_a_blocked_loop_as_a_stall_and_round_trips_its_report():
    async def go():
        mon = StallMonitor(period_s=0.001, threshold_us=5000).start()
        await asyncio.sleep(0.02)
        t0 = time.monotonic_ns()
        time.sleep(0.03)  # the loop is blocked for 30 ms
        t1 = time.monotonic_ns()
        await asyncio.sleep(0.02)
        mon.stop()
        return mon, t0, t1
    mon, t0, t1 = asyncio.run(go())
    s = mon.summary()
    assert s["loop_stalls"] >= 1 and s["loop_lag_max_us"] >= 20_000
    a, b = max(mon.loop_stalls, key=lambda iv: iv[1] - iv[0])
    # the stall interval covers the block; it may start a few ticks early when the host is busy
    # (a tick before the block ran late under pytest -n), never long before it
    assert t0 - 20_000_000 <= a <= t0 + 2_000_000 and b >= t1 - 1_000_000
    rep = parse_stall_lines("noise\n" + mon.dump_line("pg") + "\nDONE queries=1\n")
    assert rep[0]["name"] == "pg" and [tuple(x) for x in rep[0]["stall_intervals"]] == \
        [tuple(x) for x in mon.loop_stalls + mon.gc_pauses]


def test_due_latencies_from_the_producer_schedule():
    """Paced runs measure each event from its due time (t0 + i / rate): event i is the i-th to
    start, whatever order the trace holds; nothing is reported when events were dropped."""
    from types import SimpleNamespace

    from beholder_amd.bench.harness import _due_latencies

    t0, rate = 1_000_000_000, 1000.0  # one event per ms
    recs = [(t0 + i * 1_000_000 + 5_000, t0 + i * 1_000_000 + 7_000, t0 + i * 1_000_000 + 9_000 + i)
            for i in range(100)]

    class S:
        def slow_deliveries(self):
            return list(reversed(recs)), 0  # settle order need not be start order
    prod = SimpleNamespace(offered=100, rate=rate, t0_ns=t0)
    d = _due_latencies(S(), prod, {"dropped_total": 0})
    assert d["due_to_recv_us"]["p50"] == 5.0 and d["due_to_recv_us"]["max"] == 5.0
    assert d["due_to_ack_us"]["p50"] == (9_000 + 50) / 1e3 and d["due_to_ack_us"]["max"] == (9_000 + 99) / 1e3
    assert _due_latencies(S(), prod, {"dropped_total": 3}) == {}
    assert _due_latencies(S(), SimpleNamespace(offered=101, rate=rate, t0_ns=t0), {"dropped_total": 0}) == {}


def test_a_long_stall_that_began_well_before_the_delivery_is_still_seen():
    """a 2 s stall that started 1.5 s before the delivery started covers all of it;
    the lookback is the longest stall, not a fixed 200 ms."""
    from beholder_amd.bench.stallmon import attribute
    s0 = 10_000_000_000
    stall = (s0, s0 + 2_000_000_000)
    start = s0 + 1_500_000_000
    slow = [(start - 10, start, start + 5_000_000)]
    out = attribute(slow, {"pg": [stall], "http": [(start + 4_000_000, start + 4_100_000)]})
    assert out["blamed"]["pg"] == 1 and out["blamed"]["none"] == 0
    assert out["time_share"]["pg"] == 1.0


def test_a_stall_records_the_work_done_inside_it():
    """``work``: each stall says how much work the loop did while its timer was late, so a long
    callback working through a batch (work > 0) is told apart from a loop that was blocked or not
    scheduled (work 0)."""
    import time as _time

    from beholder_amd.bench.stallmon import StallMonitor
    done = [0]

    async def go():
        mon = StallMonitor(work=lambda: done[0]).start(asyncio.get_running_loop())
        await asyncio.sleep(0.01)
        for _ in range(300):  # one 6 ms callback that does 300 units of work
            _time.sleep(0.00002)
            done[0] += 1
        await asyncio.sleep(0.01)
        _time.sleep(0.006)  # one that does none
        await asyncio.sleep(0.01)
        mon.stop()
        return mon.summary()["stall_work"]
    work = asyncio.run(go())
    assert any(w == 300 for _, w in work) and any(w == 0 for _, w in work), work
    assert all(us >= 1000 for us, _ in work)


def test_loop_lags_take_fixed_memory():
    """Every tick's lateness goes into a fixed-size histogram: a list of one int per tick grew
    the consumer's RSS ~2 MB a minute on a paced soak (profiles/box_r6_psoak/)."""
    import asyncio
    import sys

    from beholder_amd.bench.stallmon import StallMonitor

    async def go():
        m = StallMonitor(period_s=0.0002).start(asyncio.get_running_loop())
        await asyncio.sleep(0.05)
        size0, n0 = sys.getsizeof(m.lags_ns), m.lags_ns.count
        await asyncio.sleep(0.25)
        m.stop()
        return m, size0, n0
    m, size0, n0 = asyncio.run(go())
    assert m.lags_ns.count > n0 > 0 and sys.getsizeof(m.lags_ns) == size0
    s = m.summary()
    assert s["loop_lag_max_us"] >= s["loop_lag_p999_us"] >= s["loop_lag_p99_us"] >= 0
    m.reset()
    assert m.lags_ns.count == 0 and m.summary()["loop_lag_p99_us"] is None
