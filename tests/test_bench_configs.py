"""Every bench config (`python -m beholder_amd bench <config>`, BASELINE.json configs plus the
transport/I-O ones) runs end to end at a small size on CPU and accounts for every event. The
full-size runs are the box tier (tests/test_box_tier.py); this catches a broken harness before
a box run does."""
import pytest

from beholder_amd.bench import harness

SMALL = {"firehose_1k": {"duration_s": 0.5}, "rate_10k": {"duration_s": 0.5}, "backpressure": {"duration_s": 0.2},
         "io_bound": {"events": 3000}, "io_bound_wide": {"events": 4000}, "http_tcp": {"events": 3000},
         "tcp_e2e": {"events": 4000}, "tls_e2e": {"events": 4000}, "amqp": {"events": 6000},
         "soak": {"events": 20000}, "tcp_e2e_preconnect": {"events": 4000}, "tls_e2e_preconnect": {"events": 4000}}


def test_every_config_is_covered():
    assert set(SMALL) | {"plumbing"} == set(harness.CONFIGS)


@pytest.mark.parametrize("name", sorted(SMALL))
def test_config_runs_small(name):
    res = harness.run_config(name, **SMALL[name])
    assert res["config"] == name
    if name == "http_tcp":
        for kind in ("h1", "aiohttp"):
            assert res[kind]["acked"] == 3000 and res[kind]["errors"] == 0
    elif name == "backpressure":
        assert res["accepted"] + res["dropped"] == res["offered"]
    elif "events" in SMALL[name]:
        assert res["acked"] == SMALL[name]["events"], res
    if name in ("tcp_e2e", "tls_e2e", "amqp") or name.endswith("_preconnect"):
        assert res["ingest_rate_eps"] > 0 and res["cpu_us_per_event"] > 0
        assert 0 < res["measured_events"] <= res["acked"]
    if name.endswith("_preconnect"):
        assert res["preconnect"] == 100 and res["errors"] == 0
        assert res["http"]["connections"] >= 100  # opened at init, before the first delivery


def test_paced_run_in_windows_accounts_for_every_event(tmp_path, capsys):
    """scripts/paced_soak.py's mode: the paced production path measured in windows of settled
    deliveries. Every window reports its own percentiles and RSS; the whole phase's percentiles
    are the windows' histograms merged (so they count every measured delivery, not just the last
    window's)."""
    import json
    import runpy
    out = tmp_path / "soak.json"
    script = harness.__file__.replace("beholder_amd/bench/harness.py", "scripts/paced_soak.py")
    mod = runpy.run_path(script, run_name="paced_soak")
    rc = mod["main"](["--rate", "4000", "--seconds", "0.9", "--window-s", "0.3", "--out", str(out)])
    r = json.loads(out.read_text())
    assert rc == 0 and r["errors"] == 0 and r["acked"] == 3600 + 400
    ws = r["windows"]
    # windows end at the first poll past each 1,200th settled delivery: a few more or less
    assert len(ws) == 3 and all(abs(w["events"] - 1200) <= 100 for w in ws), ws
    assert sum(w["events"] for w in ws) == r["measured_events"] and abs(r["measured_events"] - 3600) <= 100
    assert all(w["handle_p50_us"] > 0 and w["handle_p99_us"] >= w["handle_p50_us"] and w["rss_mb"] > 0 for w in ws)
    assert all(w["cpu_us_per_event"] > 0 and w["nivcsw"] >= 0 and "run_delay_ms" in w for w in ws)
    assert all(w["heap_mb"] is None or 0 < w["heap_mb"]["inuse"] <= w["heap_mb"]["size"] for w in ws)
    p50s = [w["handle_p50_us"] for w in ws]
    assert min(p50s) * 0.99 <= r["handle_latency_us"]["p50"] <= max(p50s) * 1.01  # all windows, merged
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["config"] == "tcp_e2e" and len(line["window_p99_us"]) == 3
