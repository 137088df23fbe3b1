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
