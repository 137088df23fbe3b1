"""Round-4 native tools: the SIGPROF sampler (scripts/cprof.py), the fixed-work calibrations
(bench.py calib_*), and the recorder core behind the in-process sink stub."""
import asyncio
import collections
import threading

import pytest

from beholder_amd import ops
from beholder_amd.ops import native


def test_sampler_collects_main_thread_samples_and_stops_cleanly():
    native.prof_start(2000)
    with pytest.raises(RuntimeError):
        native.prof_start(2000)
    x = 0
    for i in range(3_000_000):  # ~0.1-0.3 s of CPU
        x += i
    samples, lost = native.prof_stop()
    with pytest.raises(RuntimeError):
        native.prof_stop()
    assert lost == 0 and len(samples) >= 3
    me = threading.get_native_id()
    assert all(isinstance(ip, int) and ip > 0 for ip, _ in samples)
    assert any(tid == me for _, tid in samples)
    with pytest.raises(ValueError):
        native.prof_start(0)
    native.prof_start(50)  # a second profile in the same process works
    assert native.prof_stop()[1] == 0


def test_calibrations_are_fixed_work():
    ns1, c1 = ops.calib(200_000)
    ns2, c2 = ops.calib(200_000)
    assert c1 == c2 and ns1 > 0 and ns2 > 0  # same work, same checksum
    m1, k1 = ops.calib_mem(1 << 20, 50_000)
    m2, k2 = ops.calib_mem(1 << 20, 50_000)
    assert k1 == k2 and m1 > 0
    with pytest.raises(ValueError):
        ops.calib_mem(64, 10)


def test_recorder_core_builds_urls_like_restler_and_counts():
    calls = collections.deque(maxlen=2)
    ok = object()
    rec = ops.Recorder(calls, ok)
    assert rec.record("POST", "https://t/1/cards/a?b/actions", {"key": "k", "token": None, "text": "a b"}) == \
        "https://t/1/cards/a?b/actions?key=k&text=a%20b"  # "?" even after a "?", None dropped
    assert rec.record("GET", "https://x/y?q=1", None) == "https://x/y?q=1"
    assert rec.record("GET", "https://x/y", {}) == "https://x/y"
    assert rec.count == 3 and list(calls) == [("GET", "https://x/y?q=1"), ("GET", "https://x/y")]
    with pytest.raises(TypeError):
        rec.record("GET", "u", [("a", 1)])


def test_recording_client_fast_path_only_without_rules_delay_or_override():
    from beholder_amd.sinks import RecordingHttpClient
    plain = RecordingHttpClient(keep=4)
    assert plain.native_record is not None
    plain.fail("POST", "https://api")
    assert plain.native_record is None  # rules: the Python path decides every answer
    assert RecordingHttpClient(delay_s=0.01).native_record is None

    class Sub(RecordingHttpClient):
        async def request(self, method, url, *, params=None, timeout=None):
            return await super().request(method, url, params=params, timeout=timeout)
    assert Sub().native_record is None

    async def go():
        r = await plain.request("post", "https://api/x", params={"a": 1})
        return r
    with pytest.raises(Exception):
        asyncio.run(go())  # the rule added above fails POSTs to https://api
    assert plain.count == 1 and plain.urls() == ["https://api/x?a=1"]
    with pytest.raises(AttributeError):
        plain.rules.append(("*", "", None))  # read-only: a stale native_record cannot happen
    plain.clear_rules()
    assert plain.rules == () and plain.native_record is not None


def test_recording_client_fast_path_follows_a_later_delay():
    from beholder_amd.sinks import RecordingHttpClient
    c = RecordingHttpClient()
    assert c.native_record is not None
    c.delay_s = 0.01
    assert c.native_record is None
    c.delay_s = 0.0
    assert c.native_record is not None
