"""Bench and diagnostic natives (``_native_bench``, ops/csrc_bench/): the SIGPROF sampler
(scripts/cprof.py), the fixed-work calibrations (bench.py calib_*), and the recorder core behind
the in-process sink stub. None of it is in the service's extension."""
import asyncio
import collections
import threading

import pytest

from beholder_amd import ops
from beholder_amd.ops import bench_native
from beholder_amd.ops import bench_native as native


def test_service_extension_has_no_bench_or_profiler_code():
    for name in ("Recorder", "Ready", "prof_start", "prof_stop", "calib", "calib_mem", "paced_write"):
        assert not hasattr(ops.native, name), name
        assert not hasattr(ops, name), name
        if name != "Ready":
            assert hasattr(bench_native, name), name
    assert "_native_bench" not in ops.native.__file__ and ops.native._C_API is not None


def _recorder(calls, mode="h1"):
    from beholder_amd.sinks.h1 import H1Client
    from beholder_amd.sinks.http import STUB_RESPONSE, HttpResponse
    shape = H1Client()

    def origin(key):
        o = shape._origin(key)
        return o.host_header, o.auth
    return bench_native.Recorder(calls, HttpResponse(200, b"{}", None, ""), ops.H1Parser(), STUB_RESPONSE, origin,
                                 shape._tail, shape._tail_cl0, mode=mode)


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
    ns1, c1 = bench_native.calib(200_000)
    ns2, c2 = bench_native.calib(200_000)
    assert c1 == c2 and ns1 > 0 and ns2 > 0  # same work, same checksum
    m1, k1 = bench_native.calib_mem(1 << 20, 50_000)
    m2, k2 = bench_native.calib_mem(1 << 20, 50_000)
    assert k1 == k2 and m1 > 0
    with pytest.raises(ValueError):
        bench_native.calib_mem(64, 10)


def test_recorder_core_builds_urls_like_restler_and_counts():
    calls = collections.deque(maxlen=2)
    rec = _recorder(calls)
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


def test_stub_request_bytes_are_the_h1_clients():
    """The stub builds each request with the H1 client's own builder: the bytes its native path
    writes to the socket (request line with the encodeURIComponent query, Host, Authorization
    from the URL's userinfo, User-Agent, Content-Length: 0 for a PUT/POST)."""
    rec = _recorder(collections.deque())
    rec.record("PUT", "https://api.trello.com/1/cards/c1/idList", {"key": "k", "token": "t", "value": "l 2"})
    assert rec.last_request == (b"PUT /1/cards/c1/idList?key=k&token=t&value=l%202 HTTP/1.1\r\n"
                                b"Host: api.trello.com\r\nUser-Agent: beholder/1.0\r\nContent-Length: 0\r\n\r\n")
    rec.record("GET", "http://u:p%40ss@emby:8096/Library/Refresh?api_key=x", None)
    assert rec.last_request == (b"GET /Library/Refresh?api_key=x HTTP/1.1\r\nHost: emby:8096\r\n"
                                b"Authorization: Basic dTpwQHNz\r\nUser-Agent: beholder/1.0\r\n\r\n")
    assert rec.built == 2 and rec.count == 2 and rec.bytes_out > 200


def test_stub_answers_with_a_parsed_response_carrying_the_url():
    """Each answer is the canned bytes through an H1Parser and the H1 client's HttpResponse, with
    the request's own URL (round 4's fast path shared one response whose url was "")."""
    from beholder_amd.sinks.http import HttpResponse
    rec = _recorder(collections.deque())

    async def go():
        a = await rec.request("POST", "https://api.trello.com/1/cards/c/actions/comments", {"key": "k", "text": "hi"})
        b = await rec.request("GET", "https://api.telegram.org/botT/sendMessage?chat_id=1", None)
        return a, b
    a, b = asyncio.run(go())
    assert type(a) is HttpResponse and a is not b
    assert a.status == 200 and a.body == b"{}" and a.headers["content-length"] == "2"
    assert a.url == "https://api.trello.com/1/cards/c/actions/comments?key=k&text=hi"
    assert b.url == "https://api.telegram.org/botT/sendMessage?chat_id=1"
    old = _recorder(collections.deque(), mode="url")  # the round-4 arm of the A/B

    async def go_old():
        return await old.request("GET", "https://x/y", {"a": 1})
    assert asyncio.run(go_old()).url == "" and old.built == 0 and old.count == 1


def test_recording_client_exposes_a_sink_hook_capsule():
    from beholder_amd.sinks import RecordingHttpClient
    c = RecordingHttpClient()
    assert type(c.native_record).__name__ == "PyCapsule" and "beholder_amd.sink_hook" in repr(c.native_record)
    with pytest.raises(ValueError):
        RecordingHttpClient(stub="nope")


def test_scratch_strings_stay_with_the_owner_thread():
    """ScratchStr (py_common.hpp) lends strings of one pool, last in first out. Python
    code runs while a string is lent and may let another thread run: that thread's scratch string
    must not be a pool slot, or the owner, returning its own slot and lending it again, would
    overwrite the other thread's text while that thread still builds it."""
    f = native.native_bench.scratch_probe
    entered, release = threading.Event(), threading.Event()
    out = {}

    def other_thread():
        out["b"] = f("bbbb", lambda: (entered.set(), release.wait(10)))

    def start_other():  # runs while this thread's "aaaa" is lent
        out["t"] = threading.Thread(target=other_thread)
        out["t"].start()
        assert entered.wait(10)

    out["a"] = f("aaaa", start_other)
    out["c"] = f("cccc", lambda: None)  # this thread again, while the other one's string is lent
    release.set()
    out["t"].join(10)
    assert (out["a"], out["b"], out["c"]) == ("aaaa", "bbbb", "cccc")


def test_request_text_does_not_trust_a_key_len_that_does_not_fit():
    """_C_API h1_request_text: a caller's key_len is trusted (the shape scan skipped)
    only when u[0..k) is the URL's "scheme://authority"; any other value gets the full check,
    so it builds the same request as no key_len at all, or refuses the URL as the H1 client would."""
    f = native.native_bench.request_text_probe
    url = "https://api.trello.com/1/cards/c1"
    want = f("PUT", url, {"pos": "2"}, 0)
    assert want[0] == 1 and want[3] == len("https://api.trello.com")
    for k in (1, 5, 8, 9, 21, 23, 30, len(url), len(url) + 4):
        assert f("PUT", url, {"pos": "2"}, k) == want, k
    assert f("PUT", url, {"pos": "2"}, want[3]) == want
    for bad in ("https://api.trello.com/1/cards#frag", "https://api.trello.com/a\x01b", "https://api.trello.com/a b"):
        assert f("GET", bad, None, 0)[0] == 0, bad
        assert f("GET", bad, None, 3)[0] == 0, bad  # a wrong key_len: scanned, refused


def test_request_text_trusts_a_key_len_only_for_the_url_it_was_taken_for():
    """h1_origin_key remembers the objects it checked and h1_request_text skips the scan only for
    those very objects. The entry holds references: once the checked URL is dropped, a URL of the
    same length allocated after it (pymalloc hands the freed block straight back) is still
    scanned, and a fragment in it is refused."""
    key = native.native_bench.origin_key_probe
    f = native.native_bench.request_text_probe
    head = "https://api.trello.com/1/cards/"
    rc, k = key("GET", head + str(10**8 + 1), None)
    assert (rc, k) == (1, len("https://api.trello.com"))
    assert f("GET", head + str(10**8 + 1), None, k)[0] == 1
    n = len(head) + 9
    sources = [f"{head}c{j}#frag" + "y" * 64 for j in range(10)]  # longer: another size class
    for i in range(50):
        url = head + str(10**8 + i)
        assert len(url) == n and key("GET", url, None)[0] == 1
        del url
        bad = sources[i % 10][:n]  # the one allocation of url's size between the two calls
        assert "#" in bad
        assert f("GET", bad, None, len("https://api.trello.com"))[0] == 0, bad
