"""Native JS-semantics text helpers vs their Python reference implementations."""
import io
import json
import math
import random
import struct

from hypothesis import given, settings
from hypothesis import strategies as st

from beholder_amd import ops
from beholder_amd.sinks.http import encode_query, py_encode_query
from beholder_amd.utils import log


def test_js_number_known_values():
    cases = {45.0: "45", 45.5: "45.5", 1e21: "1e+21", 1e-7: "1e-7", 1e-6: "0.000001", 100.0: "100",
             -2.5: "-2.5", 0.1 + 0.2: "0.30000000000000004", 1e20: "100000000000000000000",
             123456789.125: "123456789.125", 5e-324: "5e-324", math.inf: "Infinity", -math.inf: "-Infinity",
             float("nan"): "NaN", 0.0: "0", -0.0: "0"}
    for x, want in cases.items():
        assert log.js_number(x) == want, x
        assert ops.js_number(x) == want, x


def test_js_number_random_doubles_agree():
    rng = random.Random(7)
    for _ in range(20000):
        x = struct.unpack("d", struct.pack("Q", rng.getrandbits(64)))[0]
        if x != x:
            continue
        assert ops.js_number(x) == log.js_number(x), x


def test_js_str():
    for v, want in [(None, "undefined"), (True, "true"), (3, "3"), (2.0, "2"), ("s", "s"), ([1, None, 2], "1,,2"),
                    ({"a": 1}, "[object Object]")]:
        assert log.js_str(v) == want
        assert ops.js_str(v) == want


ARGS = st.lists(st.one_of(st.text(max_size=12), st.integers(-10**6, 10**6), st.floats(allow_nan=False),
                          st.none(), st.booleans()), max_size=5)
FMT = st.text(alphabet="ab %sdifjoO", max_size=16)


@settings(max_examples=500, deadline=None)
@given(FMT, ARGS)
def test_quick_format_native_matches_python(fmt, args):
    assert ops.quick_format(fmt, *args) == log.quick_format((fmt, *args))


def test_quick_format_q11_fix_appends_extra_args():
    """pino v5 would drop these (index.js:51); we append them."""
    assert ops.quick_format("creating comment on", "C1", "with text:", "X") == "creating comment on C1 with text: X"
    assert ops.quick_format("a %s %% %d", "x", 4.0, "tail") == "a x % 4 tail"


def test_format_line_is_valid_pino_json():
    line = ops.format_line(40, 1700000000000, '"pid":1,"hostname":"h","name":"index.js"', None,
                           ('he said "hi"\n\x01 é', 3))
    rec = json.loads(line)
    assert list(rec) == ["level", "time", "pid", "hostname", "name", "msg", "v"]
    assert rec["msg"] == 'he said "hi"\n\x01 é 3' and rec["level"] == 40 and rec["v"] == 1
    assert line.endswith("}\n")


@settings(max_examples=300, deadline=None)
@given(st.dictionaries(st.text(max_size=6), st.one_of(st.text(max_size=20), st.integers(), st.booleans(),
                                                       st.none(), st.floats(allow_nan=False)), max_size=5))
def test_encode_query_native_matches_python(d):
    assert encode_query(d) == py_encode_query(d)


def test_encode_query_matches_encodeURIComponent():
    assert encode_query({"text": "A: **45%** (_h_) é/?&="}) == \
        "text=A%3A%20**45%25**%20(_h_)%20%C3%A9%2F%3F%26%3D"


def test_native_log_line_matches_python_formatter():
    """utils.log.Logger.py_line is the readable reference of the native pino line formatter."""
    from beholder_amd.ops import native
    from beholder_amd.utils.log import Logger, NullStream
    lg = Logger(stream=NullStream())
    cases = [("plain",), ("creating comment on", "c1", "with text:", "DEPLOYED: Progress **5%** (_h_)"),
             ("processing progress update on media", "m", "status", 4, "percent", 99.5),
             ("quote \" and \\ and \n", None, True, -0.0, 1e21), ("%s and %d", "x", 42)]
    for args in cases:
        want = lg.py_line(30, args, time_ms=1234)
        got = native.format_line(30, 1234, lg._prefix, None, args)
        assert got == want, args


def test_logger_writes_utf8_bytes_to_files_in_order(tmp_path):
    """A UTF-8 text file gets the formatted bytes directly (no decode/encode round trip);
    text written to the same stream between flushes stays in order."""
    from beholder_amd.utils.log import Logger, _writer
    p = tmp_path / "log.jsonl"
    with open(p, "w", encoding="utf-8") as f:
        assert _writer(f)[1] is True
        log = Logger(stream=f)
        log.info("first ü", 1)
        log.flush()
        f.write("between\n")
        log.info("second", "✓")
        log.flush()
    lines = p.read_text(encoding="utf-8").splitlines()
    assert [json.loads(lines[0])["msg"], lines[1], json.loads(lines[2])["msg"]] == ["first ü 1", "between", "second ✓"]
    with open(tmp_path / "latin.txt", "w", encoding="latin-1") as g:
        assert _writer(g)[1] is False  # other encodings keep the text path
    assert _writer(io.StringIO())[1] is False


@settings(max_examples=400, deadline=None)
@given(st.lists(st.one_of(st.text(alphabet=st.characters(min_codepoint=0, max_codepoint=0x2FF,
                                                         blacklist_categories=("Cs",)), max_size=40),
                          st.integers(-10**6, 10**6)), min_size=1, max_size=4))
def test_native_log_line_escaping_matches_json(args):
    """JSON escaping (8-byte SWAR scan + per-byte tail) equals json.dumps for any text: control
    characters, quotes and backslashes at every offset, multi-byte UTF-8."""
    from beholder_amd.ops import native
    from beholder_amd.utils.log import Logger, NullStream
    lg = Logger(stream=NullStream())
    args = tuple(args) if isinstance(args[0], str) else ("x",) + tuple(args)
    assert native.format_line(30, 1234, lg._prefix, None, args) == lg.py_line(30, args, time_ms=1234)
