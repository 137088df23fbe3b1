"""JS-semantics helpers checked against Node itself.

The reference renders numbers with ``String(n)`` (log lines, comment text, query strings), and
escapes log messages with ``JSON.stringify`` (pino). Query values go through
``encodeURIComponent`` (qs 1.2 under the trello client), or through RFC 3986 strict encoding
(qs 6.5 under request). The image ships Node 12, the reference's runtime family, but none of the
reference's npm packages. The oracles below therefore use only Node built-ins. They are skipped
when ``node`` is not on PATH.
"""
import json
import math
import shutil
import subprocess

import pytest
from hypothesis import given, settings, strategies as st

from beholder_amd.ops import encode_query, js_number, native, quote_component

NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="needs node")


def node_map(js_fn: str, inputs: list) -> list:
    """Applies the JS function expression ``js_fn`` to every input (JSON in, JSON out)."""
    script = ("const f = " + js_fn + ";"
              "let s = ''; process.stdin.on('data', d => s += d);"
              "process.stdin.on('end', () => process.stdout.write(JSON.stringify(JSON.parse(s).map(f))));")
    r = subprocess.run([NODE, "-e", script], input=json.dumps(inputs), capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def _num_token(x: float) -> str:
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0 and math.copysign(1, x) < 0:
        return "-0"
    return repr(x)  # shortest round-trip repr: Number(repr) is the same double


SPECIAL = [0.0, -0.0, 1.0, -1.5, 0.1 + 0.2, 1e21, 1e-7, 123456789012345680000.0, 5e-324, 1.7976931348623157e308,
           float("nan"), float("inf"), -float("inf"), 100.0, 2.5e-6, 1e-6, 999999999999999900000.0, 0.000001]


@settings(max_examples=1, deadline=None)
@given(st.lists(st.floats(allow_nan=True, allow_infinity=True), min_size=300, max_size=300))
def test_number_to_string_matches_node(xs):
    xs = SPECIAL + xs
    want = node_map("t => String(Number(t))", [_num_token(x) for x in xs])
    got = [js_number(x) for x in xs]
    assert got == want


def test_integers_match_node_within_safe_range():
    import random
    rng = random.Random(5)
    ints = [0, 1, -1, 2 ** 53 - 1, -(2 ** 53 - 1), 100, 2 ** 31] + [rng.randint(-2 ** 53, 2 ** 53) for _ in range(200)]
    want = node_map("t => String(Number(t))", [str(i) for i in ints])
    assert [js_number(i) for i in ints] == want


_TEXT = st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=40)


@settings(max_examples=1, deadline=None)
@given(st.lists(_TEXT, min_size=300, max_size=300))
def test_encode_uri_component_matches_node(ss):
    ss = ["", "a b", "!'()*~-_.", "€ & = ? / #", "emoji 🎬", "\x00\x7f"] + ss
    want = node_map("s => encodeURIComponent(s)", ss)
    assert [quote_component(s) for s in ss] == want
    assert [encode_query({"k": s})[2:] for s in ss] == want


@settings(max_examples=1, deadline=None)
@given(st.lists(_TEXT, min_size=300, max_size=300))
def test_rfc3986_query_encoding_matches_strict_encoder(ss):
    """request's `qs` option (qs 6.5) escapes !'()* on top of encodeURIComponent."""
    ss = ["!'()*", "*New Anime:* Bebop\nKitsu: https://kitsu.io/anime/1"] + ss
    want = node_map("s => encodeURIComponent(s).replace(/[!'()*]/g, c => '%' + "
                    "c.charCodeAt(0).toString(16).toUpperCase())", ss)
    assert [encode_query({"k": s}, rfc3986=True)[2:] for s in ss] == want


@settings(max_examples=1, deadline=None)
@given(st.lists(_TEXT.filter(lambda s: "%" not in s), min_size=300, max_size=300))
def test_log_message_escaping_matches_json_stringify(ss):
    """pino writes `"msg":` + JSON.stringify(message)."""
    ss = ['he said "hi"', "tab\tnew\nline", "\x00\x01\x1f", "  ", "é/ü", "\\"] + ss
    want = node_map("s => JSON.stringify(s)", ss)
    got = []
    for s in ss:
        line = native.format_line(30, 0, '{"level":30,', None, (s,))
        got.append(line[line.index('"msg":') + 6:line.rindex(',"v":1}')])
    assert got == want
