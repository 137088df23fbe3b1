"""One table of reference-visible strings (beholder_amd/texts.py) behind both handler implementations.

The compiled handlers (ops/csrc/py_handlers.cpp) must not spell any text the reference emits
(log lines, sink paths and bodies, query names, JS error text; index.js:50-155): they read
``TEXTS`` when a NativeHandlers is built. This file enforces that on the C++ source and checks
that the native side really renders from the table.
"""
import os
import re

import pytest

import helpers
from beholder_amd import texts
from beholder_amd.texts import TEXTS, fill, pieces

from helpers import Rig, progress_msg, status_msg, trello_media

CPP = os.path.join(os.path.dirname(__file__), "..", "beholder_amd", "ops", "csrc", "py_handlers.cpp")

# Python attribute / keyword / module names the C++ uses to reach its dependencies, type names,
# the HTTP method tokens the reference passes (trello 'post'/'put', request 'GET'), and
# Py_BuildValue formats. None of these is message text.
ALLOWED_IDENTIFIERS = {
    "EmbyClient", "GET", "HandlerCall", "JsTypeError", "Media", "MediaNotFound", "MemoryStore", "NativeHandlers",
    "O", "POST", "PUT", "PostgresStore", "TEXTS", "TelegramClient", "TrelloClient", "__module__", "_comment_inc",
    "_deployed_hooks", "_fields", "_get", "_get_nowait", "_hooks_plan", "_pool", "_replace", "_rows", "_select",
    "_status_names_p", "_status_names_s", "_store", "_update", "_update_nowait", "_warn_missing_list", "ack",
    "api_key", "base_url", "beholder_amd.ops._native.HandlerCall", "beholder_amd.ops._native.NativeHandlers",
    "beholder_amd.sinks.emby", "beholder_amd.sinks.telegram", "beholder_amd.sinks.trello", "beholder_amd.store.base",
    "beholder_amd.store.memory", "beholder_amd.store.postgres", "beholder_amd.texts", "child_for", "close",
    "completed_sync", "content", "creator", "creatorId", "decode_progress", "decode_status", "deployed", "done",
    "emby", "err_message", "execute", "field_names", "get_by_id", "get_calls", "handlers", "host", "http", "inc",
    "key", "limiter", "lists", "log", "lower", "make_request", "mediaId", "message", "metadataId", "name",
    "native_log", "no_trello", "on_progress", "on_status", "params", "post", "progress", "progress_counter", "put",
    "py_common.hpp", "raise_for_status", "record", "refresh_library", "request", "result_type", "retry", "ring.hpp", "gil_clock.hpp",
    "row_to_media", "send", "send_message", "state", "stats", "status", "strict", "suspended", "telegram",
    "throw", "timeout", "token", "trello", "trello_creator", "update_calls", "update_status",
    "{s:K,s:K,s:O}", "{s:O}", "{}",
    # the capabilities a Pool (`native_pick`, over its connections) and an H1Client (`native_call`)
    # hand out, called directly
    "Pool", "_conns", "_nets", "native_pick", "beholder_amd.ops._native", "beholder_amd.store.pgwire", "pg_pool_execute",
    "size", "spread_at", "native_call", "native_record", "h1_fast",
}
# internal errors and docstrings (Python-level diagnostics, never emitted by the reference)
ALLOWED_MESSAGES = {
    "HandlerCall: bad state", "native_api.hpp", "native_record: incompatible sink hook",
    "NativeHandlers(handlers): the status / progress handlers compiled to native state machines",
    "TelegramClient.base_url missing", "TrelloClient attributes missing", "_hooks_plan() must return a 6-tuple",
    "calls finished without / after suspending", "can't send non-None value to a just-started handler call",
    "cannot reuse already awaited handler call", "close(): abandon the call", "enum name tables must be dicts",
    "finished (returned or raised)", "handler call is not suspended", "handlers have no attribute %U",
    "object %.100s can't be used in 'await' expression",
    "on_progress(rmsg) -> awaitable: the v1.telemetry.progress handler (index.js:127-155)",
    "on_status(rmsg) -> awaitable: the v1.telemetry.status handler (index.js:62-125)",
    "one native handler invocation: an awaitable iterator (send / throw / close)",
    "resume point (per-handler numbering)", "send(value): resume at the current await",
    "sink client attributes missing", "texts.TEXTS must be a dict", "texts.TEXTS[%s]: expected a str with %d holes",
    "texts.TEXTS[%s]: missing or of the wrong type", "throw expected 1 to 3 arguments",
    "throw(exc): raise at the current await", "unexpected Postgres result",
}


def cpp_literals(src: str):
    """String literals of a C++ source, comments and char literals skipped."""
    out, i, n = [], 0, len(src)
    while i < n:
        if src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            i = src.index("*/", i) + 2
        elif src[i] in "'\"":
            q, j, buf = src[i], i + 1, []
            while src[j] != q:
                if src[j] == "\\":
                    buf.append(src[j:j + 2])
                    j += 2
                else:
                    buf.append(src[j])
                    j += 1
            if q == '"':
                out.append("".join(buf))
            i = j + 1
        else:
            i += 1
    return out


def table_strings():
    for v in TEXTS.values():
        for s in (v if isinstance(v, tuple) else (v,)):
            if isinstance(s, str):
                yield from (p for p in s.split("{}") if p)


def test_cpp_spells_no_reference_visible_text():
    lits = cpp_literals(open(CPP, encoding="utf-8").read())
    assert lits, "no literals found: parser broken?"
    unknown = sorted(set(lits) - ALLOWED_IDENTIFIERS - ALLOWED_MESSAGES - set(TEXTS))
    assert not unknown, f"literals in py_handlers.cpp that belong in beholder_amd/texts.py: {unknown}"
    # no table text hidden inside an allowed literal either (pieces that double as attribute
    # names, e.g. the "status" log argument, are attribute reads there)
    for piece in set(table_strings()) - ALLOWED_IDENTIFIERS:
        if re.fullmatch(r"[A-Za-z_]+", piece):  # a name (query key): must not be a literal itself
            assert piece not in lits, piece
            continue
        if len(piece.strip()) < 3:
            continue
        hits = [lit for lit in lits if piece in lit]
        assert not hits, (piece, hits)


def test_every_table_entry_is_used_by_the_native_loader():
    src = open(CPP, encoding="utf-8").read()
    for key in TEXTS:
        if key == "log_missing_list":  # the native side calls handlers._warn_missing_list
            continue
        assert f'"{key}"' in src, key


def test_fill_and_pieces():
    assert pieces("log_move") == ("moving media card ", " (card id ", ")")
    assert fill("comment", "CONVERTING", 45.0) == "CONVERTING: Progress **45%**"
    assert fill("path_telegram", None) == "/botundefined/sendMessage"
    with pytest.raises(ValueError):
        fill("log_move", "only one")


@pytest.fixture
def native(monkeypatch):
    monkeypatch.setattr(helpers, "HANDLER_IMPL", "native")


def test_native_renders_from_the_table(native, monkeypatch):
    """Changing TEXTS before construction changes what the compiled handlers send and log."""
    table = dict(TEXTS)
    table.update({"log_move": "MOVE {} -> card {}", "path_card": "/2/c/{}", "q_list": "list",
                  "comment": "[{}] {} pct", "log_comment": ("COMMENT", "TEXT"), "trello_move_pos": 7})
    monkeypatch.setattr(texts, "TEXTS", table)
    r = Rig(medias=[trello_media("m1", "QUEUED", card="C9")])
    r.status(status_msg("m1", "DOWNLOADING"))
    r.progress_(progress_msg("m1", "CONVERTING", 5, ""))
    assert ("PUT", "https://api.trello.com/2/c/C9", {"key": "TK", "token": "TT", "list": "L-dl", "pos": "7"}) \
        in r.calls()
    assert "MOVE m1 -> card C9" in r.msgs()
    assert "COMMENT C9 TEXT [CONVERTING] 5 pct" in r.msgs()
    assert r.calls()[-1][2]["text"] == "[CONVERTING] 5 pct"


def test_native_rejects_a_template_with_the_wrong_holes(native, monkeypatch):
    monkeypatch.setattr(texts, "TEXTS", dict(TEXTS, log_status="no holes"))
    with pytest.raises(ValueError, match="log_status"):
        Rig()
    monkeypatch.setattr(texts, "TEXTS", {k: v for k, v in TEXTS.items() if k != "q_pos"})
    with pytest.raises(TypeError, match="q_pos"):
        Rig()


def test_python_side_has_no_duplicate_literals():
    """handlers.py and the sink clients take their text from the table too (string constants of
    their code, docstrings aside)."""
    import ast
    root = os.path.join(os.path.dirname(__file__), "..", "beholder_amd")
    for rel in ("handlers.py", "sinks/trello.py", "sinks/telegram.py", "sinks/emby.py"):
        tree = ast.parse(open(os.path.join(root, rel), encoding="utf-8").read())
        docs = {id(n.body[0].value) for n in ast.walk(tree)
                if isinstance(n, (ast.Module, ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef))
                and n.body and isinstance(n.body[0], ast.Expr) and isinstance(n.body[0].value, ast.Constant)}
        consts = [n.value for n in ast.walk(tree)
                  if isinstance(n, ast.Constant) and isinstance(n.value, str) and id(n) not in docs
                  and n.value not in TEXTS]  # table keys
        for piece in table_strings():
            if len(piece) >= 6 and piece not in ALLOWED_IDENTIFIERS:
                assert not [c for c in consts if piece in c], (rel, piece)
