"""``service.log.positional_args``: ``append`` (default, the Q11 fix) vs ``drop`` (pino@5's
message text exactly). Table-driven over every log call in the reference (index.js:51,66,82,88,
98,111,121,133,150,157), under both handler implementations.

pino@5 formats ``logger.info(f, ...args)`` with quick-format-unescaped: ``%s``/``%d``/... consume
arguments, and arguments no specifier consumes are dropped. None of index.js's calls has a
specifier, so in ``drop`` mode every multi-argument call logs only its first argument.
"""

import pytest

import helpers
from beholder_amd.utils.log import Logger, MemoryStream, quick_format
from beholder_amd.ops import native

from helpers import ENUM, Rig, api_media, cfg, progress_msg, status_msg, trello_media


@pytest.fixture(params=["python", "native"])
def impl(request, monkeypatch):
    monkeypatch.setattr(helpers, "HANDLER_IMPL", request.param)
    return request.param


def _status_move(mode):
    r = Rig(medias=[trello_media("m1", "QUEUED", card="CARD9")], positional_args=mode)
    r.status(status_msg("m1", "DOWNLOADING"))
    return r


def _status_missing_list(mode):
    r = Rig(medias=[trello_media("m1")], positional_args=mode)
    r.status(status_msg("m1", "UPLOADING"))
    return r


def _status_deployed(mode):
    r = Rig(medias=[api_media("m2", "UPLOADING", name="Bebop")], positional_args=mode)
    r.status(status_msg("m2", "DEPLOYED"))
    return r


def _status_hooks_fail(mode):
    r = Rig(medias=[api_media("m2")], positional_args=mode)
    r.http.fail("GET", "https://api.telegram.org", message="ECONNREFUSED")
    r.status(status_msg("m2", "DEPLOYED"))
    return r


def _progress_comment(mode):
    r = Rig(medias=[trello_media("m1", card="CARD1")], positional_args=mode)
    r.progress_(progress_msg("m1", "CONVERTING", 45, "w3"))
    return r


def _progress_fail(mode):
    r = Rig(positional_args=mode)
    r.progress_(progress_msg("missing", "QUEUED", 1))
    return r


CONV, DL, UP, DEP, Q = ENUM["CONVERTING"], ENUM["DOWNLOADING"], ENUM["UPLOADING"], ENUM["DEPLOYED"], ENUM["QUEUED"]
# (index.js line, scenario, level, pino@5 text ("drop"), this service's default text ("append"))
SITES = [
    (66, _status_move, 30, f"processing status update for media m1, status: {DL}", None),
    (82, _status_move, 30, "moving media card m1 (card id CARD9)", None),
    (88, _status_missing_list, 40, "unable to find list for status",
     f"unable to find list for status {UP} (UPLOADING) avail ([queued,downloading,converting,deployed])"),
    (98, _status_deployed, 30, "informing telegram that media 'm2' is available", None),
    (111, _status_deployed, 30, "telling emby to refresh at http://emby:8096", None),
    (121, _status_hooks_fail, 40, "failed to run deployed hooks:", "failed to run deployed hooks: ECONNREFUSED"),
    (133, _progress_comment, 30, "processing progress update on media",
     f"processing progress update on media m1 status {CONV} percent 45"),
    (51, _progress_comment, 30, "creating comment on", "creating comment on CARD1 with text: CONVERTING: Progress **45%** (_w3_)"),
    (150, _progress_fail, 40, "failed to update media progress",
     "failed to update media progress media missing not found"),
]


@pytest.mark.parametrize("mode", ["drop", "append"])
@pytest.mark.parametrize("line,scenario,level,pino,ours", SITES, ids=[f"index.js:{s[0]}" for s in SITES])
def test_reference_log_sites(impl, mode, line, scenario, level, pino, ours):
    r = scenario(mode)
    want = pino if mode == "drop" else (ours or pino)
    assert want in r.msgs(level), (line, r.msgs())


def test_initialized_line_is_identical_in_both_modes():
    """index.js:157 has one argument: both modes log exactly "initialized"."""
    for mode in ("drop", "append"):
        s = MemoryStream()
        Logger(stream=s, positional_args=mode).info("initialized")
        assert s.records()[-1]["msg"] == "initialized"


@pytest.mark.parametrize("args,drop,append", [
    (("a", "b", 1), "a", "a b 1"),
    (("x %s y", "S", "extra"), "x S y", "x S y extra"),
    (("100%% %d", 5, 6), "100% 5", "100% 5 6"),
    (("%s %s", "one"), "one %s", "one %s"),  # missing argument: the specifier stays
    ((7, "x"), "7", "7 x"),
])
def test_quick_format_modes_native_matches_python(args, drop, append):
    assert quick_format(args, drop=True) == native.quick_format_drop(*args) == drop
    assert quick_format(args) == native.quick_format(*args) == append


def test_mode_from_config_and_children_share_it():
    from beholder_amd.config import ConfigError
    from beholder_amd.service import Service
    c = cfg({"service": {"log": {"positional_args": "drop"}}})
    svc = Service(c, serve_metrics=False)
    assert svc.log.positional_args == "drop"
    s = MemoryStream()
    lg = Logger(stream=s, positional_args="drop")
    lg.child(media="m1").warn("a", "b")
    lg.positional_args = "append"
    lg.warn("a", "b")
    lg.flush()
    assert [r["msg"] for r in s.records()] == ["a", "a b"]
    with pytest.raises(ConfigError):
        cfg({"service": {"log": {"positional_args": "keep"}}})
