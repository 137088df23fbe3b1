"""Every reference-visible string of the handlers, in one table (index.js:50-155).

Log messages, the text and URL paths sent to Trello / Telegram / Emby, query parameter names,
fallback text and the JS error text of quirk Q6. Both implementations of the business logic
read this table: :mod:`beholder_amd.handlers` (and the sink clients) directly, the compiled
handlers (``ops/csrc/py_handlers.cpp``) once, when :class:`~beholder_amd.ops.NativeHandlers` is
constructed. The C++ source holds none of these strings (``tests/test_texts.py`` fails if one
appears there), so a behaviour change to any of them is made here, once.

Templates mark each value with ``{}``; values are rendered with JavaScript ``String()`` rules
(:func:`~beholder_amd.utils.log.js_str`), as the reference's template literals do.
"""
from __future__ import annotations

from typing import Any, Dict, Tuple, Union

TEXTS: Dict[str, Union[str, int, Tuple[str, ...]]] = {
    # -- log lines (one argument: a template) -------------------------------------------
    "log_status": "processing status update for media {}, status: {}",          # index.js:66
    "log_move": "moving media card {} (card id {})",                             # index.js:82
    "log_telegram": "informing telegram that media '{}' is available",           # index.js:98
    "log_emby": "telling emby to refresh at {}",                                 # index.js:111
    # -- log calls with positional arguments (Q11): the literal arguments, in order -------
    "log_comment": ("creating comment on", "with text:"),                        # index.js:51
    "log_progress": ("processing progress update on media", "status", "percent"),  # index.js:133
    "log_missing_list": ("unable to find list for status", "({})", "avail ([{}])"),  # index.js:88
    "warn_hooks": "failed to run deployed hooks:",                               # index.js:121
    "warn_progress": "failed to update media progress",                          # index.js:150
    # -- what the sinks are sent -------------------------------------------------------
    "comment": "{}: Progress **{}%**",                                           # index.js:143-145 (Q8)
    "comment_host": " (_{}_)",                                                   # index.js:146 (Q8)
    "comment_fallback": "Failed to retrieve comment text.",                      # index.js:54
    "telegram_text": "*New Anime:* {}\nKitsu: https://kitsu.io/anime/{}",        # index.js:104
    "telegram_parse_mode": "markdown",                                           # index.js:105
    "trello_move_pos": 2,                                                        # index.js:85 (Q8)
    # -- URL paths (appended to the client's base URL / the configured Emby host) --------
    "path_comment": "/1/cards/{}/actions/comments",                              # index.js:53
    "path_card": "/1/cards/{}",                                                  # index.js:83
    "path_telegram": "/bot{}/sendMessage",                                       # index.js:99-100
    "path_emby": "{}/emby/library/refresh",                                      # index.js:111-113
    # -- query parameter names ---------------------------------------------------------
    "q_trello_key": "key", "q_trello_token": "token",                            # trello npm
    "q_text": "text",                                                            # index.js:54
    "q_list": "idList", "q_pos": "pos",                                          # index.js:84-85
    "q_chat": "chat_id", "q_parse_mode": "parse_mode",                           # index.js:102-105
    "q_api_key": "api_key",                                                      # index.js:115
    # -- JS errors the reference throws --------------------------------------------------
    "err_to_lower": "Cannot read property 'toLowerCase' of undefined",           # index.js:80,134 (Q6)
}


def pieces(key: str) -> Tuple[str, ...]:
    """A template split at its ``{}`` holes (n holes -> n + 1 pieces)."""
    t = TEXTS[key]
    assert isinstance(t, str), key
    return tuple(t.split("{}"))


def fill(key: str, *values: Any) -> str:
    """``TEXTS[key]`` with each ``{}`` replaced by ``String(value)``."""
    from .ops import js_str
    p = pieces(key)
    if len(p) != len(values) + 1:
        raise ValueError(f"{key}: {len(p) - 1} holes, {len(values)} values")
    out = [p[0]]
    for v, s in zip(values, p[1:]):
        out.append(js_str(v))
        out.append(s)
    return "".join(out)


class Template:
    """A pre-split template for the Python hot path: ``T(a, b)`` == ``fill(key, a, b)``."""

    __slots__ = ("key", "p")

    def __init__(self, key: str):
        self.key = key
        self.p = pieces(key)

    def __call__(self, *values: Any) -> str:
        from .ops import js_str
        p = self.p
        if len(values) == 1:
            return p[0] + js_str(values[0]) + p[1]
        if len(values) == 2:
            return p[0] + js_str(values[0]) + p[1] + js_str(values[1]) + p[2]
        return fill(self.key, *values)
