"""Telegram sink — ``GET https://api.telegram.org/bot{token}/sendMessage`` (index.js:99-106)."""
from __future__ import annotations

from typing import Any, Optional

from .http import HttpClient, HttpResponse, observed, with_query
from .ratelimit import guarded
from ..texts import TEXTS, Template

_TEXT = Template("telegram_text")
_PATH = Template("path_telegram")
_Q_CHAT, _Q_TEXT, _Q_MODE = TEXTS["q_chat"], TEXTS["q_text"], TEXTS["q_parse_mode"]


def deployed_text(name: Any, metadata_id: Any) -> str:
    """``*New Anime:* ${media.name}\\nKitsu: https://kitsu.io/anime/${media.metadataId}`` (index.js:103)."""
    return _TEXT(name, metadata_id)


class TelegramClient:
    def __init__(self, token: Optional[str], http: HttpClient, base_url: str = "https://api.telegram.org",
                 timeout: Optional[float] = None, observer=None, limiter=None, retry=None):
        self.limiter = limiter  # opt-in rate limit / 429 retries (sinks/ratelimit.py)
        self.retry = retry
        self.token = token
        self.http = http
        self.base_url = base_url.rstrip("/")
        self.timeout = timeout
        self.stats = observer.child("telegram") if observer is not None else None

    async def send_message(self, chat_id: Any, text: str, parse_mode: str = TEXTS["telegram_parse_mode"],
                           token: Any = ...) -> HttpResponse:
        # `bot${token}` — an undefined token renders as "botundefined" in the reference
        tok = self.token if token is ... else token
        url = self.base_url + _PATH(tok)
        # request-promise `qs` option -> qs 6.5 (RFC 3986 strict) query encoding
        full = with_query(url, {_Q_CHAT: chat_id, _Q_TEXT: text, _Q_MODE: parse_mode}, rfc3986=True)
        if self.limiter is not None or self.retry is not None:
            r = await guarded(self.limiter, self.retry,
                              lambda: observed(self.stats, self.http.request("GET", full, timeout=self.timeout)))
        else:
            r = await observed(self.stats, self.http.request("GET", full, timeout=self.timeout))
        return r.raise_for_status()  # request-promise: reject on non-2xx
