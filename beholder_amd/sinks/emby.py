"""Emby sink — ``GET {emby.host}/emby/library/refresh?api_key=...`` (index.js:110-118)."""
from __future__ import annotations

from typing import Any, Optional

from .http import HttpClient, HttpResponse, observed, with_query
from .ratelimit import guarded
from ..texts import TEXTS, Template

_PATH = Template("path_emby")
_Q_KEY = TEXTS["q_api_key"]


class EmbyClient:
    def __init__(self, host: Optional[str], api_key: Optional[str], http: HttpClient, timeout: Optional[float] = None,
                 observer=None, limiter=None, retry=None):
        self.limiter = limiter  # opt-in rate limit / 429 retries (sinks/ratelimit.py)
        self.retry = retry
        self.host = host
        self.api_key = api_key
        self.http = http
        self.timeout = timeout
        self.stats = observer.child("emby") if observer is not None else None

    async def refresh_library(self, host: Any = ..., api_key: Any = ...) -> HttpResponse:
        h = self.host if host is ... else host
        k = self.api_key if api_key is ... else api_key
        url = _PATH(h)
        full = with_query(url, {_Q_KEY: k}, rfc3986=True)  # request `qs` -> qs 6.5 encoding
        if self.limiter is not None or self.retry is not None:
            r = await guarded(self.limiter, self.retry,
                              lambda: observed(self.stats, self.http.request("GET", full, timeout=self.timeout)))
        else:
            r = await observed(self.stats, self.http.request("GET", full, timeout=self.timeout))
        return r.raise_for_status()
