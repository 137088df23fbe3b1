"""Trello sink — the subset of the ``trello`` npm client (0.9.1) beholder uses.

Reference: ``new Trello(key, token)`` (index.js:25) and
``trello.makeRequest(method, path, body)`` for

* comments: ``POST /1/cards/{cardId}/actions/comments {text}`` (index.js:53-55);
* card moves: ``PUT /1/cards/{creatorId} {idList, pos: 2}`` (index.js:83-86).

The npm client sends ``key``/``token`` and every body field as query-string
parameters against ``https://api.trello.com`` and resolves with the response
body on any HTTP status (only transport errors reject). Both behaviours are
kept; ``strict=True`` opts into raising on non-2xx.
"""
from __future__ import annotations

import time
from typing import Any, Mapping, Optional

from .http import HttpClient, HttpError, HttpResponse
from .ratelimit import guarded
from ..texts import TEXTS, Template

COMMENT_FALLBACK = TEXTS["comment_fallback"]  # index.js:54
_K, _T = TEXTS["q_trello_key"], TEXTS["q_trello_token"]
_COMMENT_PATH, _CARD_PATH = Template("path_comment"), Template("path_card")

_METHODS = {"get": "GET", "post": "POST", "put": "PUT", "delete": "DELETE"}


class TrelloClient:
    def __init__(self, key: Optional[str], token: Optional[str], http: HttpClient,
                 base_url: str = "https://api.trello.com", strict: bool = False, timeout: Optional[float] = None,
                 observer=None, limiter=None, retry=None):
        self.limiter = limiter  # opt-in rate limit / 429 retries (sinks/ratelimit.py)
        self.retry = retry
        self.key = key
        self.token = token
        self.http = http
        self.base_url = base_url.rstrip("/")
        self.strict = strict
        self.timeout = timeout
        self.stats = observer.child("trello") if observer is not None else None

    def create_query(self) -> dict:
        return {_K: self.key, _T: self.token}

    async def make_request(self, method: str, path: str, options: Optional[Mapping[str, Any]] = None) -> HttpResponse:
        """``trello.makeRequest(requestMethod, path, options)``."""
        m = _METHODS.get(method) or _METHODS.get(method.lower())
        if m is None:
            raise HttpError("Unsupported requestMethod. Pass one of these methods: POST, GET, PUT, DELETE.")
        if not path.startswith("/"):
            raise HttpError("Path must start with /")
        query = {_K: self.key, _T: self.token, **options} if options else {_K: self.key, _T: self.token}
        if self.limiter is not None or self.retry is not None:
            r = await guarded(self.limiter, self.retry, lambda: self._send(m, path, query))
        else:
            r = await self._send(m, path, query)
        if self.strict:
            r.raise_for_status()
        return r

    async def _send(self, m: str, path: str, query: dict) -> HttpResponse:
        stats = self.stats
        if stats is None:
            return await self.http.request(m, self.base_url + path, params=query, timeout=self.timeout)
        t0 = time.perf_counter()
        try:
            r = await self.http.request(m, self.base_url + path, params=query, timeout=self.timeout)
        except Exception:
            stats.record(None, time.perf_counter() - t0)
            raise
        stats.record(r.status, time.perf_counter() - t0)
        return r

    makeRequest = make_request  # noqa: N815 (reference name)

    async def add_comment(self, card_id: str, text: Optional[str]) -> HttpResponse:
        return await self.make_request("post", _COMMENT_PATH(card_id), {TEXTS["q_text"]: text or COMMENT_FALLBACK})

    async def move_card(self, card_id: str, list_id: str, pos: Any = TEXTS["trello_move_pos"]) -> HttpResponse:
        return await self.make_request("put", _CARD_PATH(card_id), {TEXTS["q_list"]: list_id, TEXTS["q_pos"]: pos})
