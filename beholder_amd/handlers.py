"""Telemetry handlers — the business logic of the reference (index.js:50-155).

:class:`TelemetryHandlers` reproduces, branch for branch:

* ``comment(cardId, text)`` — index.js:50-58 (C8);
* the status handler for ``v1.telemetry.status`` — index.js:62-125 (C10);
* the progress handler for ``v1.telemetry.progress`` — index.js:127-155 (C11).

Quirks kept on purpose, each covered by tests/test_handlers.py:

Q1  status handler has no try/catch: decode / DB / enum / Trello-move errors
    escape and the delivery is left un-acked (the service applies
    ``service.on_status_error``; default ``leave_unacked`` = reference).
Q2  ``NO_TRELLO`` acks right after the DB update and skips Trello, Telegram
    and Emby — for the status handler only.
Q3  Telegram / Emby fire when the *re-read* DB status is ``DEPLOYED``.
Q4  Telegram and Emby share one try: a Telegram failure skips Emby; errors
    are logged at warn and the message is still acked.
Q5  a missing flow-list mapping logs a warn (with the available keys).
Q6  an unknown status enum: status handler throws (un-acked); progress
    handler warns + acks without touching the counter.
Q7  the progress handler always acks.
Q8  card moves use ``pos: 2``; comment text is
    ``"{STATUS}: Progress **{p}%**"`` + ``" (_{host}_)"`` if host is truthy.
Q9  no per-media ordering (opt-in serialisation lives in
    :mod:`beholder_amd.parallel.ordering`).

Log messages are the reference's text, rendered with JS ``String()`` rules. Every
reference-visible string (log text, sink paths and bodies, query names) comes from
:data:`beholder_amd.texts.TEXTS`, which the compiled handlers read too.
"""
from __future__ import annotations

from typing import Any, Callable, Mapping, Optional

from .models import proto
from .sinks.trello import COMMENT_FALLBACK
from .sinks.telegram import deployed_text
from .ops import js_str
from .texts import TEXTS, Template

_LOG_STATUS, _LOG_MOVE = Template("log_status"), Template("log_move")
_LOG_TELEGRAM, _LOG_EMBY = Template("log_telegram"), Template("log_emby")
_LOG_COMMENT, _LOG_PROGRESS, _LOG_MISSING = TEXTS["log_comment"], TEXTS["log_progress"], TEXTS["log_missing_list"]
_WARN_HOOKS, _WARN_PROGRESS = TEXTS["warn_hooks"], TEXTS["warn_progress"]
_COMMENT, _COMMENT_HOST = Template("comment"), Template("comment_host")
_PATH_COMMENT, _PATH_CARD = Template("path_comment"), Template("path_card")
_Q_TEXT, _Q_LIST, _Q_POS = TEXTS["q_text"], TEXTS["q_list"], TEXTS["q_pos"]
_MOVE_POS, _PARSE_MODE, _ERR_TO_LOWER = TEXTS["trello_move_pos"], TEXTS["telegram_parse_mode"], TEXTS["err_to_lower"]

TRELLO_CREATOR = 1  # index.js:79 compares `media.creator === 1`


def js_truthy(v: Any) -> bool:
    """JavaScript truthiness (``""``, ``0``, ``NaN``, ``None``/undefined, ``False`` are falsy)."""
    t = type(v)
    if t is str:
        return v != ""
    if t is bool:
        return v
    if v is None:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v == v and v != 0
    if isinstance(v, str):
        return v != ""
    return True  # objects / arrays (even empty) are truthy


def err_message(err: BaseException) -> str:
    """``err.message || err``."""
    msg = getattr(err, "message", None)
    if isinstance(msg, str) and msg:
        return msg
    s = str(err)
    return s if s else type(err).__name__


def js_object_keys(obj: Mapping) -> list:
    """``Object.keys(obj)`` as strings, in ECMAScript property order: array-index keys
    (canonical integers below 2**32 - 1) ascending, then the other keys in insertion order."""
    idx, rest = [], []
    for k in obj.keys():
        s = k if type(k) is str else js_str(k)
        if s.isdigit() and s.isascii() and (s == "0" or s[0] != "0") and int(s) < 4294967295:
            idx.append((int(s), s))
        else:
            rest.append(s)
    idx.sort()
    return [s for _, s in idx] + rest


class JsTypeError(TypeError):
    """What V8 raises where the reference dereferences ``undefined``."""


def _get(obj: Any, key: str) -> Any:
    """``obj[key]`` with JS semantics on config nodes / dicts (``undefined`` → None)."""
    if type(obj) is dict:
        return obj.get(key)
    if obj is None:
        raise JsTypeError(f"Cannot read property '{key}' of undefined")
    if isinstance(obj, Mapping):
        return obj.get(key)
    try:
        return obj[key]
    except (KeyError, TypeError, IndexError):
        return getattr(obj, key, None)


class TelemetryHandlers:
    """Status / progress handlers bound to their dependencies.

    ``decode_status`` / ``decode_progress`` default to the native codec built
    from the ``.proto`` schema (upb fallback for non-flat schemas).
    """

    def __init__(self, *, config, store, trello, telegram, emby, progress_counter, comments_counter,
                 logger, no_trello: Optional[bool] = None,
                 decode_status: Optional[Callable] = None, decode_progress: Optional[Callable] = None):
        self.config = config
        self.store = store
        self.trello = trello
        self.telegram = telegram
        self.emby = emby
        self.progress_counter = progress_counter
        self.comments_counter = comments_counter
        # hot-path handle (native counter) when the registry provides one
        self._comment_inc = comments_counter.child().inc if hasattr(comments_counter, "child") else \
            comments_counter.inc
        self.log = logger
        self.no_trello = config.no_trello if no_trello is None else bool(no_trello)

        self.status_proto = proto.load("api.TelemetryStatus")      # index.js:47
        self.progress_proto = proto.load("api.TelemetryProgress")  # index.js:46
        self.media_proto = proto.load("api.Media")                 # index.js:48
        dialect = _dialect(config)
        self.decode_status = decode_status or _decoder(self.status_proto, dialect)
        self.decode_progress = decode_progress or _decoder(self.progress_proto, dialect)

        # enumToString tables (index.js:74,134): number -> name, first name wins
        self._status_names_s = self.status_proto.enum("TelemetryStatusEntry")[0]
        self._status_names_p = self.progress_proto.enum("TelemetryStatusEntry")[0]
        # status -> (statusText, progress_updates_total{status=statusText.toLowerCase()}.inc),
        # filled on first use so the labelled child appears exactly when the reference creates it
        self._progress_plan: dict = {}
        # stringToEnum (index.js:94,142)
        self.deployed = proto.string_to_enum(self.status_proto, "TelemetryStatusEntry", "DEPLOYED")
        self.trello_creator = proto.string_to_enum(self.media_proto, "CreatorType", "TRELLO")
        self.lists = config.flow_ids  # index.js:60

    def _hooks_plan(self):
        """The DEPLOYED-hook config reads of index.js:97-115, evaluated once.

        The config is immutable, so the JS expressions are evaluated at first
        use and cached. Dereferences that throw in the reference (e.g.
        ``config.keys.telegram.token`` with no ``keys.telegram``) are kept
        lazy: the cached plan re-raises at the same point of the handler.
        """
        plan = self.__dict__.get("_plan")
        if plan is None:
            cfg = self.config
            inst = cfg.instance
            tg = _get(inst, "telegram")
            tg_on = js_truthy(tg) and js_truthy(_get(tg, "enabled"))
            chat_id = _get(tg, "channel") if tg_on else None
            try:
                token_val = _get(_get(cfg.keys, "telegram"), "token")
                token_exc = None
            except JsTypeError as e:
                token_val, token_exc = None, e

            def tg_token(v=token_val, e=token_exc):
                if e is not None:
                    raise JsTypeError(str(e))
                return v

            keys_emby = _get(cfg.keys, "emby")
            inst_emby = _get(inst, "emby")
            emby_on = (js_truthy(keys_emby) and js_truthy(_get(keys_emby, "token")) and js_truthy(inst_emby)
                       and js_truthy(_get(inst_emby, "enabled")))
            plan = (tg_on, chat_id, tg_token, emby_on, _get(inst_emby, "host") if emby_on else None,
                    _get(keys_emby, "token") if emby_on else None)
            self._plan = plan
        return plan

    @property
    def store(self):
        return self._store

    @store.setter
    def store(self, store) -> None:
        self._store = store
        # synchronous accessors when the backend has them (memory); None -> await the async API
        self._get_nowait = getattr(store, "get_by_id_nowait", None)
        self._update_nowait = getattr(store, "update_status_nowait", None)

    # ------------------------------------------------------------------ C8 ---
    async def comment(self, card_id: Any, text: Optional[str]) -> None:
        """index.js:50-58."""
        self.log.info(_LOG_COMMENT[0], card_id, _LOG_COMMENT[1], text)
        await self.trello.make_request("post", _PATH_COMMENT(card_id), {_Q_TEXT: text or COMMENT_FALLBACK})
        self._comment_inc()

    # ----------------------------------------------------------------- C10 ---
    async def on_status(self, rmsg) -> Any:
        """``v1.telemetry.status`` (index.js:62-125). Exceptions escape on purpose (Q1)."""
        log = self.log
        msg = self.decode_status(rmsg.message.content)  # index.js:63
        media_id = msg.mediaId
        status = msg.status

        log.info(_LOG_STATUS(media_id, status))

        upd = self._update_nowait
        if upd is not None:
            upd(media_id, status)  # index.js:68
        else:
            await self.store.update_status(media_id, status)

        if self.no_trello:  # index.js:70-72 (Q2)
            return rmsg.ack()

        status_text = self._status_names_s.get(status)  # index.js:74 (None = undefined)

        get = self._get_nowait
        media = get(media_id) if get is not None else await self.store.get_by_id(media_id)  # index.js:76

        # TRELLO Movement (index.js:78-90)
        if media.creator == TRELLO_CREATOR:
            if status_text is None:  # `statusText.toLowerCase()` on undefined (Q6)
                raise JsTypeError(_ERR_TO_LOWER)
            lists = self.lists
            list_pointer = _get(lists, status_text.lower())
            if js_truthy(list_pointer):
                log.info(_LOG_MOVE(media_id, media.creatorId))
                await self.trello.make_request("put", _PATH_CARD(media.creatorId),
                                               {_Q_LIST: list_pointer, _Q_POS: _MOVE_POS})
            else:  # Q5
                self._warn_missing_list(status, status_text)

        try:  # index.js:92-122 (Q3, Q4)
            if media.status == self.deployed:
                await self._deployed_hooks(media, media_id)
        except Exception as err:  # noqa: BLE001 — reference catches everything here
            log.warn(_WARN_HOOKS, err_message(err))

        return rmsg.ack()  # index.js:124

    def _warn_missing_list(self, status: Any, status_text: Optional[str]) -> None:
        """index.js:88 (Q5)."""
        text, paren, avail = _LOG_MISSING
        self.log.warn(text, status, paren.replace("{}", js_str(status_text)),
                      avail.replace("{}", ",".join(js_object_keys(self.lists))))  # `${Object.keys(lists)}`

    async def _deployed_hooks(self, media, media_id: Any) -> None:
        """Body of the DEPLOYED branch, index.js:95-118 (the caller holds the try of index.js:92)."""
        log = self.log
        tg_on, chat_id, tg_token, emby_on, emby_host, emby_key = self._hooks_plan()
        if tg_on:
            log.info(_LOG_TELEGRAM(media_id))
            await self.telegram.send_message(chat_id, deployed_text(media.name, media.metadataId),
                                             _PARSE_MODE, token=tg_token())
        if emby_on:
            log.info(_LOG_EMBY(emby_host))
            await self.emby.refresh_library(host=emby_host, api_key=emby_key)

    # ----------------------------------------------------------------- C11 ---
    async def on_progress(self, rmsg) -> Any:
        """``v1.telemetry.progress`` (index.js:127-155). Always acks (Q7)."""
        log = self.log
        try:
            msg = self.decode_progress(rmsg.message.content)  # index.js:129
            media_id = msg.mediaId
            status = msg.status
            progress = msg.progress
            host = msg.host

            log.info(_LOG_PROGRESS[0], media_id, _LOG_PROGRESS[1], status, _LOG_PROGRESS[2], progress)
            plan = self._progress_plan.get(status)
            if plan is None:
                status_text = self._status_names_p.get(status)  # index.js:134
                if status_text is None:  # Q6
                    raise JsTypeError(_ERR_TO_LOWER)
                plan = self._progress_plan[status] = (status_text,
                                                      self.progress_counter.child_for(status_text.lower()).inc)
            status_text, count = plan
            count()  # index.js:136-138

            get = self._get_nowait
            media = get(media_id) if get is not None else await self.store.get_by_id(media_id)  # index.js:140

            if media.creator == self.trello_creator:  # index.js:142
                comment_text = _COMMENT(status_text, progress)  # Q8
                if js_truthy(host):
                    comment_text += _COMMENT_HOST(host)
                await self.comment(media.creatorId, comment_text)
        except Exception as err:  # noqa: BLE001 — index.js:149-151
            log.warn(_WARN_PROGRESS, err_message(err))
            return rmsg.ack()

        return rmsg.ack()  # index.js:154


def native_handlers(handlers: TelemetryHandlers):
    """The compiled handlers (``ops/csrc/py_handlers.cpp``) bound to ``handlers``, or None.

    They run index.js:62-155 as native state machines with the same dependencies
    (logger, decoders, store, sinks, counters), so behaviour is identical to the
    methods above; ``tests/test_handlers.py`` runs every case against both, and
    ``tests/test_native_handlers.py`` fuzzes them against each other. A subclass
    that overrides a handler method keeps the Python path.
    """
    if type(handlers) is not TelemetryHandlers:
        return None
    from .ops import native
    return native.NativeHandlers(handlers)


def _dialect(config) -> str:
    """``service.proto.dialect`` (default ``protobufjs``, the reference's reader)."""
    try:
        d = config.data.get("service", {}).get("proto", {}).get("dialect")
    except AttributeError:
        d = None
    return d or "protobufjs"


def _decoder(ptype, dialect: str = "protobufjs") -> Callable:
    """Native decode if the schema is flat (in ``dialect``), else upb (same field names either way)."""
    from .ops import codec_for
    codec = codec_for(ptype, dialect) or codec_for(ptype)
    if codec is not None:
        return codec.decode
    return lambda data: proto.decode(ptype, data)
