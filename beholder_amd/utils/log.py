"""pino-compatible JSON-lines logger (reference: ``index.js:11-13``).

The reference logs with ``pino({name: path.basename(__filename)})``, i.e. one
JSON object per line::

    {"level":30,"time":1571234567890,"pid":7,"hostname":"box","name":"index.js","msg":"initialized","v":1}

Levels are pino's numeric levels (trace 10 … fatal 60). ``logger.info(obj,
'msg')`` merges ``obj``'s keys into the line, as pino does.

Message formatting follows pino's ``quick-format-unescaped`` for ``%s %d %i
%f %j %o %O %%``. **Documented fix of quirk Q11** (SURVEY.md §2.6): pino v5
silently *drops* positional arguments that have no format specifier, so the
reference's ``logger.info('creating comment on', cardId, 'with text:', text)``
(index.js:51) logs only ``"creating comment on"``. By default we append such extra
arguments space-separated (like ``util.format``) so the information survives;
``service.log.positional_args: drop`` (``Logger(positional_args="drop")``) keeps
pino@5's exact message text, for log-based alerts written against the reference.

Values are rendered with JavaScript's ``String()`` rules (:func:`js_str`), so
message text matches the reference's template literals (``45`` not ``45.0``,
``undefined`` for a missing value).
"""
from __future__ import annotations

import codecs
import json
import math
import os
import socket
import sys
import time
from typing import Any, Dict, Optional, TextIO

LEVELS: Dict[str, float] = {
    "trace": 10, "debug": 20, "info": 30, "warn": 40, "error": 50, "fatal": 60,
    "silent": math.inf,
}


def js_number(x: float) -> str:
    """``String(x)`` for a JS number (ECMAScript Number::toString)."""
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, int):
        return str(x)
    if x != x:
        return "NaN"
    if x == math.inf:
        return "Infinity"
    if x == -math.inf:
        return "-Infinity"
    if x == 0:
        return "0"
    sign = "-" if x < 0 else ""
    r = repr(abs(x))  # shortest round-trip digits
    if "e" in r:
        mant, exp = r.split("e")
        exp_i = int(exp)
    else:
        mant, exp_i = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # decimal point position n relative to the first significant digit
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    n = len(ip) - lead_zeros + exp_i
    digits = digits.rstrip("0") or "0"
    k = len(digits)
    if k <= n <= 21:
        s = digits + "0" * (n - k)
    elif 0 < n <= 21:
        s = digits[:n] + "." + digits[n:]
    elif -6 < n <= 0:
        s = "0." + "0" * (-n) + digits
    else:
        e = n - 1
        es = ("+" if e >= 0 else "-") + str(abs(e))
        s = digits[0] + ("." + digits[1:] if k > 1 else "") + "e" + es
    return sign + s


def js_str(v: Any) -> str:
    """``String(v)`` with JS semantics for the types the service logs."""
    if v is None:
        return "undefined"
    if isinstance(v, str):
        return v
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return js_number(v)
    if isinstance(v, (list, tuple)):
        return ",".join("" if x is None else js_str(x) for x in v)
    if isinstance(v, dict):
        return "[object Object]"
    if isinstance(v, BaseException):
        return f"{type(v).__name__}: {v}"
    return str(v)


def _json_safe(v: Any) -> Any:
    try:
        json.dumps(v)
        return v
    except (TypeError, ValueError):
        return js_str(v)


POSITIONAL_ARGS = ("append", "drop")


def quick_format(args: tuple, drop: bool = False) -> str:
    """Format positional args like pino v5 (see module doc for the Q11 fix; ``drop``: pino v5
    exactly, arguments no format specifier consumes are dropped)."""
    if not args:
        return ""
    f = args[0]
    rest = args[1:]
    if not isinstance(f, str):
        return js_str(f) if drop else " ".join(js_str(a) for a in args)
    if not rest:
        return f
    out = []
    ai = 0
    i = 0
    last = 0
    n = len(f)
    while i < n - 1:
        if f[i] == "%":
            c = f[i + 1]
            if c == "%":
                out.append(f[last:i] + "%")
                i += 2
                last = i
                continue
            if c in "sdifjoO" and ai < len(rest):
                a = rest[ai]
                ai += 1
                if c == "s":
                    rep = js_str(a)
                elif c in "di":
                    try:
                        num = float(a) if not isinstance(a, (int, float)) or isinstance(a, bool) else a
                        if c == "i" and num == num and abs(num) != math.inf:
                            num = float(math.floor(num)) if isinstance(num, float) else num
                        rep = js_number(num)
                    except (TypeError, ValueError):
                        rep = "NaN"
                elif c == "f":
                    try:
                        rep = js_number(float(a))
                    except (TypeError, ValueError):
                        rep = "NaN"
                else:
                    try:
                        rep = json.dumps(a, separators=(",", ":"), ensure_ascii=False)
                    except (TypeError, ValueError):
                        rep = '"[Circular]"'
                out.append(f[last:i] + rep)
                i += 2
                last = i
                continue
        i += 1
    out.append(f[last:])
    s = "".join(out)
    if ai < len(rest) and not drop:
        s += " " + " ".join(js_str(a) for a in rest[ai:])
    return s


from ..ops import native as _native  # noqa: E402  (after js_str: ops configures its fallbacks from us)

_native.configure_text(js_str, lambda v: json.dumps(v, separators=(",", ":"), ensure_ascii=False, default=js_str))


def _writer(stream):
    """``(write, binary)`` for the native sink. A UTF-8 text file with a binary buffer
    (``sys.stdout``, ``open(path, "w")``) takes the formatted bytes directly. The text layer is
    flushed first, so lines never reorder against other writers of the same stream. Anything
    else gets ``str`` through its own ``write``."""
    raw = getattr(stream, "buffer", None)
    enc = getattr(stream, "encoding", None)
    try:
        utf8 = enc is not None and codecs.lookup(enc).name == "utf-8"
    except LookupError:
        utf8 = False
    if raw is None or not utf8 or not callable(getattr(raw, "write", None)):
        return stream.write, False
    text_flush, raw_write = stream.flush, raw.write

    def write(data: bytes) -> int:
        text_flush()
        return raw_write(data)
    return write, True


class _Shared:
    """State shared by a logger and its children: one native sink, one stream."""

    __slots__ = ("stream", "pid", "hostname", "sink")

    def __init__(self, stream, buffer_bytes: int, drop_extra: bool = False):
        self.stream = stream
        self.pid = os.getpid()
        self.hostname = socket.gethostname()
        write, binary = _writer(stream)
        self.sink = _native.LogSink(write, getattr(stream, "flush", None), buffer_bytes, binary, drop_extra)


class Logger(_native.LogCore):
    """pino-compatible logger: ``trace/debug/info/warn/error/fatal(*args)``, ``child(**bindings)``.

    The level methods are implemented in C (:class:`~beholder_amd.ops.LogCore`):
    lines are formatted straight into a native :class:`~beholder_amd.ops.LogSink`
    buffer that is handed to ``stream.write`` in large chunks — on
    :meth:`flush`, when 64 KiB accumulate, and immediately for error/fatal.
    The service flushes after every delivery batch and every 100 ms. A dict
    (merge object) or exception first argument goes through :meth:`_emit`.
    """

    def __init__(self, name: str = "index.js", level: str = "info", stream: Optional[TextIO] = None,
                 bindings: Optional[dict] = None, _shared: Optional[_Shared] = None, buffer_bytes: int = 65536,
                 positional_args: str = "append"):
        super().__init__()
        if level not in LEVELS:
            raise ValueError(f"unknown log level {level!r}")
        if positional_args not in POSITIONAL_ARGS:
            raise ValueError(f"positional_args must be append|drop, not {positional_args!r}")
        self.name = name
        self._shared = _shared or _Shared(stream if stream is not None else sys.stdout, buffer_bytes,
                                          positional_args == "drop")
        self._bindings = dict(bindings or {})
        self._prefix = self._make_prefix()
        self.set_level(level)

    def _make_prefix(self) -> str:
        sh = self._shared
        head = f'"pid":{sh.pid},"hostname":{json.dumps(sh.hostname)},"name":{json.dumps(self.name)}'
        for k, v in self._bindings.items():
            head += f",{json.dumps(str(k))}:{json.dumps(_json_safe(v), ensure_ascii=False)}"
        return head

    # -- configuration -------------------------------------------------------
    def set_level(self, level: str) -> None:
        if level not in LEVELS:
            raise ValueError(f"unknown log level {level!r}")
        self.level = level
        self._min = LEVELS[level]
        self.is_trace = self._min <= 10
        self.is_debug = self._min <= 20
        self.is_info = self._min <= 30
        self._set_core(self._shared.sink, self._prefix, float(self._min))

    @property
    def stream(self) -> TextIO:
        return self._shared.stream

    @stream.setter
    def stream(self, s: TextIO) -> None:
        self._shared.stream = s
        write, binary = _writer(s)
        self._shared.sink.retarget(write, getattr(s, "flush", None), binary)

    @property
    def positional_args(self) -> str:
        """``append`` (Q11 fix) or ``drop`` (pino@5's text); shared with children."""
        return "drop" if self._shared.sink.drop_extra else "append"

    @positional_args.setter
    def positional_args(self, mode: str) -> None:
        if mode not in POSITIONAL_ARGS:
            raise ValueError(f"positional_args must be append|drop, not {mode!r}")
        self._shared.sink.drop_extra = mode == "drop"

    @property
    def counts(self) -> Dict[str, int]:
        """Lines emitted per level (a logger and its children share one table)."""
        return dict(self._shared.sink.counts)

    def child(self, **bindings) -> "Logger":
        b = dict(self._bindings)
        b.update(bindings)
        return Logger(self.name, self.level, bindings=b, _shared=self._shared)

    # -- slow path (merge object / exception first argument) -----------------
    def _emit(self, lvl: int, lname: str, args: tuple) -> None:
        extra_s = None
        if args:
            a0 = args[0]
            if isinstance(a0, dict):
                extra_s = "".join(f",{json.dumps(str(k))}:{json.dumps(_json_safe(v), ensure_ascii=False)}"
                                  for k, v in a0.items()) or None
                args = args[1:]
            elif isinstance(a0, BaseException):
                extra_s = (f',"type":{json.dumps(type(a0).__name__)},'
                           f'"stack":{json.dumps(f"{type(a0).__name__}: {a0}", ensure_ascii=False)}')
                args = args[1:] if len(args) > 1 else (str(a0),)
        self._shared.sink.emit(lvl, self._prefix, extra_s, args)

    def py_line(self, lvl: int, args: tuple, time_ms: Optional[int] = None) -> str:
        """Pure-Python line formatter — the reference the native one is tested against."""
        parts = [f'{{"level":{lvl},"time":{int(time.time() * 1000) if time_ms is None else time_ms},',
                 self._prefix]
        if args:
            parts.append(',"msg":')
            parts.append(json.dumps(quick_format(args, self._shared.sink.drop_extra), ensure_ascii=False))
        parts.append(',"v":1}\n')
        return "".join(parts)

    def flush(self) -> None:
        try:
            self._shared.sink.flush()
        except (OSError, ValueError):
            pass


class NullStream:
    """A write-only sink that discards (used by benches that still format every line)."""

    def __init__(self):
        self.bytes = 0
        self.lines = 0

    def write(self, s: str) -> int:
        self.bytes += len(s)
        self.lines += s.count("\n")
        return len(s)

    def flush(self) -> None:
        pass


class ErrorSampleStream:
    """Discards lines but keeps the first ``keep`` error-level (50+) lines (benches: why did a
    run report handler errors?)."""

    def __init__(self, keep: int = 5):
        self.keep = keep
        self.samples: list = []
        self.bytes = 0

    def write(self, s: str) -> int:
        self.bytes += len(s)
        if len(self.samples) < self.keep and ('"level":50' in s or '"level":60' in s):
            for line in s.split("\n"):  # not splitlines(): U+0085 / U+2028 are text in a JSON string
                if ('"level":50' in line or '"level":60' in line) and len(self.samples) < self.keep:
                    self.samples.append(line[:400])
        return len(s)

    def flush(self) -> None:
        pass


class MemoryStream:
    """Collects lines in memory (tests)."""

    def __init__(self):
        self.lines = []

    def write(self, s: str) -> int:
        self.lines.extend(x for x in s.split("\n") if x)  # lines end in \n only (see ErrorSampleStream)
        return len(s)

    def flush(self) -> None:
        pass

    def records(self):
        return [json.loads(x) for x in self.lines]

    def __iter__(self):
        return iter(self.lines)
