"""Prometheus metrics registry with prom-client semantics (reference: index.js:27-40,57,136-138).

Why not ``prometheus_client``: it renames counters (appends ``_total`` and
emits ``_created`` samples), but the reference exports a counter literally
named ``beholder_trello_comments`` (no suffix, index.js:36). This registry
renders exactly what prom-client 11 renders:

* ``# HELP`` / ``# TYPE`` per metric, samples ``name{l="v"} value``;
* an unlabelled metric is exported with value ``0`` before its first ``inc``;
  a labelled metric with no children only emits HELP/TYPE;
* numbers are formatted with JavaScript rules (``3`` not ``3.0``).

Counter children are native (:class:`beholder_amd.ops.Counter`) so the hot
path (``progress_updates_total.inc({status})``) is one dict lookup + one C call.
"""
from __future__ import annotations

import math
import re
import threading
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Tuple

from ..ops import Counter as _NativeCounter
from ..ops import native as _native
from ..utils.log import js_number

_Buckets = _native.Buckets

_NAME_RE = re.compile(r"^[a-zA-Z_:][a-zA-Z0-9_:]*$")
_LABEL_RE = re.compile(r"^[a-zA-Z_][a-zA-Z0-9_]*$")

DEFAULT_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10)  # prom-client defaults


def _escape_help(s: str) -> str:
    return s.replace("\\", "\\\\").replace("\n", "\\n")


def _escape_label(s: str) -> str:
    return s.replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def fmt_value(v: float) -> str:
    if v == math.inf:
        return "+Inf"
    if v == -math.inf:
        return "-Inf"
    return js_number(v)


def _label_str(names: Sequence[str], values: Sequence[str], extra: Optional[Tuple[str, str]] = None) -> str:
    pairs = [f'{n}="{_escape_label(str(v))}"' for n, v in zip(names, values)]
    if extra:
        pairs.append(f'{extra[0]}="{_escape_label(extra[1])}"')
    return "{" + ",".join(pairs) + "}" if pairs else ""


class Metric:
    type_name = "untyped"

    def __init__(self, name: str, help: str, label_names: Sequence[str] = ()):
        if not _NAME_RE.match(name):
            raise ValueError(f"invalid metric name {name!r}")
        for ln in label_names:
            if not _LABEL_RE.match(ln) or ln.startswith("__"):
                raise ValueError(f"invalid label name {ln!r}")
        if not help:
            raise ValueError("help is required")
        self.name = name
        self.help = help
        self.label_names = tuple(label_names)
        self._lock = threading.Lock()

    def _key(self, labels) -> Tuple[str, ...]:
        if not self.label_names:
            if labels:
                raise ValueError(f"{self.name} has no labels, got {sorted(labels)}")
            return ()
        if labels is None:
            labels = {}
        if set(labels) - set(self.label_names):
            # prom-client: "Added label "x" is not included in initial labelset"
            bad = sorted(set(labels) - set(self.label_names))
            raise ValueError(f'Added label "{bad[0]}" is not included in initial labelset: {list(self.label_names)}')
        return tuple("" if labels.get(n) is None else str(labels.get(n)) for n in self.label_names)

    def header(self) -> List[str]:
        return [f"# HELP {self.name} {_escape_help(self.help)}", f"# TYPE {self.name} {self.type_name}"]

    def samples(self) -> List[str]:
        raise NotImplementedError

    def render(self) -> str:
        return "\n".join(self.header() + self.samples())


class Counter(Metric):
    """prom-client ``Counter``: ``inc()``, ``inc(n)``, ``inc({labels})``, ``inc({labels}, n)``."""

    type_name = "counter"

    def __init__(self, name: str, help: str, label_names: Sequence[str] = ()):
        super().__init__(name, help, label_names)
        self._children: Dict[Tuple[str, ...], _NativeCounter] = {}
        if not self.label_names:
            self._children[()] = _NativeCounter()
        # fast path: single-label counters keyed by the raw label value
        self._by_value: Dict[str, _NativeCounter] = {}

    def labels(self, *values, **kw) -> _NativeCounter:
        if values and kw:
            raise ValueError("pass label values positionally or by name, not both")
        if values:
            if len(values) != len(self.label_names):
                raise ValueError(f"{self.name} expects {len(self.label_names)} label values")
            key = tuple(str(v) for v in values)
        else:
            key = self._key(kw)
        c = self._children.get(key)
        if c is None:
            with self._lock:
                c = self._children.get(key)
                if c is None:
                    c = _NativeCounter()
                    self._children[key] = c
        return c

    def child(self) -> _NativeCounter:
        """The native counter behind an unlabelled metric (hot-path handle)."""
        if self.label_names:
            raise ValueError(f"{self.name} has labels; use labels()/child_for()")
        return self._children[()]

    def child_for(self, value: str) -> _NativeCounter:
        """Fast path for single-label counters (``progress_updates_total{status}``)."""
        c = self._by_value.get(value)
        if c is None:
            c = self.labels(value)
            self._by_value[value] = c
        return c

    def inc(self, labels=None, value: float = 1.0) -> None:
        if isinstance(labels, (int, float)) and not isinstance(labels, bool):
            labels, value = None, labels
        key = self._key(labels)
        c = self._children.get(key)
        if c is None:
            c = self.labels(*key) if key else self._children[()]
        c.inc(value)

    def get(self, labels=None) -> float:
        c = self._children.get(self._key(labels))
        return c.value if c is not None else 0.0

    def reset(self) -> None:
        with self._lock:
            self._children.clear()
            self._by_value.clear()
            if not self.label_names:
                self._children[()] = _NativeCounter()

    def values(self) -> Dict[Tuple[str, ...], float]:
        return {k: c.value for k, c in list(self._children.items())}

    def samples(self) -> List[str]:
        return [f"{self.name}{_label_str(self.label_names, k)} {fmt_value(c.value)}"
                for k, c in list(self._children.items())]


class Gauge(Metric):
    type_name = "gauge"

    def __init__(self, name: str, help: str, label_names: Sequence[str] = (),
                 collect: Optional[Callable[["Gauge"], None]] = None):
        super().__init__(name, help, label_names)
        self._values: Dict[Tuple[str, ...], float] = {}
        if not self.label_names:
            self._values[()] = 0.0
        self._collect = collect

    def set(self, labels=None, value: Optional[float] = None) -> None:
        if value is None:
            labels, value = None, labels
        self._values[self._key(labels)] = float(value)

    def inc(self, labels=None, value: float = 1.0) -> None:
        if isinstance(labels, (int, float)) and not isinstance(labels, bool):
            labels, value = None, labels
        k = self._key(labels)
        self._values[k] = self._values.get(k, 0.0) + value

    def dec(self, labels=None, value: float = 1.0) -> None:
        if isinstance(labels, (int, float)) and not isinstance(labels, bool):
            labels, value = None, labels
        self.inc(labels, -value)

    def get(self, labels=None) -> float:
        return self._values.get(self._key(labels), 0.0)

    def samples(self) -> List[str]:
        if self._collect is not None:
            self._collect(self)
        return [f"{self.name}{_label_str(self.label_names, k)} {fmt_value(v)}"
                for k, v in list(self._values.items())]


class Histogram(Metric):
    """prom-client ``Histogram`` with fixed cumulative ``le`` buckets."""

    type_name = "histogram"

    def __init__(self, name: str, help: str, label_names: Sequence[str] = (),
                 buckets: Sequence[float] = DEFAULT_BUCKETS):
        if "le" in label_names:
            raise ValueError("le is a reserved label")
        super().__init__(name, help, label_names)
        b = sorted(float(x) for x in buckets)
        if not b:
            raise ValueError("at least one bucket required")
        self.buckets = tuple(b)
        # one native Buckets cell (ops/csrc/py_metrics.cpp) per label set
        self._data: Dict[Tuple[str, ...], Any] = {}
        if not label_names:
            self._data[()] = _Buckets(self.buckets)

    def observe(self, labels=None, value: Optional[float] = None) -> None:
        if value is None:
            labels, value = None, labels
        k = self._key(labels)
        d = self._data.get(k)
        if d is None:
            d = self._data.setdefault(k, _Buckets(self.buckets))
        d.observe(value)

    def labels(self, *values):
        """Pre-resolved per-labelset cell with ``observe(value)`` (hot path: native, no label
        handling per call)."""
        key = tuple(str(v) for v in values) if values else ()
        if len(key) != len(self.label_names):
            raise ValueError(f"{self.name} expects {len(self.label_names)} label values")
        d = self._data.get(key)
        if d is None:
            d = self._data.setdefault(key, _Buckets(self.buckets))
        return d

    def samples(self) -> List[str]:
        out = []
        for k, cell in list(self._data.items()):
            counts, total, n = cell.snapshot()
            cum = 0
            for b, c in zip(self.buckets, counts):
                cum += c
                out.append(f"{self.name}_bucket{_label_str(self.label_names, k, ('le', fmt_value(b)))} {cum}")
            out.append(f"{self.name}_bucket{_label_str(self.label_names, k, ('le', '+Inf'))} {n}")
            out.append(f"{self.name}_sum{_label_str(self.label_names, k)} {fmt_value(total)}")
            out.append(f"{self.name}_count{_label_str(self.label_names, k)} {n}")
        return out


class NativeHistogramView(Metric):
    """Exposes a native log-linear :class:`~beholder_amd.ops.Histogram` (ns) as a
    Prometheus histogram in seconds. Bucket counts are exact up to the native
    histogram's resolution (<0.8% in value)."""

    type_name = "histogram"

    def __init__(self, name: str, help: str, source: Callable[[], object],
                 buckets: Sequence[float] = (0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025,
                                             0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10)):
        super().__init__(name, help, ())
        self._source = source
        self.buckets = tuple(sorted(buckets))

    def samples(self) -> List[str]:
        h = self._source()
        if h is None:
            return []
        out = []
        for b in self.buckets:
            out.append(f'{self.name}_bucket{{le="{fmt_value(b)}"}} {h.count_le(int(b * 1e9))}')
        out.append(f'{self.name}_bucket{{le="+Inf"}} {h.count}')
        out.append(f"{self.name}_sum {fmt_value(h.sum / 1e9)}")
        out.append(f"{self.name}_count {h.count}")
        return out


class Registry:
    """``Prom.new('beholder')`` (index.js:27): a named registry of metrics."""

    def __init__(self, name: str = "beholder"):
        self.name = name
        self._metrics: Dict[str, Metric] = {}
        self._collectors: List[Callable[[], Iterable[Metric]]] = []
        self._lock = threading.Lock()

    def register(self, m: Metric) -> Metric:
        with self._lock:
            if m.name in self._metrics:
                # prom-client: "A metric with the name X has already been registered."
                raise ValueError(f"A metric with the name {m.name} has already been registered.")
            self._metrics[m.name] = m
        return m

    def counter(self, name: str, help: str, label_names: Sequence[str] = ()) -> Counter:
        return self.register(Counter(name, help, label_names))  # type: ignore[return-value]

    def gauge(self, name: str, help: str, label_names: Sequence[str] = (), collect=None) -> Gauge:
        return self.register(Gauge(name, help, label_names, collect))  # type: ignore[return-value]

    def histogram(self, name: str, help: str, label_names: Sequence[str] = (),
                  buckets: Sequence[float] = DEFAULT_BUCKETS) -> Histogram:
        return self.register(Histogram(name, help, label_names, buckets))  # type: ignore[return-value]

    def add_collector(self, fn: Callable[[], Iterable[Metric]]) -> None:
        """Register a callable producing extra metrics at scrape time."""
        self._collectors.append(fn)

    def get(self, name: str) -> Optional[Metric]:
        return self._metrics.get(name)

    def metrics(self) -> List[Metric]:
        ms = list(self._metrics.values())
        for c in self._collectors:
            ms.extend(c())
        return ms

    def render(self) -> str:
        """Prometheus text exposition format 0.0.4."""
        return "\n\n".join(m.render() for m in self.metrics()) + "\n"

    CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"


def parse_exposition(text: str) -> Dict[str, float]:
    """Parse sample lines of a text exposition into ``{'name{labels}': value}`` (tests/tools)."""
    out: Dict[str, float] = {}
    for line in text.split("\n"):
        if not line or line.startswith("#"):
            continue
        key, _, val = line.rpartition(" ")
        v = {"+Inf": math.inf, "-Inf": -math.inf, "NaN": math.nan}.get(val)
        out[key] = float(val) if v is None else v
    return out
