"""Cluster-wide ``/metrics`` for ``beholder run --workers N``.

The reference exposes one registry per process (``Prom.expose()``, index.js:28).
With N competing-consumer workers on one host, a scraper should still see one
target, so the supervisor serves the merged exposition on the configured port.
Workers listen on internal ports. This is prom-client's ``AggregatorRegistry``
idea, rebuilt for processes that share no memory: the supervisor fetches each
worker's text exposition and merges the samples.

Merge rules, per metric family:

* counters and histograms (buckets, ``_sum``, ``_count``) are summed;
* gauges are summed (in-flight handlers, ring depth, resident memory), except:
  * ``*_start_time_seconds``: min;
  * ``*_info`` and ``process_max_fds``: first value seen;
* a sample present in only some workers is summed over the workers that have it.

The output keeps family order, HELP and TYPE lines from the first worker that
reports them.
"""
from __future__ import annotations

import json
import math
import threading
import time
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .registry import fmt_value

_SUFFIXES = ("_bucket", "_sum", "_count")


def _strategy(family: str, mtype: str) -> str:
    if mtype == "gauge":
        if family.endswith("_start_time_seconds"):
            return "min"
        if family.endswith("_info") or family == "process_max_fds":
            return "first"
    return "sum"


def _parse_value(s: str) -> float:
    return {"+Inf": math.inf, "-Inf": -math.inf, "NaN": math.nan}.get(s) or float(s)


def aggregate(texts: Sequence[str]) -> str:
    """Merges Prometheus text expositions (see module docstring for the rules)."""
    order: List[str] = []
    meta: Dict[str, Dict[str, str]] = {}
    samples: Dict[str, Dict[str, float]] = {}  # family -> {sample key: value}
    sample_order: Dict[str, List[str]] = {}
    for text in texts:
        family = None
        for line in text.split("\n"):  # exposition lines end in \n; a label value may hold U+0085
            if not line:
                continue
            if line.startswith("#"):
                parts = line.split(" ", 3)
                if len(parts) >= 3 and parts[1] in ("HELP", "TYPE"):
                    family = parts[2]
                    if family not in meta:
                        meta[family] = {}
                        order.append(family)
                        samples[family] = {}
                        sample_order[family] = []
                    meta[family].setdefault(parts[1], parts[3] if len(parts) > 3 else "")
                continue
            key, _, val = line.rpartition(" ")
            if not key:
                continue
            name = key.split("{", 1)[0]
            fam = family if family is not None and (name == family or (
                name.startswith(family) and name[len(family):] in _SUFFIXES)) else name
            if fam not in meta:
                meta[fam] = {}
                order.append(fam)
                samples[fam] = {}
                sample_order[fam] = []
            try:
                v = _parse_value(val)
            except ValueError:
                continue
            bucket = samples[fam]
            if key not in bucket:
                bucket[key] = v
                sample_order[fam].append(key)
                continue
            how = _strategy(fam, meta[fam].get("TYPE", "untyped"))
            if how == "sum":
                bucket[key] += v
            elif how == "min":
                bucket[key] = min(bucket[key], v)
            # "first": keep
    out: List[str] = []
    for fam in order:
        m = meta[fam]
        if "HELP" in m:
            out.append(f"# HELP {fam} {m['HELP']}")
        if "TYPE" in m:
            out.append(f"# TYPE {fam} {m['TYPE']}")
        for key in sample_order[fam]:
            out.append(f"{key} {fmt_value(samples[fam][key])}")
    return "\n".join(out) + "\n"


def fetch(url: str, timeout: float = 2.0) -> Optional[str]:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:  # noqa: S310 (loopback worker endpoints)
            return r.read().decode("utf-8", "replace")
    except (OSError, ValueError):
        return None


class ClusterMetricsServer:
    """Supervisor-side HTTP endpoint: ``/metrics`` (merged), ``/healthz`` (all workers up),
    ``/stats`` (per-worker JSON)."""

    def __init__(self, host: str, port: int, worker_ports: Callable[[], List[Tuple[int, int]]],
                 alive: Callable[[], bool], stale_after: int = 5, stale_s: float = 60.0):
        self.host = host
        self.port = port
        self._worker_ports = worker_ports  # [(worker id, port)]
        self._alive = alive
        self._httpd: Optional[ThreadingHTTPServer] = None
        self._thread: Optional[threading.Thread] = None
        # last good exposition per worker: a worker that misses one scrape (a loaded host, a long
        # GC pause) is served from it, so the merged counters never step back (Prometheus would
        # read a drop in a summed counter as a reset); beholder_cluster_worker_up says it was stale
        self._last: Dict[int, Tuple[str, float]] = {}  # worker -> (exposition, monotonic time it was scraped)
        self._failures: Dict[int, int] = {}
        self._streak: Dict[int, int] = {}  # consecutive failed scrapes per worker
        # a worker that keeps failing (dead, wedged) stops being served from its last exposition after
        # `stale_after` consecutive failures or `stale_s` seconds, whichever comes first: its frozen
        # counters must not stay in the merged totals for good
        self.stale_after = stale_after
        self.stale_s = stale_s
        self._lock = threading.Lock()

    def _gather(self, path: str) -> List[Tuple[int, Optional[str]]]:
        return [(i, fetch(f"http://127.0.0.1:{p}{path}")) for i, p in self._worker_ports()]

    def merged_metrics(self) -> str:
        """The workers' expositions summed, a worker whose scrape failed taken from its last good
        one, plus ``beholder_cluster_worker_up{worker}`` and
        ``beholder_cluster_scrape_failures_total{worker}``."""
        got = self._gather("/metrics")
        texts, up = [], []
        now = time.monotonic()
        with self._lock:
            for i in [i for i in self._last if i not in {w for w, _ in got}]:
                del self._last[i]  # no longer a worker of this supervisor
                self._streak.pop(i, None)
            for i, t in got:
                up.append((i, bool(t)))
                if t:
                    self._last[i] = (t, now)
                    self._streak[i] = 0
                else:
                    self._failures[i] = self._failures.get(i, 0) + 1
                    self._streak[i] = self._streak.get(i, 0) + 1
                    last = self._last.get(i)
                    if last is not None and (self._streak[i] > self.stale_after or now - last[1] > self.stale_s):
                        del self._last[i]
                        last = None
                    t = last[0] if last is not None else None
                if t:
                    texts.append(t)
            fails = dict(self._failures)
        extra = ["# HELP beholder_cluster_worker_up 1 when the worker answered this scrape (0: its last good "
                 "exposition was used)", "# TYPE beholder_cluster_worker_up gauge"]
        extra += [f'beholder_cluster_worker_up{{worker="{i}"}} {1 if ok else 0}' for i, ok in up]
        extra += ["# HELP beholder_cluster_scrape_failures_total Worker scrapes that failed since the supervisor "
                  "started", "# TYPE beholder_cluster_scrape_failures_total counter"]
        extra += [f'beholder_cluster_scrape_failures_total{{worker="{i}"}} {fails.get(i, 0)}' for i, _ in up]
        return aggregate(texts) + "\n".join(extra) + "\n"

    def start(self) -> "ClusterMetricsServer":
        outer = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *a):  # quiet
                pass

            def _send(self, code: int, body: bytes, ctype: str) -> None:
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):  # noqa: N802
                path = self.path.split("?", 1)[0]
                if path == "/metrics":
                    self._send(200, outer.merged_metrics().encode(), "text/plain; version=0.0.4; charset=utf-8")
                elif path == "/healthz":
                    ok = outer._alive() and all(t is not None and t.strip() == "ok"
                                                for _, t in outer._gather("/healthz"))
                    self._send(200 if ok else 503, b"ok\n" if ok else b"unavailable\n", "text/plain")
                elif path == "/stats":
                    body = {str(i): (json.loads(t) if t else None) for i, t in outer._gather("/stats")}
                    self._send(200, json.dumps({"workers": body}).encode(), "application/json")
                else:
                    self._send(404, b"not found\n", "text/plain")

        self._httpd = ThreadingHTTPServer((self.host, self.port), Handler)
        self._httpd.daemon_threads = True
        self.port = self._httpd.server_address[1]
        self._thread = threading.Thread(target=self._httpd.serve_forever, daemon=True, name="cluster-metrics")
        self._thread.start()
        return self

    def stop(self) -> None:
        if self._httpd is not None:
            self._httpd.shutdown()
            self._httpd.server_close()
            self._httpd = None
