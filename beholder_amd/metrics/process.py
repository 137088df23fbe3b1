"""Default process metrics — the analogue of prom-client's ``collectDefaultMetrics``.

triton-core's ``Prom.new`` may enable prom-client default metrics (SURVEY.md
§2.5, [inferred]); we export the language-neutral ``process_*`` family with
the same names, plus ``python_gc_*`` in place of the ``nodejs_*`` family.
"""
from __future__ import annotations

import gc
import os
import resource
import time
from typing import List

from .registry import Counter, Gauge, Metric

_CLK_TCK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100
_PAGE = resource.getpagesize()


def _proc_stat():
    try:
        with open("/proc/self/stat", "rb") as f:
            parts = f.read().rsplit(b")", 1)[1].split()
        # fields after ")" start at index 2 (state) of the full list
        utime = int(parts[11]) / _CLK_TCK
        stime = int(parts[12]) / _CLK_TCK
        starttime_ticks = int(parts[19])
        vsize = int(parts[20])
        rss = int(parts[21]) * _PAGE
        return utime, stime, starttime_ticks, vsize, rss
    except (OSError, IndexError, ValueError):
        ru = resource.getrusage(resource.RUSAGE_SELF)
        return ru.ru_utime, ru.ru_stime, 0, 0, ru.ru_maxrss * 1024


def _boot_time() -> float:
    try:
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("btime"):
                    return float(line.split()[1])
    except OSError:
        pass
    return time.time() - time.monotonic()


_START = None


def process_start_time() -> float:
    global _START
    if _START is None:
        st = _proc_stat()
        _START = _boot_time() + st[2] / _CLK_TCK if st[2] else time.time()
    return _START


class _Static(Metric):
    def __init__(self, name, help, type_name, value_fn, label_names=()):
        super().__init__(name, help, label_names)
        self.type_name = type_name
        self._fn = value_fn

    def samples(self) -> List[str]:
        from .registry import _label_str, fmt_value
        out = []
        for labels, v in self._fn():
            out.append(f"{self.name}{_label_str(self.label_names, labels)} {fmt_value(v)}")
        return out


def default_metrics(prefix: str = "") -> List[Metric]:
    """Build the default-metric set (evaluated at scrape time)."""
    p = prefix

    def cpu(idx):
        return lambda: [((), _proc_stat()[idx])]

    def fds():
        try:
            return [((), float(len(os.listdir("/proc/self/fd"))))]
        except OSError:
            return [((), 0.0)]

    def max_fds():
        return [((), float(resource.getrlimit(resource.RLIMIT_NOFILE)[0]))]

    def gc_collections():
        return [((str(i),), float(s.get("collections", 0))) for i, s in enumerate(gc.get_stats())]

    def gc_collected():
        return [((str(i),), float(s.get("collected", 0))) for i, s in enumerate(gc.get_stats())]

    return [
        _Static(p + "process_cpu_user_seconds_total", "Total user CPU time spent in seconds.", "counter", cpu(0)),
        _Static(p + "process_cpu_system_seconds_total", "Total system CPU time spent in seconds.", "counter", cpu(1)),
        _Static(p + "process_cpu_seconds_total", "Total user and system CPU time spent in seconds.", "counter",
                lambda: [((), sum(_proc_stat()[:2]))]),
        _Static(p + "process_start_time_seconds", "Start time of the process since unix epoch in seconds.", "gauge",
                lambda: [((), float(int(process_start_time())))]),
        _Static(p + "process_resident_memory_bytes", "Resident memory size in bytes.", "gauge",
                lambda: [((), float(_proc_stat()[4]))]),
        _Static(p + "process_virtual_memory_bytes", "Virtual memory size in bytes.", "gauge",
                lambda: [((), float(_proc_stat()[3]))]),
        _Static(p + "process_open_fds", "Number of open file descriptors.", "gauge", fds),
        _Static(p + "process_max_fds", "Maximum number of open file descriptors.", "gauge", max_fds),
        _Static(p + "python_gc_collections_total", "Number of times this generation was collected.", "counter",
                gc_collections, ("generation",)),
        _Static(p + "python_gc_objects_collected_total", "Objects collected during gc.", "counter",
                gc_collected, ("generation",)),
    ]


__all__ = ["default_metrics", "process_start_time", "Counter", "Gauge"]
