"""The five BASELINE.json measurement configs.

====  ============  ==========================================================
 #    name          what is measured
====  ============  ==========================================================
 1    plumbing      100 synthetic events on **stdin** of ``python -m beholder_amd run``
                    (real CLI process): all acked, counters exposed
 2    firehose_1k   1k events/s paced producer for N s: sustained ingest rate,
                    receive→ack latency
 3    rate_10k      10k events/s: p50 / p99 ingest (receive→ack) latency
 4    backpressure  100k events/s offered into a small ring with the
                    ``drop_newest`` policy (drop accounting) and with ``block``
                    (producer stall time)
 5    soak          1M events unpaced: throughput, RSS growth, GC pause
                    distribution
====  ============  ==========================================================

Every in-process config runs the real service path (native reader thread on
an OS pipe → ring → handlers → store → metrics → sinks → acks) with sinks
stubbed in-process and info logs written to /dev/null.

Usage: ``python -m beholder_amd bench [all|<name>...] [--out FILE]``
"""
from __future__ import annotations

import argparse
import asyncio
import gc
import json
import os
import resource
import subprocess
import sys
import tempfile
import threading
import time
from typing import Dict, List, Optional

from .generator import Workload, bench_config

CONFIGS = ("plumbing", "firehose_1k", "rate_10k", "backpressure", "soak", "amqp", "io_bound", "io_bound_wide", "http_tcp", "tcp_e2e", "tls_e2e",
           "tcp_e2e_preconnect", "tls_e2e_preconnect")


def _rss_mb() -> float:
    try:
        with open("/proc/self/statm") as f:
            return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2**20
    except OSError:
        return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024


def _heap_mb() -> Optional[Dict[str, float]]:
    """glibc's view of this process's malloc heap (mallinfo2): bytes in use, bytes free inside
    the heap, and the heap's size (main arena plus mmapped chunks). RSS growth with ``inuse``
    flat is fragmentation, not a leak. None off glibc."""
    global _MALLINFO
    if _MALLINFO is None:
        try:
            import ctypes

            class _MI2(ctypes.Structure):
                _fields_ = [(n, ctypes.c_size_t) for n in ("arena", "ordblks", "smblks", "hblks", "hblkhd",
                                                           "usmblks", "fsmblks", "uordblks", "fordblks",
                                                           "keepcost")]
            fn = ctypes.CDLL("libc.so.6").mallinfo2
            fn.restype = _MI2
            _MALLINFO = fn
        except (OSError, AttributeError):
            _MALLINFO = False
    if not _MALLINFO:
        return None
    m = _MALLINFO()
    mb = 1 / 2**20
    return {"inuse": round(m.uordblks * mb, 2), "free": round(m.fordblks * mb, 2),
            "size": round((m.arena + m.hblkhd) * mb, 2)}


_MALLINFO = None


class GcPauses:
    """Collects GC pause durations through ``gc.callbacks``."""

    def __init__(self):
        self.pauses_ns: List[int] = []
        self.by_gen = [0, 0, 0]
        self._t0 = 0

    def _cb(self, phase, info):
        if phase == "start":
            self._t0 = time.perf_counter_ns()
        elif self._t0:
            self.pauses_ns.append(time.perf_counter_ns() - self._t0)
            self.by_gen[info["generation"]] += 1
            self._t0 = 0

    def __enter__(self):
        gc.callbacks.append(self._cb)
        return self

    def __exit__(self, *exc):
        gc.callbacks.remove(self._cb)

    def summary(self) -> Dict[str, float]:
        p = sorted(self.pauses_ns)
        if not p:
            return {"count": 0}

        def pct(q):
            return p[min(len(p) - 1, int(q / 100 * len(p)))] / 1e3

        return {"count": len(p), "p50_us": pct(50), "p99_us": pct(99), "max_us": p[-1] / 1e3,
                "total_ms": sum(p) / 1e6, "by_generation": list(self.by_gen)}


class _Producer(threading.Thread):
    """Writes pre-framed events into a pipe at ``rate`` events/s (0 = unpaced).

    Paced runs go through :func:`~beholder_amd.ops.bench_native.paced_write`: the pacing loop is native and
    holds no GIL (clock_nanosleep to each event's due time, 1 ns timer slack), so the producer
    neither competes with the consumer's event loop for the GIL nor adds its own wake-up jitter to
    the receive→ack latency of BASELINE configs 2-4."""

    def __init__(self, wfd: int, events, rate: float):
        super().__init__(daemon=True, name="producer")
        from array import array

        from ..ops import frame
        self.wfd = wfd
        self.rate = rate
        chunks = [frame(t, p) for t, p in events]
        self.offered = len(chunks)
        ends = array("Q")
        pos = 0
        for c in chunks:
            pos += len(c)
            ends.append(pos)
        self.data = b"".join(chunks)
        self.ends = ends.tobytes()
        self.elapsed = 0.0
        self.writes = 0
        self.t0_ns = 0  # paced: CLOCK_MONOTONIC time frame 0 was due (frame i: + i * 1e9 / rate)

    def run(self):
        try:
            # the producer stands in for the broker, another process in production: when it shares
            # a CPU with the consumer's threads it yields to them (nice +10 for this thread only)
            # instead of preempting the event loop it is measuring
            try:
                os.setpriority(os.PRIO_PROCESS, threading.get_native_id(), 10)
            except (OSError, AttributeError):
                pass
            if self.rate <= 0:
                t0 = time.perf_counter()
                mv = memoryview(self.data)
                while mv:
                    n = os.write(self.wfd, mv[:1 << 20])
                    mv = mv[n:]
                self.elapsed = time.perf_counter() - t0
            else:
                from ..ops.bench_native import paced_write
                self.elapsed, self.writes, self.t0_ns = paced_write(self.wfd, self.data, self.ends,
                                                                    float(self.rate))
        except OSError:
            pass
        finally:
            os.close(self.wfd)


async def _run_inproc(events, rate: float, *, policy: str = "block", capacity_events: int = 0,
                      n_media: int = 10000, media=None, log_level: str = "info", rss_probe=None,
                      sink_delay_s: float = 0.0, gc_probe: "Optional[GcPauses]" = None,
                      http=None, sink_url: Optional[str] = None, prefetch: Optional[int] = None,
                      reset_latency_after: int = 0) -> dict:
    from ..config import Config
    from ..service import Service
    from ..sinks import RecordingHttpClient
    from ..store import MemoryStore
    from ..transport.ingest import FdSource
    from ..utils.hostinfo import thread_run_delay_ns
    from ..utils.log import Logger

    rfd, wfd = os.pipe()
    cfgd = bench_config()
    cfgd["service"]["log"]["level"] = log_level
    if prefetch is not None:
        cfgd["service"]["prefetch"] = prefetch
    if sink_url:  # real HTTP: every sink points at the fake endpoint
        cfgd["service"]["endpoints"] = {"trello": sink_url, "telegram": sink_url}
        cfgd["instance"]["emby"]["host"] = sink_url
    from ..utils.log import ErrorSampleStream
    sink = ErrorSampleStream()
    src = FdSource(fd=rfd, policy=policy, capacity_events=capacity_events)
    if http is None:
        http = RecordingHttpClient(keep=8, delay_s=sink_delay_s)
    svc = Service(Config.from_dict(cfgd), source=src, store=MemoryStore(media), http=http,
                  logger=Logger(stream=sink, level=log_level), serve_metrics=False)
    max_inflight = [0]
    rss_curve: List[float] = []
    sampler = None
    if rss_probe is not None:
        async def sample_rss():
            while True:
                await asyncio.sleep(0.5)
                rss_curve.append(round(_rss_mb(), 1))
    if sink_delay_s:
        async def watch():
            while True:
                max_inflight[0] = max(max_inflight[0], len(svc._inflight))
                await asyncio.sleep(0.001)
        watcher = asyncio.ensure_future(watch())
    await svc.init()
    prod = _Producer(wfd, events, rate)
    if rss_probe is not None:
        gc.collect()
        rss_probe.append(_rss_mb())  # service initialised, workload already in memory
    if gc_probe is not None:
        gc_probe.__enter__()  # steady state only: init's own collect+freeze is not a run pause
    if rss_probe is not None:
        sampler = asyncio.ensure_future(sample_rss())
    cold: dict = {}
    if reset_latency_after:  # warm-up (connection pools filling) kept out of the latency histograms
        async def reset_later():
            while _settled(src.settler) < reset_latency_after:
                await asyncio.sleep(0.001)
            cold.update(src.settler.handle_latency.summary())
            src.settler.reset_latency()
        resetter = asyncio.ensure_future(reset_later())
    mon = None
    if rate > 0:  # paced: where a slow receive->ack came from (the loop stalled, or was preempted)
        from .stallmon import StallMonitor
        # 2 ms threshold: an idle loop's timer wakes up to ~1 ms late by construction (epoll_wait
        # takes whole milliseconds and asyncio rounds the timeout up), which is not a stall
        mon = StallMonitor(threshold_us=2000).start()
    if rate > 0:  # every delivery's (receive, start, ack) times, for the due -> ack latency below
        src.settler.trace_slow(1, prod.offered + 16)
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    rt0 = resource.getrusage(resource.RUSAGE_THREAD)
    rd0 = thread_run_delay_ns()
    t0 = time.perf_counter()
    prod.start()
    stats = await svc.run()
    if reset_latency_after:
        resetter.cancel()
    elapsed = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    rt1 = resource.getrusage(resource.RUSAGE_THREAD)
    rd1 = thread_run_delay_ns()
    if mon is not None:
        mon.stop()
    cpu_s = (ru1.ru_utime + ru1.ru_stime) - (ru0.ru_utime + ru0.ru_stime)
    prod.join()
    if gc_probe is not None:
        gc_probe.__exit__(None, None, None)
    if sampler is not None:
        sampler.cancel()
    if rss_probe is not None:
        rss_probe.append(_rss_mb())  # after 1M events, before teardown
    if sink_delay_s:
        watcher.cancel()
    due = _due_latencies(src.settler, prod, stats["source"]) if rate > 0 else {}
    await svc.close()
    s = stats["source"]
    return {
        **due,
        "offered": prod.offered, "accepted": s["pushed"], "dropped": s["dropped_total"],
        "acked": s["acked"], "abandoned": s["abandoned"], "errors": sum(stats.get("handler_errors", {}).values()),
        "elapsed_s": elapsed, "producer_s": prod.elapsed,
        "ingest_rate_eps": s["acked"] / elapsed if elapsed else 0.0,
        "offered_rate_eps": prod.offered / prod.elapsed if prod.elapsed else 0.0,
        "ingest_latency_us": {k: v / 1e3 for k, v in stats["ingest_latency_ns"].items() if k.startswith("p")},
        "handle_latency_us": {k: v / 1e3 for k, v in stats["handle_latency_ns"].items() if k.startswith("p")},
        # the two hops of ingest latency: reader push -> handler start (ring + loop wake), start -> ack
        "queue_latency_us": {k: v / 1e3 for k, v in stats["queue_latency_ns"].items() if k.startswith("p")},
        "idle_wakeups": s.get("idle_wakeups"),
        "producer_writes": prod.writes,
        "producer_blocked_ms": s["blocked_ns"] / 1e6, "ring_high_water": s["high_water_events"],
        "sink_requests": (http.count if hasattr(http, "count") else
                          http.counts["requests"] if hasattr(http, "counts") else None),
        "max_inflight": max_inflight[0],
        "cpu_us_per_event": cpu_s / s["acked"] * 1e6 if s["acked"] else None,
        # the event loop's thread: preemptions by other work on its CPU, and its stalls >= 2 ms
        "loop_thread_nivcsw": rt1.ru_nivcsw - rt0.ru_nivcsw,
        # ... and its time runnable but without a CPU (a wake-up the host delayed)
        "loop_run_delay_us": (rd1 - rd0) / 1e3 if rd0 is not None and rd1 is not None else None,
        **({"loop": mon.summary()} if mon is not None else {}),
        "error_samples": sink.samples,
        **({"rss_curve_mb": rss_curve} if rss_probe is not None else {}),
        **({"warmup_events": reset_latency_after,
            "warmup_handle_latency_us": {k: v / 1e3 for k, v in cold.items() if k.startswith("p")}}
           if reset_latency_after else {}),
    }


def _due_latencies(settler, prod: "_Producer", source_stats: dict) -> dict:
    """For a paced run: each event's latency from its *due time* (when the producer was to write
    it: ``t0 + i / rate``), not from when the reader thread received it. ``due_to_ack`` therefore
    also holds the producer's own lateness, the pipe and the reader thread's wake-up, which the
    receive -> ack histograms cannot see; ``due_to_recv`` is that part alone. Computed only when
    every offered event was delivered and traced (no drops), so event i is the i-th started."""
    recs, lost = settler.slow_deliveries()
    if lost or source_stats.get("dropped_total") or len(recs) != prod.offered or not prod.t0_ns:
        return {}
    recs.sort(key=lambda r: r[1])  # dispatch order = arrival order = frame order
    ns_per = 1e9 / prod.rate
    to_ack = []
    to_recv = []
    for i, (recv, _start, settle) in enumerate(recs):
        d = prod.t0_ns + int(i * ns_per)
        to_ack.append(max(0, settle - d))
        to_recv.append(max(0, recv - d))

    def pct(xs):
        xs.sort()
        n = len(xs)
        return {"p50": xs[n // 2] / 1e3, "p99": xs[min(n - 1, int(n * 0.99))] / 1e3,
                "p999": xs[min(n - 1, int(n * 0.999))] / 1e3, "max": xs[-1] / 1e3}
    return {"due_to_ack_us": pct(to_ack), "due_to_recv_us": pct(to_recv)}


def run_config(name: str, *, duration_s: Optional[float] = None, events: Optional[int] = None,
               seed: int = 0) -> dict:
    w = Workload(n_media=10000, seed=seed)
    if name == "plumbing":
        return _plumbing(w)
    if name == "firehose_1k":
        d = duration_s or 5.0
        res = asyncio.run(_run_inproc(w.events(int(1000 * d)), 1000, media=w.media))
    elif name == "rate_10k":
        d = duration_s or 5.0
        res = asyncio.run(_run_inproc(w.events(int(10000 * d)), 10000, media=w.media))
    elif name == "backpressure":
        d = duration_s or 3.0
        evs = w.events(int(100000 * d))
        res = {"drop_newest": asyncio.run(_run_inproc(evs, 100000, policy="drop_newest", capacity_events=4096,
                                                      media=w.media)),
               "block": asyncio.run(_run_inproc(evs, 100000, policy="block", capacity_events=4096,
                                                media=w.media)),
               # overload: the same events offered unpaced (pipe speed) into the small ring
               "overload_drop_newest": asyncio.run(_run_inproc(evs, 0, policy="drop_newest",
                                                               capacity_events=4096, media=w.media))}
        dn = res["drop_newest"]
        res.update({"offered": dn["offered"], "accepted": dn["accepted"], "dropped": dn["dropped"]})
    elif name == "io_bound":
        # every sink call waits 2 ms (network): throughput is bounded by prefetch / latency
        res = asyncio.run(_run_inproc(w.events(events or 100_000), 0, media=w.media, sink_delay_s=0.002))
        res["sink_delay_ms"] = 2.0
        res["prefetch"] = 100
    elif name == "io_bound_wide":
        # production sinks answer in ~tens of ms (Trello / Telegram over the internet): throughput per
        # worker is prefetch / latency, so raise prefetch. 20 ms sinks with prefetch 2000.
        res = asyncio.run(_run_inproc(w.events(events or 200_000), 0, media=w.media, sink_delay_s=0.020,
                                      prefetch=2000))
        res["sink_delay_ms"] = 20.0
        res["prefetch"] = 2000
    elif name == "http_tcp":
        res = _http_tcp(w, events or 100_000)
    elif name == "tcp_e2e":
        res = _tcp_e2e(events or 100_000)
    elif name == "tls_e2e":
        res = _tcp_e2e(events or 100_000, http_servers=4, tls=True)  # TLS fakes cost more CPU per request
    elif name in ("tcp_e2e_preconnect", "tls_e2e_preconnect"):
        # service.http.preconnect = prefetch: the warm-up no longer opens sink connections per delivery
        tls = name.startswith("tls")
        res = _tcp_e2e(events or 100_000, http_servers=4 if tls else 2, tls=tls, preconnect=100)
    elif name == "amqp":
        res = _amqp(events or 200_000)
    elif name == "soak":
        n = events or 1_000_000
        evs = w.events(n)
        probe: list = []
        g = GcPauses()
        res = asyncio.run(_run_inproc(evs, 0, media=w.media, rss_probe=probe, gc_probe=g))
        # RSS of the service itself: measured after init with the workload already generated,
        # and again after all n events went through (so the workload's own memory is excluded)
        res["rss_start_mb"] = probe[0]
        res["rss_end_mb"] = probe[1]
        res["rss_growth_mb"] = probe[1] - probe[0]
        res["rss_peak_mb"] = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024
        res["gc_pauses"] = g.summary()
    else:
        raise ValueError(f"unknown config {name!r} (one of {', '.join(CONFIGS)})")
    res["config"] = name
    return res


SLOW_TRACE_NS = 500_000  # deliveries slower than this (start -> ack) are traced for attribution


def _settled(settler) -> int:
    return settler.acked + settler.abandoned + settler.nacked + settler.rejected


async def _wait_acked(settler, n: int, task, stall_s: float = 15.0) -> None:
    """Until n deliveries are settled one way or another (acked, or abandoned under Q1), the
    service stops, or nothing moves for ``stall_s`` (a broken run must not hang the bench).

    The poll runs on the measured event loop, so it sleeps about a quarter of the remaining time
    at the rate seen so far (at least 1 ms, at most 50 ms and twice the previous sleep): a fixed
    1 ms poll made ~1,000 bench wake-ups per second of the consumer's CPU."""
    last, t_last = -1, time.monotonic()
    rate = 0.0
    prev = 0.001  # each sleep at most doubles the last one: a rate still ramping up (the
    # warm-up's first connections) is not trusted for a long sleep that would overshoot n
    while not task.done():
        done = _settled(settler)
        if done >= n:
            return
        now = time.monotonic()
        if done != last:
            if last >= 0 and now > t_last:
                rate = (done - last) / (now - t_last)
            last, t_last = done, now
        elif now - t_last > stall_s:
            return
        wait = (n - done) / rate / 4 if rate > 0 else 0.001
        prev = min(0.05, max(0.001, min(wait, 2 * prev)))
        await asyncio.sleep(prev)


def _die_with_parent():
    """preexec_fn: the endpoint gets SIGTERM when the process that started it dies (a bench
    killed by a timeout must not leave its fakes running). Resolved before the fork."""
    try:
        import ctypes
        prctl = ctypes.CDLL(None, use_errno=True).prctl
    except (OSError, AttributeError):
        return None
    parent = os.getpid()

    def arm():
        prctl(1, 15, 0, 0, 0)  # PR_SET_PDEATHSIG, SIGTERM
        if os.getppid() != parent:  # the parent died before the signal was armed
            os._exit(1)
    return arm


def _spawn(module: str, copies: int = 1, args=()) -> "tuple":
    """Starts ``copies`` of a bench endpoint process sharing one port (SO_REUSEPORT).
    Returns ``(port, procs)``; each process printed ``READY <port>``."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    procs: list = []
    port = 0
    try:
        for _ in range(copies):
            p = subprocess.Popen([sys.executable, "-m", module, "--port", str(port), *args],
                                 stdout=subprocess.PIPE, text=True, env=env, cwd=root,
                                 preexec_fn=_die_with_parent())
            procs.append(p)
            line = p.stdout.readline().split()
            if not line or line[0] != "READY":
                raise RuntimeError(f"{module} failed to start")
            port = int(line[1])
    except BaseException:
        _reap(procs)
        raise
    return port, procs


def _reap(procs, stalls: Optional[list] = None) -> Dict[str, int]:
    """SIGTERM the endpoint processes; sums their ``DONE key=value`` counters. ``stalls``
    collects each process's ``STALLS`` report (:mod:`.stallmon`)."""
    import subprocess

    from .stallmon import parse_stall_lines
    total: Dict[str, int] = {}
    for p in procs:
        if p.poll() is None:
            p.terminate()
        try:
            out = p.communicate(timeout=10)[0] or ""
        except subprocess.TimeoutExpired:
            p.kill()
            continue
        for ln in out.split("\n"):
            if ln.startswith("DONE "):
                for kv in ln.split()[1:]:
                    k, _, v = kv.partition("=")
                    if v.isdigit():
                        total[k] = total.get(k, 0) + int(v)
        if stalls is not None:
            stalls.extend(parse_stall_lines(out))
    return total


def _slowest(slow, n_measured: int, frac: float = 0.001) -> list:
    """The slowest ``frac`` of ``n_measured`` deliveries among the traced ``(recv, start, settle)``."""
    k = max(1, int(round(n_measured * frac)))
    return sorted(slow, key=lambda x: x[2] - x[1], reverse=True)[:k]


def _attribution(slow, consumer, fakes: list) -> dict:
    """Blames the slow deliveries on the process that stalled under them (:func:`.stallmon.attribute`),
    and reports each process's own loop lag / GC figures next to it."""
    from .stallmon import attribute
    sources: Dict[str, list] = {"consumer": consumer.loop_stalls + consumer.gc_pauses}
    per_proc = {"consumer": consumer.summary()}
    for i, f in enumerate(fakes):
        name = f.get("name", "fake")
        sources.setdefault(name, []).extend(tuple(x) for x in f.get("stall_intervals", []))
        per_proc[f"{name}{i}"] = {k: v for k, v in f.items() if k not in ("stall_intervals", "name")}
    out = attribute(slow, sources)
    out["slowest_us"] = [round((e - s) / 1e3, 1) for _, s, e in slow[:5]]
    out["processes"] = per_proc
    return out


def _http_tcp(w: Workload, n: int, servers: int = 3, clients=("h1", "aiohttp")) -> dict:
    """Sinks over real TCP: n events through the service with the production HTTP client
    (``h1``) and with ``aiohttp``, against ``servers`` fake endpoint processes sharing one
    port. About half the events make a Trello / Telegram / Emby request. ``prefetch`` (100)
    bounds the requests in flight, as in production."""
    from ..sinks import AiohttpClient, H1Client

    port, procs = _spawn("beholder_amd.bench.http_sink_server", servers)
    out: dict = {"servers": servers, "events": n}
    try:
        url = f"http://127.0.0.1:{port}"
        evs = w.events(n)
        for kind, cls in (("h1", H1Client), ("aiohttp", AiohttpClient)):
            if kind not in clients:
                continue
            out[kind] = asyncio.run(_run_inproc(evs, 0, media=w.media, http=cls(timeout_s=30), sink_url=url,
                                                reset_latency_after=min(5000, n // 10)))
    finally:
        out["server_requests_total"] = _reap(procs).get("requests", 0)
    return out


def _io_counts(src) -> Dict[str, int]:
    """Socket call counts of this process so far: NetConn sends / receives by kind, NetPoller
    callbacks (ops io_counts) and the AMQP connection's reads / writes."""
    from ..ops import native
    c = dict(native.io_counts())
    st = src.stats()
    c["amqp_reads"], c["amqp_writes"] = st.get("reads", 0), st.get("writes", 0)
    return c


async def _windows(settler, mon, start: int, n: int, size: int, task, t0: float, out: dict):
    """_tcp_e2e's measured phase in windows of ``size`` settled deliveries: per window the
    handle / ingest latency percentiles (the settler's histograms, merged into the whole phase's
    and then cleared), the RSS and the loop stalls seen. Returns (RSS half-way, merged histograms)."""
    from ..ops import Histogram
    from ..utils.hostinfo import thread_run_delay_ns
    kinds = ("handle", "ingest", "queue")
    merged = {k: Histogram() for k in kinds}
    windows: list = []
    rss_mid = None
    done, t_prev = start, t0
    stalls_prev = 0
    rq_prev, ru_prev = thread_run_delay_ns(), resource.getrusage(resource.RUSAGE_SELF)
    while done < n and not task.done():
        target = min(n, done + size)
        await _wait_acked(settler, target, task)
        now = time.perf_counter()
        got = _settled(settler) - done
        w = {"t_s": round(now - t0, 2), "events": got,
             "events_per_sec": round(got / (now - t_prev), 1) if now > t_prev else None}
        for k in kinds:
            h = getattr(settler, f"{k}_latency")
            summ = h.summary()
            if k != "queue":
                w[f"{k}_p50_us"] = round(summ["p50"] / 1e3, 2) if summ["count"] else None
                w[f"{k}_p99_us"] = round(summ["p99"] / 1e3, 2) if summ["count"] else None
                w[f"{k}_p999_us"] = round(summ["p999"] / 1e3, 2) if summ["count"] else None
                w[f"{k}_max_us"] = round(summ["max"] / 1e3, 2) if summ["count"] else None
            merged[k].merge(h)
        settler.reset_latency()
        w["rss_mb"] = round(_rss_mb(), 2)
        w["heap_mb"] = _heap_mb()
        w["loop_stalls"] = len(mon.loop_stalls) - stalls_prev
        stalls_prev = len(mon.loop_stalls)
        # the loop thread's wait for a CPU and the process's involuntary switches in the window:
        # stalls with little work settled inside them and a high run delay were the consumer
        # descheduled, not its loop blocked
        rq, ru = thread_run_delay_ns(), resource.getrusage(resource.RUSAGE_SELF)
        w["run_delay_ms"] = round((rq - rq_prev) / 1e6, 2) if rq is not None and rq_prev is not None else None
        w["nivcsw"] = ru.ru_nivcsw - ru_prev.ru_nivcsw
        w["cpu_us_per_event"] = round(((ru.ru_utime + ru.ru_stime) - (ru_prev.ru_utime + ru_prev.ru_stime)) / got * 1e6,
                                      2) if got else None
        rq_prev, ru_prev = rq, ru
        windows.append(w)
        print("window " + json.dumps(w), file=sys.stderr, flush=True)  # a long run shows progress
        if rss_mid is None and target >= start + (n - start) // 2:
            rss_mid = _rss_mb()
        done, t_prev = _settled(settler), now
    out["windows"] = windows
    return (rss_mid if rss_mid is not None else _rss_mb()), merged


def _tcp_e2e(n: int, http_servers: int = 2, pg_servers: int = 1, tls: bool = False, preconnect: int = 0,
             max_connecting: int = 8, hooks: Optional[tuple] = None, rate: float = 0.0,
             window_events: int = 0, stall_period_s: float = 0.001) -> dict:
    """Production-shaped: every dependency over real TCP. A replay AMQP broker streams n
    events (prefetch 100, index.js:43). Each handler reads / updates the media row in a
    fake Postgres (pipelined ``pgwire``). Every sink call goes to a fake HTTP endpoint
    (keep-alive ``h1`` client). The fakes are separate processes; the numbers describe
    the consumer process. Postgres is one native fake process (pg_sink_server.py: the asyncio one
    saturated when SO_REUSEPORT put the pool on one of two copies). ``tls`` (config ``tls_e2e``): the sinks are HTTPS, as Trello and
    Telegram are in production (certificate verified against the bench's own CA). ``preconnect``:
    ``service.http.preconnect`` (sink connections opened at init, before the clock).
    ``max_connecting``: ``service.http.max_connecting`` (connects + handshakes in flight per origin).
    ``hooks``: ``(start, stop)`` callables run around the measured phase (scripts/cprof.py).
    ``rate``: the broker paces its sends at that many events per second (BASELINE configs 2-4 on
    the production path: each event's receive->ack latency with its Postgres and HTTP round trips,
    not queueing behind a saturated prefetch window); the warm-up is then a tenth of the events.
    ``window_events``: the measured phase is cut into windows of that many settled deliveries
    (paced: a fixed time each); each window's latency percentiles, RSS and loop stalls are
    reported (``windows``), and the whole-phase percentiles merge the windows' histograms
    (scripts/paced_soak.py: is the production path as fast in its tenth minute as in its first?).
    ``stall_period_s``: the stall monitor's tick on the consumer's loop (each tick is a wake-up of
    that loop, billed to the consumer's CPU: at 1k events/s the default is one tick per event)."""
    from ..config import Config
    from ..service import Service
    from ..sinks import H1Client
    from ..store.postgres import PostgresStore
    from ..transport.amqp import AmqpSource
    from ..utils.hostinfo import cgroup_cpu_stat, cgroup_delta, proc_cpu_s, thread_run_delay_ns
    from ..utils.log import Logger
    from .stallmon import StallMonitor

    warm = n // 10 if rate else min(5000, n // 10)
    bargs = ("--events", str(n)) + (("--rate", str(rate)) if rate else ())
    bport, bprocs = _spawn("beholder_amd.bench.replay_broker", 1, bargs)
    procs = list(bprocs)
    out: dict = {"events": n, "prefetch": 100, "preconnect": preconnect, "max_connecting": max_connecting,
                 "rate": rate}
    diag = None
    try:
        hport, hp = _spawn("beholder_amd.bench.http_sink_server", http_servers, ("--tls",) if tls else ())
        procs += hp
        pport, pp = _spawn("beholder_amd.bench.pg_sink_server", pg_servers, ("--media", "10000", "--seed", "0"))
        procs += pp
        url = f"{'https' if tls else 'http'}://127.0.0.1:{hport}"
        out["tls"] = tls
        kinds = [("broker", p) for p in bprocs] + [("http", p) for p in hp] + [("pg", p) for p in pp]
        # the box's core speed right before the phase (the same fixed-work loop as bench.py's
        # calib_ns): a slow phase on a slow core says so on the line
        from ..ops.bench_native import calib
        out["calib_ns"] = min(calib(4_000_000)[0] for _ in range(3))

        async def go():
            cfgd = bench_config()
            cfgd["service"]["endpoints"] = {"trello": url, "telegram": url}
            cfgd["instance"]["emby"]["host"] = url
            cfgd["service"].setdefault("http", {})["preconnect"] = preconnect
            sink = open(os.devnull, "w", buffering=1 << 16)
            src = AmqpSource(f"amqp://guest:guest@127.0.0.1:{bport}/", prefetch=100)
            store = PostgresStore(f"postgres://beholder@127.0.0.1:{pport}/media", pool_size=4)
            if tls:
                from .http_sink_server import TLS_CERT
                http = H1Client(timeout_s=30, ssl_cafile=TLS_CERT, max_connecting=max_connecting)
            else:
                http = H1Client(timeout_s=30, max_connecting=max_connecting)
            svc = Service(Config.from_dict(cfgd), source=src, store=store, http=http, logger=Logger(stream=sink),
                          serve_metrics=False)
            t_init = time.perf_counter()
            await svc.init()  # connects to the broker and PG; preconnect opens the sink connections
            out["init_ms"] = round((time.perf_counter() - t_init) * 1e3, 2)
            mon = StallMonitor(period_s=stall_period_s, work=lambda: _settled(src.settler)).start()
            src.settler.trace_slow(SLOW_TRACE_NS)
            cg0 = cgroup_cpu_stat()
            task = asyncio.ensure_future(svc.run())
            # warm-up: connection pools fill (up to prefetch sink connections, the PG pool), code
            # paths get hot; then the latency histograms restart and the clock starts
            await _wait_acked(src.settler, warm, task)
            cold = dict(src.settler.handle_latency.summary())
            warm_slow = _slowest(src.settler.slow_deliveries()[0], _settled(src.settler))
            warm_mon = (list(mon.loop_stalls), list(mon.gc_pauses))
            src.settler.reset_latency()
            src.settler.trace_slow(SLOW_TRACE_NS)
            settled0 = _settled(src.settler)
            gc.collect()
            mon.reset()
            rss0 = _rss_mb()  # pools full, code paths warm: later growth would be a leak
            cg1 = cgroup_cpu_stat()
            fcpu0 = [proc_cpu_s(p.pid) for _, p in kinds]
            io0 = _io_counts(src)
            rq0 = thread_run_delay_ns()  # this (the event loop's) thread
            ru0 = resource.getrusage(resource.RUSAGE_SELF)
            if hooks:
                hooks[0]()
            t0 = time.perf_counter()
            if window_events > 0:
                rss_mid, merged = await _windows(src.settler, mon, settled0, n, window_events, task, t0, out)
            else:
                merged = None
                # half-way: the RSS there against the end is the leak check (the first half still
                # grows the sink pool towards its steady size: tens of connections with their buffers)
                await _wait_acked(src.settler, warm + (n - warm) // 2, task)
                rss_mid = _rss_mb()
                await _wait_acked(src.settler, n, task)
            elapsed = time.perf_counter() - t0
            if hooks:
                hooks[1]()
            ru1 = resource.getrusage(resource.RUSAGE_SELF)
            rq1 = thread_run_delay_ns()
            io1 = _io_counts(src)
            fcpu1 = [proc_cpu_s(p.pid) for _, p in kinds]
            cg2 = cgroup_cpu_stat()
            mon.stop()
            gc.collect()
            # before the slow-delivery list is made: up to 65,536 traced (recv, start, settle)
            # tuples are ~10 MB of Python objects whose pymalloc arenas stay mapped afterwards
            rss1 = _rss_mb()
            steady_slow = _slowest(src.settler.slow_deliveries()[0], _settled(src.settler) - settled0)
            measured = _settled(src.settler) - settled0
            await asyncio.sleep(0.05)  # let the last acks flush
            svc.request_stop()
            await task
            stats = svc.stats()
            if merged is not None:  # the windows reset the settler's histograms: their merge
                for kind, h in merged.items():
                    stats[f"{kind}_latency_ns"] = h.summary()
            pg_conns = store._pool.connections if store._pool else 0
            http_stats = http.stats()
            await svc.close()
            sink.close()
            cpu = (ru1.ru_utime + ru1.ru_stime) - (ru0.ru_utime + ru0.ru_stime)
            fakes_cpu: Dict[str, float] = {}
            fakes_util: Dict[str, list] = {}  # each fake process's CPU share of the window
            for (kind, _), a0, a1 in zip(kinds, fcpu0, fcpu1):
                if a0 is not None and a1 is not None:
                    fakes_cpu[kind] = fakes_cpu.get(kind, 0.0) + (a1 - a0)
                    fakes_util.setdefault(kind, []).append(round((a1 - a0) / elapsed, 3) if elapsed > 0 else None)
            diag = {"warm_slow": warm_slow, "steady_slow": steady_slow, "mon": mon, "warm_mon": warm_mon,
                    "nivcsw": ru1.ru_nivcsw - ru0.ru_nivcsw, "cgroup_warmup": cgroup_delta(cg0, cg1),
                    "cgroup_steady": cgroup_delta(cg1, cg2), "fakes_cpu_s": fakes_cpu, "fakes_util": fakes_util,
                    "minflt": ru1.ru_minflt - ru0.ru_minflt, "majflt": ru1.ru_majflt - ru0.ru_majflt, "rss0": rss0,
                    "io": {k: io1[k] - io0[k] for k in io0}, "rss_mid": rss_mid,
                    "run_delay_ms": (rq1 - rq0) / 1e6 if rq0 is not None and rq1 is not None else None}
            return elapsed, stats, cpu, ru1.ru_stime - ru0.ru_stime, pg_conns, http_stats, measured, cold, rss1 - rss0, diag

        elapsed, stats, cpu, sys_s, pg_conns, http_stats, m, cold, rss_growth, diag = asyncio.run(go())
        acked = stats["source"]["acked"]
        out.update({
            "acked": acked, "warmup_events": warm, "measured_events": m, "elapsed_s": elapsed,
            "ingest_rate_eps": m / elapsed if elapsed > 0 else None,
            "cpu_us_per_event": cpu / m * 1e6 if m else None,
            "sys_cpu_us_per_event": sys_s / m * 1e6 if m else None,
            "handle_latency_us": {k: v / 1e3 for k, v in stats["handle_latency_ns"].items() if k.startswith("p")},
            # receive -> ack (the handler's wait for the loop included) and receive -> handler start
            "ingest_latency_us": {k: v / 1e3 for k, v in stats["ingest_latency_ns"].items() if k.startswith("p")},
            "queue_latency_us": {k: v / 1e3 for k, v in stats["queue_latency_ns"].items() if k.startswith("p")},
            "warmup_handle_latency_us": {k: v / 1e3 for k, v in cold.items() if k.startswith("p")},
            "errors": sum(stats.get("handler_errors", {}).values()),
            "pg_connections": pg_conns, "http": http_stats, "rss_growth_mb": round(rss_growth, 2),
            # second half of the window only (see rss_mid): growth there would be per event
            "rss_growth_second_half_mb": round(rss_growth - (diag["rss_mid"] - diag["rss0"]), 2),
            "nivcsw": diag["nivcsw"], "cgroup_warmup": diag["cgroup_warmup"], "cgroup_steady": diag["cgroup_steady"],
            "minflt": diag["minflt"], "majflt": diag["majflt"],
            # each fake's CPU over the measured window, per consumed event (broker / pg / http(s)):
            # the share of the phase's CPU the consumer does not own
            "fakes_cpu_us_per_event": {k: round(v / m * 1e6, 3) for k, v in diag["fakes_cpu_s"].items()} if m else {},
            # ... and each fake process's busy share of the window: one near 1.0 was the bottleneck
            # (the consumer then waits on it, with smaller batches per loop turn)
            "fakes_util": diag["fakes_util"],
            # the consumer's socket calls per event over the window, by connection (VERDICT r4
            # item 4: which writes could share a wake-up): AMQP reads / writes (acks), sink and
            # Postgres sends / receives, NetPoller callbacks and the sockets each found ready
            "io_per_event": {k: round(v / m, 4) for k, v in diag["io"].items()} if m else {},
            # the consumer's loop thread's time runnable but waiting for a CPU over the window
            "run_delay_ms": diag["run_delay_ms"],
        })
    finally:
        if diag is not None:  # the broker prints its DONE line (paced: how late its sends were) and exits
            for p in bprocs:
                try:
                    p.wait(timeout=3)
                except Exception:  # noqa: BLE001 - reaped below either way
                    pass
        stalls: list = []
        counters = _reap(procs, stalls)
        out["server_side"] = counters
    if diag is not None:
        mon = diag["mon"]
        out["attribution_steady"] = _attribution(diag["steady_slow"], mon, stalls)
        warm_mon = StallMonitor()
        warm_mon.loop_stalls, warm_mon.gc_pauses = diag["warm_mon"]
        out["attribution_warmup"] = _attribution(diag["warm_slow"], warm_mon, stalls)
    return out


def _amqp(n: int) -> dict:
    """AMQP ingest (the reference's transport): a replay broker process streams n pre-encoded
    deliveries over TCP; this process runs the service (AmqpSource, prefetch 100, native
    delivery demux) and acks every message. Measures the consumer side end to end."""
    import subprocess

    from ..config import Config
    from ..service import Service
    from ..sinks import RecordingHttpClient
    from ..store import MemoryStore
    from ..transport.amqp import AmqpSource
    from ..utils.log import Logger

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    proc = subprocess.Popen([sys.executable, "-m", "beholder_amd.bench.replay_broker", "--events", str(n)],
                            stdout=subprocess.PIPE, text=True, env=env, cwd=root)
    try:
        line = proc.stdout.readline().split()
        if not line or line[0] != "READY":
            raise RuntimeError("replay broker failed to start")
        port = int(line[1])
        w = Workload(n_media=10000, seed=0)
        warm = min(5000, n // 10)

        async def go():
            sink = open(os.devnull, "w", buffering=1 << 16)
            src = AmqpSource(f"amqp://guest:guest@127.0.0.1:{port}/", prefetch=100)
            svc = Service(Config.from_dict(bench_config()), source=src, store=MemoryStore(w.media),
                          http=RecordingHttpClient(keep=8), logger=Logger(stream=sink), serve_metrics=False)
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            # warm-up (code paths get hot), then the latency histograms restart and the clock starts
            await _wait_acked(src.settler, warm, task)
            src.settler.reset_latency()
            settled0 = _settled(src.settler)
            ru0 = resource.getrusage(resource.RUSAGE_SELF)
            t0 = time.perf_counter()
            await _wait_acked(src.settler, n, task)
            elapsed = time.perf_counter() - t0
            ru1 = resource.getrusage(resource.RUSAGE_SELF)
            measured = _settled(src.settler) - settled0
            await asyncio.sleep(0.05)  # let the last acks flush
            svc.request_stop()
            await task
            stats = svc.stats()
            await svc.close()
            sink.close()
            return elapsed, stats, (ru1.ru_utime + ru1.ru_stime) - (ru0.ru_utime + ru0.ru_stime), measured

        elapsed, stats, cpu, measured = asyncio.run(go())
        tail = proc.stdout.readline().strip()
        proc.wait(30)
    finally:
        if proc.poll() is None:
            proc.kill()
    return {"events": n, "acked": stats["source"]["acked"], "warmup_events": warm, "measured_events": measured,
            "elapsed_s": elapsed, "ingest_rate_eps": measured / elapsed if elapsed > 0 else None,
            "handle_latency_us": {k: v / 1e3 for k, v in stats["handle_latency_ns"].items() if k.startswith("p")},
            # receive -> ack (the handler's wait for the loop included) and receive -> handler start
            "ingest_latency_us": {k: v / 1e3 for k, v in stats["ingest_latency_ns"].items() if k.startswith("p")},
            "queue_latency_us": {k: v / 1e3 for k, v in stats["queue_latency_ns"].items() if k.startswith("p")},
            "broker": tail, "prefetch": 100, "native_demux": True,
            "cpu_us_per_event": cpu / measured * 1e6 if measured else None,
            "ack_frames": stats["source"].get("ack_frames")}


def _free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _scrape(port: int, path: str = "/metrics", timeout: float = 2.0) -> Optional[str]:
    import urllib.request
    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=timeout) as r:
            return r.read().decode()
    except OSError:
        return None


def _metric_value(text: str, name: str, labels: str = "") -> Optional[float]:
    """Value of ``name{labels}`` in a Prometheus text exposition (first match)."""
    want = f"{name}{{{labels}}}" if labels else name
    for ln in text.split("\n"):
        if ln.startswith("#"):
            continue
        key, _, val = ln.rpartition(" ")
        if key == want:
            return float(val)
    return None


def _plumbing(w: Workload, *, timeout_s: float = 120.0) -> dict:
    """Config 1: 100 events on the stdin of the real CLI process (``python -m beholder_amd run
    --source stdin``, the analogue of ``node index.js``, package.json:5, index.js:160).

    The events go in, then ``/metrics`` is scraped over HTTP while the process still runs (stdin
    open) until all 100 deliveries show as acked; then stdin closes and the process must exit 0.
    Reports whether both reference counters (index.js:29-40) are in the scrape."""
    import yaml

    from .fakes import FakeHttpServer
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    port = _free_port()
    scrape = None
    with tempfile.TemporaryDirectory() as td, FakeHttpServer() as fake:
        cfgd = bench_config()
        cfgd["service"]["endpoints"] = {"trello": fake.url, "telegram": fake.url}
        cfgd["instance"]["emby"]["host"] = fake.url
        cfgd["service"]["http"] = {"timeout_s": 5.0}
        cfgd["service"]["transport"] = {"kind": "stdin"}
        cp = os.path.join(td, "events.yaml")
        with open(cp, "w") as f:
            yaml.safe_dump(cfgd, f)
        mp = os.path.join(td, "media.json")
        with open(mp, "w") as f:
            json.dump([m._asdict() for m in w.media], f)
        data = w.framed(100)
        env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
        t0 = time.perf_counter()
        p = subprocess.Popen([sys.executable, "-m", "beholder_amd", "run", "--config", cp, "--media-fixture", mp,
                              "--source", "stdin", "--metrics-port", str(port), "--stats"],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, cwd=root,
                             preexec_fn=_die_with_parent())
        try:
            p.stdin.write(data)
            p.stdin.flush()
            deadline = time.monotonic() + timeout_s
            while time.monotonic() < deadline and p.poll() is None:
                text = _scrape(port)
                if text is not None and (_metric_value(text, "beholder_deliveries", 'state="acked"') or 0) >= 100:
                    scrape = text
                    break
                time.sleep(0.05)
            # communicate() closes stdin (EOF: the service drains and exits) and collects the output
            out, err = p.communicate(timeout=max(5.0, deadline - time.monotonic()))
        except BaseException:
            p.kill()
            p.communicate()
            raise
        elapsed = time.perf_counter() - t0
    if p.returncode != 0:
        raise RuntimeError(f"plumbing run failed ({p.returncode}): {err.decode()[-2000:]}")
    stats = json.loads(err.decode().strip().splitlines()[-1])
    lines = [json.loads(x) for x in out.decode().split("\n") if x.startswith("{")]
    s = stats["source"]
    scrape = scrape or ""
    return {"config": "plumbing", "offered": 100, "rc": p.returncode, "acked": s["acked"], "abandoned": s["abandoned"],
            "errors": sum(stats.get("handler_errors", {}).values()), "process_wall_s": elapsed,
            "http_requests": len(fake.requests),
            "log_lines": len(lines), "warn_lines": sum(1 for x in lines if x["level"] == 40),
            "received": stats["received"],
            "metrics_scraped": bool(scrape),
            "scrape_acked": _metric_value(scrape, "beholder_deliveries", 'state="acked"'),
            # the reference's two counters (index.js:29-40): names, the "crreated" typo, no _total on comments
            "scrape_has_progress_counter": "\n# TYPE beholder_progress_updates_total counter" in scrape
                                           and "beholder_progress_updates_total{" in scrape,
            "scrape_has_trello_counter": "\n# TYPE beholder_trello_comments counter" in scrape
                                         and "\nbeholder_trello_comments " in scrape,
            "scrape_trello_comments": _metric_value(scrape, "beholder_trello_comments")}


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="beholder bench", description="BASELINE.json measurement configs")
    ap.add_argument("configs", nargs="*", default=["all"])
    ap.add_argument("--duration", type=float, default=None)
    ap.add_argument("--events", type=int, default=None)
    ap.add_argument("--out", default=None, help="write results JSON here")
    a = ap.parse_args(argv)
    names = CONFIGS if (not a.configs or a.configs == ["all"]) else a.configs
    results = {}
    for n in names:
        t0 = time.perf_counter()
        results[n] = run_config(n, duration_s=a.duration, events=a.events)
        results[n]["wall_s"] = time.perf_counter() - t0
        print(json.dumps(results[n], default=str), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(results, f, indent=2, default=str)
    return 0
