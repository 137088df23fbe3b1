#!/usr/bin/env python3
"""Headline benchmark: metric-events/sec ingested + p50 handle latency (BASELINE.json ``metric``).

BASELINE.json's configs are all **single process**, so ``value`` is the ingest rate of ONE
consumer process per rank (for N ranks: N such consumers, whole-job events/s; weak scaling).
One *step* = ``--events-per-step`` synthetic telemetry events (90% progress / 10% status,
protobuf-encoded, framed) pushed through the **whole** service path of the consumer:

    producer thread -> OS pipe -> native reader thread (framing, ring)
      -> event loop: Delivery batches -> eager handler dispatch
      -> native protobuf decode -> handler logic (index.js:62-155)
      -> media store (in-memory, 10k rows) -> Prometheus counters
      -> Trello/Telegram/Emby request construction (URL + query encoding)
         into an in-process HTTP stub that does the production client's
         per-request work minus the socket: the request bytes from the H1
         client's own builder, a canned `200 {}` through an H1Parser, the H1
         client's HttpResponse (ops/csrc_bench/recorder.cpp, in the bench
         extension; the compiled handlers call it through its sink hook, as they
         call the H1 client's native path in production)
      -> pino JSON log line per reference log call (info level, to /dev/null)
      -> ack (latency recorded natively)

A step ends when every event of the step has been settled. ``W`` warm-up steps run untimed,
then exactly ``K`` steps are timed, bracketed by a gloo barrier and ``torch.cuda.synchronize()``
on both sides (the service queues no device work: the reference has none).
The elapsed time is the MAX over ranks.

The same run also measures, as extra keys of the one JSON line (rank 0, outside the timed
region):

* ``all_procs_*``: every CPU of the rank's share busy: ``--procs-per-rank`` consumer processes
  (competing consumers) on independent streams. This moves with the host's load.
* ``rate_1k_*``: BASELINE config 2, 1k events/s paced for 1 s: sustained ingest, p50/p99
  receive→ack latency.
* ``rate_10k_*``: BASELINE config 3, 10k events/s paced for 1 s: p50/p99 receive→ack latency.
  Every paced config also reports ``_due_to_ack`` (from the time the producer was to write the
  event: its lateness, the pipe and the reader thread's wake-up included) and ``_due_to_recv``.
* ``rate_100k_*``: BASELINE config 4, 100k events/s paced for 1 s into a 4096-event ring with
  ``drop_newest``: offered / accepted / dropped (``offered == accepted + dropped``), p99 latency.
* ``burst_*``: 200k events written unpaced (pipe speed) into the same ring: drop accounting
  under overload, beyond config 4.
* ``soak_*``: BASELINE config 5, 1M events unpaced: the service's RSS growth over the run
  (workload excluded) and GC pauses. ``bench_proc_maxrss_mb`` is the whole bench process's peak:
  pre-generated workloads and the torch import included.
* ``tcp_e2e_*`` / ``http_tcp_h1_*``: the production-shaped path, every dependency over TCP (an
  AMQP replay broker, a Postgres fake and HTTP fakes in their own processes).
* ``tls_e2e_*``: the same with HTTPS sinks, as Trello and Telegram are in production.
  ``tls_e2e_preconnect_*``: the same again with ``service.http.preconnect`` = 100 (sink
  connections and their handshakes made in init, ``_init_ms``; the default is 0, on demand).

Order of the phases: (1) everything that starts child processes (config 1's CLI process, the TCP
fakes, the all-process consumers); (2) the paced configs 2-4, in process, before HIP is touched;
(3) the headline between two calibration runs, whose ``torch.cuda.synchronize()`` is the first
HIP call of this process (a process that initialised the GPU must not start programs); (4) the
soak (config 5).

* ``plumbing_*``: BASELINE config 1, 100 events on the stdin of ``python -m beholder_amd run``
  with ``/metrics`` scraped before it exits.
* ``calib_*``: fixed-work calibrations before and after the headline (see CALIB_REF below).
* ``*_slow_*``: the slowest 0.1% of ``tcp_e2e`` / ``tls_e2e`` deliveries blamed on the process
  that stalled under them (bench/stallmon.py).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import asyncio
import contextlib
import ctypes
import gc
import json
import math
import multiprocessing as mp
import os
import resource
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from beholder_amd.utils.hostinfo import available_cpus, cpu_share, default_procs, gpus_on_node  # noqa: E402

BASELINE_METRIC = "metric_events_ingested_per_sec"
# the headline's sink stub (sinks/http.py RecordingHttpClient): "h1" builds every request's bytes
# with the H1 client's builder and parses a canned `200 {}` per request (production's per-request
# work minus the socket); "url" is round 4's URL-only stub, for the A/B of the two
STUB = os.environ.get("BEHOLDER_BENCH_STUB", "h1")


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1, help="number of ranks (one process group member per GPU slot)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--events-per-step", type=int, default=65536, help="events per step per consumer process")
    ap.add_argument("--procs-per-rank", type=int, default=0,
                    help="consumer processes per rank in the all-process phase (0 = min(16, CPUs per GPU slot - 1))")
    ap.add_argument("--all-procs-steps", type=int, default=10,
                    help="timed steps of the all-process phase (0 = skip it)")
    ap.add_argument("--no-extras", dest="extras", action="store_false",
                    help="skip the rate_10k / soak / overload / TCP measurements")
    ap.add_argument("--io-events", type=int, default=50000,
                    help="events of the preconnect and http_tcp measurements")
    ap.add_argument("--e2e-events", type=int, default=250000,
                    help="events of each tcp_e2e / tls_e2e measurement (the first 5,000 are the warm-up)")
    ap.add_argument("--e2e-repeats", type=int, default=3,
                    help="tcp_e2e / tls_e2e runs each; the line has the median run (by rate) and every run's figures")
    ap.add_argument("--e2e-paced-scale", type=float, default=1.0,
                    help="events of the paced tcp_e2e / tls_e2e runs (E2E_RATES) times this (0 = skip them)")
    ap.add_argument("--soak-events", type=int, default=1_000_000)
    ap.add_argument("--shared-queue-events", type=int, default=100_000,
                    help="events per worker of each shared-queue run (run --workers N on one queue; 0 = skip)")
    ap.add_argument("--media", type=int, default=10000)
    ap.add_argument("--log-level", default="info")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--full-out", default=os.environ.get("BENCH_FULL_OUT", os.path.join(ROOT, "gpurun_out", "bench_full.json")),
                    help="where the full record (every key of the run) is written; '' = nowhere")
    ap.add_argument("--ordering", default="none", choices=["none", "per_media"])
    ap.add_argument("--pin", action="store_true",
                    help="pin each all-process consumer to its own CPU of the rank's affinity mask")
    return ap.parse_args(argv)


class _Device:
    """``torch.cuda.synchronize()`` around the timed region, as the driver contract asks.

    The service queues no device work, so this only orders the (empty) stream. HIP is
    initialised lazily on the first :meth:`sync`, which ``main`` reaches only after every child
    process of the run has been started.
    """

    def __init__(self, local_rank: int):
        self.local_rank = local_rank
        self._torch = None
        self._ready = False

    def sync(self) -> None:
        if not self._ready:
            self._ready = True
            try:
                import torch
                if torch.cuda.device_count() > 0 and torch.cuda.is_available():
                    torch.cuda.set_device(self.local_rank % torch.cuda.device_count())
                    self._torch = torch
            except Exception:  # noqa: BLE001 — CPU-only environments: nothing to synchronize
                self._torch = None
        if self._torch is not None:
            self._torch.cuda.synchronize()

    @property
    def initialised(self) -> bool:
        return self._ready


@contextlib.contextmanager
def _stdout_to_stderr():
    """Points fd 1 at stderr for the block: native libraries' chatter (gloo's connection report)
    must not land on stdout, where rank 0 prints the one JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        try:
            ctypes.CDLL(None).fflush(None)  # C stdio / std::cout output written inside the block
        except (OSError, AttributeError):
            pass
        os.dup2(saved, 1)
        os.close(saved)


class _Dist:
    """gloo process group when launched under torch.distributed.run, no-op otherwise."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(self.world)))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            with _stdout_to_stderr():  # gloo prints "[Gloo] Rank r is connected to ..." on fd 1
                dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


async def run_consumer(a, seed: int, go, stop=None, *, steps: int = None, warmup: int = None) -> dict:
    """One consumer: build the service, warm up, ``go()``, time ``steps`` steps, ``stop()``."""
    from beholder_amd.bench.generator import Workload, bench_config
    from beholder_amd.config import Config
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    from beholder_amd.store import MemoryStore
    from beholder_amd.transport.ingest import FdSource
    from beholder_amd.utils.hostinfo import proc_run_delay_ns, thread_run_delay_ns
    from beholder_amd.utils.log import Logger

    steps = a.steps if steps is None else steps
    warmup = a.warmup if warmup is None else warmup
    E = a.events_per_step
    total_steps = warmup + steps
    w = Workload(n_media=a.media, seed=seed)
    step_bytes = [w.framed(E) for _ in range(total_steps)]

    rfd, wfd = os.pipe()
    cfg_d = bench_config()
    cfg_d["service"]["log"]["level"] = a.log_level
    cfg_d["service"]["ordering"] = a.ordering
    cfg = Config.from_dict(cfg_d)
    log_sink = open(os.devnull, "w", buffering=1 << 16)
    http = RecordingHttpClient(keep=16, stub=STUB)
    svc = Service(cfg, source=FdSource(fd=rfd, batch=512), store=MemoryStore(w.media), http=http,
                  logger=Logger(stream=log_sink, level=a.log_level), serve_metrics=False)
    await svc.init()
    run_task = asyncio.ensure_future(svc.run())
    settler = svc.source.settler

    pump_delay = [0, True]  # run-queue wait of the timed steps' pump threads (ns), all known

    def write_step(i: int, timed: bool) -> threading.Thread:
        def pump(data=step_bytes[i]):
            r0 = thread_run_delay_ns() if timed else None
            mv = memoryview(data)
            while mv:
                n = os.write(wfd, mv[:1 << 20])
                mv = mv[n:]
            if timed:
                r1 = thread_run_delay_ns()
                if r0 is None or r1 is None:
                    pump_delay[1] = False
                else:
                    pump_delay[0] += r1 - r0
        t = threading.Thread(target=pump, daemon=True)
        t.start()
        return t

    def settled() -> int:
        st = settler.stats()
        return st["acked"] + st["nacked"] + st["rejected"] + st["abandoned"]

    async def wait_settled(target: int):
        while settled() < target or svc._inflight:
            await asyncio.sleep(0.0002)

    t0 = 0.0
    ru0 = None
    rq0 = pq0 = rq1 = pq1 = rqg = None
    for i in range(total_steps):
        if i == warmup:
            settler.reset_latency()
            rqg = thread_run_delay_ns()
            go()
            t0 = time.perf_counter()
            ru0 = resource.getrusage(resource.RUSAGE_SELF)
            # run-queue waits over exactly the timed steps: this (the event loop's) thread, and every
            # thread of the process alive across them (the native reader thread, HIP's runtime
            # threads started by go()'s synchronize); the pump threads report their own
            rq0, pq0 = thread_run_delay_ns(), proc_run_delay_ns()
        th = write_step(i, i >= warmup)
        await wait_settled((i + 1) * E)
        th.join()
    rq1, pq1 = thread_run_delay_ns(), proc_run_delay_ns()
    if stop is not None:
        stop()
    elapsed = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    os.close(wfd)
    await run_task
    await svc.close()
    log_sink.close()
    st = svc.stats()
    return {
        "elapsed": elapsed,
        "events": E * steps,
        "handle_hist": settler.handle_latency.to_bytes(),
        "ingest_hist": settler.ingest_latency.to_bytes(),
        "http_calls": http.count,
        "errors": sum(st.get("handler_errors", {}).values()),
        "abandoned": st["source"]["abandoned"],
        # CPU of the timed steps (consumer + the thread feeding its pipe) and the times the kernel
        # took the CPU away: a low rate with unchanged CPU per event and many involuntary switches
        # is other load on the box, not the consumer
        "cpu_s": (ru1.ru_utime + ru1.ru_stime) - (ru0.ru_utime + ru0.ru_stime) if ru0 else 0.0,
        "nivcsw": ru1.ru_nivcsw - ru0.ru_nivcsw if ru0 else 0,
        # page faults in the timed steps: a box still compacting memory shows here, not in calib_*
        "minflt": ru1.ru_minflt - ru0.ru_minflt if ru0 else 0,
        "majflt": ru1.ru_majflt - ru0.ru_majflt if ru0 else 0,
        "timed_run_delay_ms": (rq1 - rq0) / 1e6 if rq0 is not None and rq1 is not None else None,
        # ... and inside go() itself (the first device synchronize: HIP's initialisation, its threads)
        "go_run_delay_ms": (rq0 - rqg) / 1e6 if rq0 is not None and rqg is not None else None,
        "timed_proc_run_delay_ms": (pq1 - pq0) / 1e6 if pq0 is not None and pq1 is not None else None,
        "timed_pump_run_delay_ms": pump_delay[0] / 1e6 if pump_delay[1] and steps else None,
    }


def run_solo(a, dist: _Dist, dev: _Device) -> dict:
    """The headline: one consumer in this process, K steps timed between barrier+sync pairs."""
    def go():
        dev.sync()
        dist.barrier()

    res = asyncio.run(run_consumer(a, a.seed + 7919 * dist.rank, go, dev.sync))
    res["procs"] = 1
    return res


def _consumer_entry(a, seed, steps, warmup, ready, go, results, cpu=None):
    """Spawned consumer process: warm up, report ready, wait for the go signal, time its steps."""
    if cpu is not None:
        try:
            os.sched_setaffinity(0, {cpu})
        except OSError:
            pass

    def start():
        ready.wait()  # warmed up
        go.wait()     # released by the coordinator, which starts its clock at the same moment

    try:
        res = asyncio.run(run_consumer(a, seed, start, steps=steps, warmup=warmup))
        results.put(res)
    except BaseException as e:  # report, never hang the coordinator
        for b in (ready, go):
            try:
                b.abort()
            except Exception:  # noqa: BLE001
                pass
        results.put({"error": f"{type(e).__name__}: {e}"})
        raise


def run_procs(a, dist: _Dist, procs: int, steps: int, warmup: int = 1) -> dict:
    """All-process phase: ``procs`` spawned consumers on independent streams, released together
    after a barrier across ranks. Runs before this process touches HIP (it starts programs)."""
    base_seed = a.seed + 7919 * dist.rank + 1
    ctx = mp.get_context("spawn")
    ready = ctx.Barrier(procs + 1)
    go = ctx.Barrier(procs + 1)
    results = ctx.Queue()
    cpus = sorted(os.sched_getaffinity(0)) if a.pin and hasattr(os, "sched_getaffinity") else []
    first = dist.local_rank * procs

    def cpu_for(i):
        return cpus[(first + i) % len(cpus)] if cpus else None
    children = [ctx.Process(target=_consumer_entry,
                            args=(a, base_seed + 104729 * i, steps, warmup, ready, go, results, cpu_for(i)),
                            daemon=True) for i in range(procs)]
    for c in children:
        c.start()
    ready.wait()            # every consumer has warmed up
    dist.barrier()          # every rank is ready
    go.wait()               # releases the consumers; the clock starts with them
    t0 = time.perf_counter()
    got = [results.get() for _ in range(procs)]
    t1 = time.perf_counter()
    for c in children:
        c.join(60)
    errs = [g["error"] for g in got if "error" in g]
    if errs:
        raise RuntimeError("consumer failed: " + "; ".join(errs))
    # each consumer also clocks its own steps from the go signal; the rank's elapsed time is never
    # shorter than the slowest consumer's (guards against any head start before t0)
    elapsed = max(t1 - t0, max(g["elapsed"] for g in got))
    return {"elapsed": elapsed, "coordinator_elapsed": t1 - t0, "events": sum(g["events"] for g in got),
            "errors": sum(g["errors"] for g in got), "procs": procs,
            "max_consumer_elapsed": max(g["elapsed"] for g in got)}


def _r(x, nd=3):
    return None if x is None else round(float(x), nd)


def _max_or_none(xs, nd=2):
    xs = list(xs)
    return None if not xs or any(x is None for x in xs) else round(max(xs), nd)


def _attr_keys(prefix: str, att: dict) -> dict:
    """Flat bench-line keys for one phase's slow-delivery attribution (bench/stallmon.py)."""
    if not att:
        return {}
    blamed = att.get("blamed", {})
    procs = att.get("processes", {})
    out = {f"{prefix}_slow_n": att.get("deliveries"),
           f"{prefix}_slow_blamed": blamed,
           f"{prefix}_slow_time_share": att.get("time_share"),
           f"{prefix}_slowest_us": att.get("slowest_us")}
    c = procs.get("consumer", {})
    out[f"{prefix}_consumer_loop_lag_max_us"] = c.get("loop_lag_max_us")
    out[f"{prefix}_consumer_loop_stalls"] = c.get("loop_stalls")
    out[f"{prefix}_consumer_gc_max_pause_us"] = c.get("gc_max_pause_us")
    # the consumer's longest loop stalls: [stall us, deliveries settled inside it] (bench/stallmon.py)
    out[f"{prefix}_consumer_stall_work"] = c.get("stall_work")
    fakes = {k: v for k, v in procs.items() if k != "consumer"}
    out[f"{prefix}_fakes_loop_lag_max_us"] = {k: v.get("loop_lag_max_us") for k, v in fakes.items()}
    out[f"{prefix}_fakes_gc_max_pause_us"] = max([v.get("gc_max_pause_us") or 0 for v in fakes.values()] or [0])
    return out


def _pool_keys(prefix: str, http: dict) -> dict:
    """Where a cold sink pool's time went (sinks/h1.py): the slowest connect (+ TLS handshake),
    and how long queued requests waited for a connection (p99 / max over the run; in steady state
    nothing queues, so these describe the warm-up)."""
    http = http or {}
    return {f"{prefix}_dial_max_us": http.get("dial_max_us"),
            f"{prefix}_queue_wait_p99_us": http.get("queue_wait_p99_us"),
            f"{prefix}_queue_wait_max_us": http.get("queue_wait_max_us")}


def _cg(prefix: str, d: dict) -> dict:
    return {f"{prefix}_nr_throttled": d.get("nr_throttled"), f"{prefix}_throttled_usec": d.get("throttled_usec")}


def _busiest(e: dict):
    """The busiest fake process's CPU share of one e2e run's window (None without the data)."""
    us = [u for v in (e.get("fakes_util") or {}).values() for u in v if u is not None]
    return max(us) if us else None


def _events_per_poll(e: dict):
    """Events per NetPoller callback over one e2e run (None without the socket-call counts)."""
    p = (e.get("io_per_event") or {}).get("poll_runs")
    return _r(1 / p, 1) if p else None


def _e2e_keys(prefix: str, run, n: int, repeats: int = 1, **kw) -> dict:
    """One production-shaped phase (harness._tcp_e2e), run ``repeats`` times: the keys are those
    of the run with the median rate (``*_runs``: every run's rate, CPU per event and p999). Each
    run: rate, CPU per event (user+sys and sys alone), latency, and what else could have moved
    them: the box's core speed right before it, page faults and involuntary switches of the
    measured window, each fake's CPU per event, the host's busy share, throttling, and the
    slow-delivery attribution."""
    from beholder_amd.utils.hostinfo import host_busy_pct, host_cpu_times
    runs = []
    for _ in range(max(1, repeats)):
        h0 = host_cpu_times()
        e = run(n, **kw)
        runs.append((e, host_busy_pct(h0, host_cpu_times())))
    order = sorted(range(len(runs)), key=lambda i: runs[i][0].get("ingest_rate_eps") or 0.0)
    e, busy = runs[order[len(order) // 2]]
    hl = e.get("handle_latency_us", {})
    wl = e.get("warmup_handle_latency_us", {})
    out = {f"{prefix}_events_per_sec": _r(e.get("ingest_rate_eps"), 1),
           f"{prefix}_measured_events": e.get("measured_events"),
           f"{prefix}_cpu_us_per_event": _r(e.get("cpu_us_per_event")),
           f"{prefix}_sys_cpu_us_per_event": _r(e.get("sys_cpu_us_per_event")),
           f"{prefix}_p50_handle_latency_us": _r(hl.get("p50")),
           f"{prefix}_p99_handle_latency_us": _r(hl.get("p99")),
           f"{prefix}_p999_handle_latency_us": _r(hl.get("p999")),
           f"{prefix}_warmup_p99_handle_latency_us": _r(wl.get("p99")),
           f"{prefix}_warmup_p999_handle_latency_us": _r(wl.get("p999")),
           f"{prefix}_errors": e.get("errors"), f"{prefix}_nivcsw": e.get("nivcsw"),
           f"{prefix}_minflt": e.get("minflt"), f"{prefix}_majflt": e.get("majflt"),
           f"{prefix}_calib_ns": e.get("calib_ns"),
           f"{prefix}_fakes_cpu_us_per_event": e.get("fakes_cpu_us_per_event"),
           f"{prefix}_fakes_util": e.get("fakes_util"),
           f"{prefix}_io_per_event": e.get("io_per_event"),
           f"{prefix}_rss_growth_mb": e.get("rss_growth_mb"),
           f"{prefix}_rss_growth_second_half_mb": e.get("rss_growth_second_half_mb"),
           f"{prefix}_run_delay_ms": _r(e.get("run_delay_ms"), 2),
           f"{prefix}_host_cpu_busy_pct": busy,
           **_cg(prefix, e.get("cgroup_steady") or {}),
           **_attr_keys(prefix, e.get("attribution_steady")),
           **_attr_keys(f"{prefix}_warmup", e.get("attribution_warmup")),
           **_pool_keys(prefix, e.get("http"))}
    if kw.get("tls"):
        http = e.get("http") or {}
        out.update({f"{prefix}_handshakes": http.get("tls_handshakes"), f"{prefix}_resumed": http.get("tls_resumed"),
                    f"{prefix}_init_ms": e.get("init_ms")})
    if len(runs) > 1:
        out[f"{prefix}_runs"] = {
            "events_per_sec": [_r(r.get("ingest_rate_eps"), 1) for r, _ in runs],
            "cpu_us_per_event": [_r(r.get("cpu_us_per_event")) for r, _ in runs],
            "p999_handle_latency_us": [_r((r.get("handle_latency_us") or {}).get("p999")) for r, _ in runs],
            # what moves CPU per event between runs of one line: system time, how many events
            # each NetPoller callback found ready (bigger batches, fewer calls), the core speed
            "sys_cpu_us_per_event": [_r(r.get("sys_cpu_us_per_event")) for r, _ in runs],
            "events_per_poll_run": [_events_per_poll(r) for r, _ in runs],
            "calib_ns": [r.get("calib_ns") for r, _ in runs],
            "run_delay_ms": [_r(r.get("run_delay_ms"), 2) for r, _ in runs],
            "busiest_fake_util": [_busiest(r) for r, _ in runs]}
    return out


# The production path at BASELINE's rates (configs 2-4: 1k, 10k, 100k events/s): tcp_e2e / tls_e2e
# with the replay broker pacing its sends, so each event's receive->ack latency is its own Postgres
# and HTTP round trips, not queueing behind a saturated prefetch window. (name, events/s, events:
# a tenth of them is the warm-up, connection pools filling at that rate)
E2E_RATES = (("1k", 1000, 3000), ("10k", 10000, 20000), ("100k", 100000, 100000))


def _paced_e2e_keys(prefix: str, name: str, e: dict) -> dict:
    """Keys of one paced production-path run: handler start->ack and receive->ack p50/p99/p999,
    the achieved rate, CPU per event, and how late the broker's sends were against their due time
    (p99; late sends mean the consumer held the prefetch window full)."""
    hl = e.get("handle_latency_us") or {}
    il = e.get("ingest_latency_us") or {}
    ss = e.get("server_side") or {}
    p = f"{prefix}_rate_{name}"
    return {f"{p}_events_per_sec": _r(e.get("ingest_rate_eps"), 1),
            f"{p}_p50_handle_latency_us": _r(hl.get("p50"), 1), f"{p}_p99_handle_latency_us": _r(hl.get("p99"), 1),
            f"{p}_p999_handle_latency_us": _r(hl.get("p999"), 1),
            f"{p}_p50_ingest_latency_us": _r(il.get("p50"), 1), f"{p}_p99_ingest_latency_us": _r(il.get("p99"), 1),
            f"{p}_cpu_us_per_event": _r(e.get("cpu_us_per_event"), 2),
            f"{p}_broker_late_p99_us": ss.get("late_p99_us"),
            f"{p}_measured_events": e.get("measured_events"), f"{p}_errors": e.get("errors"),
            f"{p}_run_delay_ms": _r(e.get("run_delay_ms"), 2)}


# the bench's stall monitor ticks on the consumer's loop; at 1 ms (the saturated runs' tick, for
# stall attribution) it billed the paced runs ~4 us per event at 1k/s, one wake-up per event
# (profiles/box_r6_tick_ab/). The paced keys use no stall data: a coarse tick keeps it off the CPU.
PACED_STALL_TICK_S = 0.05


def paced_e2e_keys(a, prefix: str, **kw) -> dict:
    from beholder_amd.bench import harness
    out = {}
    if a.e2e_paced_scale <= 0:
        return out
    for name, rate, n in E2E_RATES:
        n = max(200, int(n * a.e2e_paced_scale))
        out.update(_paced_e2e_keys(prefix, name, harness._tcp_e2e(n, rate=rate, stall_period_s=PACED_STALL_TICK_S,
                                                                 **kw)))
    out[f"{prefix}_paced_stall_tick_ms"] = PACED_STALL_TICK_S * 1e3
    return out


def shared_queue_workers(cpus: int, cap: int = 8) -> list:
    """N of the shared-queue sweep: 1, 2, 4, 8 while N workers + the broker + this process + one
    spare CPU fit in the share."""
    return [n for n in (1, 2, 4, 8) if n <= cap and n + 3 <= max(4, cpus)]


def shared_queue_keys(a) -> dict:
    """The reference's own scaling mode (competing consumers on one queue, index.js:43,62,127):
    ``run --workers N`` against one shared-queue broker, the same load per worker for each N
    (bench/shared_queue.py). Keyed by N: events/s, the broker's CPU per event, and whether every
    published event was acked exactly once."""
    from beholder_amd.bench.shared_queue import run_shared
    ns = shared_queue_workers(available_cpus())
    if a.shared_queue_events <= 0 or not ns:
        return {}
    eps, bcpu, once, acked, published, per_conn = {}, {}, {}, {}, {}, {}
    for n in ns:
        r = run_shared(n, a.shared_queue_events * n, seed=a.seed)
        key = str(n)
        eps[key] = _r(r["events_per_sec"], 1)
        bcpu[key] = _r(r["broker_cpu_us_per_event"])
        once[key] = bool(r["exactly_once"] and r.get("supervisor_rc") == 0)
        acked[key], published[key] = r["acked"], r["published"]
        per_conn[key] = r["per_connection_delivered"]
    return {"shared_queue_events_per_sec": eps, "shared_queue_exactly_once": all(once.values()),
            "shared_queue_broker_cpu_us_per_event": bcpu, "shared_queue_acked": acked,
            "shared_queue_published": published, "shared_queue_exactly_once_by_n": once,
            "shared_queue_per_worker_delivered": per_conn}


def io_extras(a) -> dict:
    """BASELINE config 1 (the real CLI on stdin) and the production-shaped TCP path. Both start
    child processes, so they run before this process touches HIP."""
    from beholder_amd.bench import harness
    from beholder_amd.bench.generator import Workload
    out = {}
    p = harness._plumbing(Workload(n_media=10000, seed=a.seed))
    out.update({"plumbing_rc": p["rc"], "plumbing_acked": p["acked"], "plumbing_errors": p["errors"],
                "plumbing_sink_requests": p["http_requests"], "plumbing_metrics_scraped": p["metrics_scraped"],
                "plumbing_scrape_acked": p["scrape_acked"],
                "plumbing_has_progress_counter": p["scrape_has_progress_counter"],
                "plumbing_has_trello_counter": p["scrape_has_trello_counter"],
                "plumbing_process_wall_s": _r(p["process_wall_s"])})
    # unmeasured: one short pass of the whole TCP path first, so the first measured e2e phase is
    # not also this process's first (first-touch page faults, the pools' and fakes' first
    # connections, lazily imported modules), as the paced configs get one
    harness._tcp_e2e(min(100000, a.e2e_events))
    out.update(_e2e_keys("tcp_e2e", harness._tcp_e2e, a.e2e_events, a.e2e_repeats))
    # and of the TLS path: its first run in a process paid ~1 µs/event more system time (OpenSSL's
    # connection buffers first touched; profiles/box_r5_runs/, box_r5_pgn/)
    out.update(paced_e2e_keys(a, "tcp_e2e"))
    harness._tcp_e2e(min(100000, a.e2e_events), http_servers=4, tls=True)
    out.update(_e2e_keys("tls_e2e", harness._tcp_e2e, a.e2e_events, a.e2e_repeats, http_servers=4, tls=True))
    out.update(paced_e2e_keys(a, "tls_e2e", http_servers=4, tls=True))
    # the same with service.http.preconnect = prefetch: the first wave of TLS handshakes happens
    # in init (`_init_ms`), not inside the first deliveries' handle latency
    pre = harness._tcp_e2e(a.io_events, http_servers=4, tls=True, preconnect=100)
    out.update({"tls_e2e_preconnect_events_per_sec": _r(pre.get("ingest_rate_eps"), 1),
                "tls_e2e_preconnect_p999_handle_latency_us": _r(pre.get("handle_latency_us", {}).get("p999")),
                "tls_e2e_preconnect_warmup_p999_handle_latency_us":
                    _r(pre.get("warmup_handle_latency_us", {}).get("p999")),
                "tls_e2e_preconnect_init_ms": pre.get("init_ms"),
                "tls_e2e_preconnect_handshakes": (pre.get("http") or {}).get("tls_handshakes"),
                "tls_e2e_preconnect_errors": pre.get("errors")})
    out.update(shared_queue_keys(a))
    h = harness._http_tcp(Workload(n_media=10000, seed=a.seed), a.io_events, clients=("h1",))["h1"]
    hl = h["handle_latency_us"]
    out.update({"http_tcp_h1_events_per_sec": _r(h["ingest_rate_eps"], 1),
                "http_tcp_h1_p99_handle_latency_us": _r(hl.get("p99")),
                "http_tcp_h1_p999_handle_latency_us": _r(hl.get("p999"))})
    return out


def _paced(prefix: str, r: dict) -> dict:
    """Keys of one paced config: receive->ack p50/p99 and its two hops (reader push -> handler
    start, handler start -> ack), and the same from each event's due time (``due_to_ack``:
    also the producer's lateness, the pipe and the reader thread's wake-up; ``due_to_recv``:
    that part alone). The due-time keys are null when events were dropped."""
    il, ql, hl = r["ingest_latency_us"], r.get("queue_latency_us", {}), r["handle_latency_us"]
    da, dr = r.get("due_to_ack_us") or {}, r.get("due_to_recv_us") or {}
    return {f"{prefix}_acked": r["acked"],
            f"{prefix}_p50_due_to_ack_us": _r(da.get("p50")),
            f"{prefix}_p99_due_to_ack_us": _r(da.get("p99")),
            f"{prefix}_p999_due_to_ack_us": _r(da.get("p999")),
            f"{prefix}_p99_due_to_recv_us": _r(dr.get("p99")),
            f"{prefix}_p50_ingest_latency_us": _r(il.get("p50")),
            f"{prefix}_p99_ingest_latency_us": _r(il.get("p99")),
            f"{prefix}_p999_ingest_latency_us": _r(il.get("p999")),
            f"{prefix}_p99_queue_latency_us": _r(ql.get("p99")),
            f"{prefix}_p99_handle_latency_us": _r(hl.get("p99")),
            f"{prefix}_idle_wakeups": r.get("idle_wakeups"),
            f"{prefix}_loop_thread_nivcsw": r.get("loop_thread_nivcsw"),
            f"{prefix}_loop_run_delay_us": _r(r.get("loop_run_delay_us"), 1),
            f"{prefix}_loop_stalls": (r.get("loop") or {}).get("loop_stalls"),
            f"{prefix}_loop_lag_max_us": (r.get("loop") or {}).get("loop_lag_max_us"),
            f"{prefix}_gc_max_pause_us": (r.get("loop") or {}).get("gc_max_pause_us"),
            f"{prefix}_cpu_us_per_event": _r(r.get("cpu_us_per_event"))}


def paced_extras(a) -> dict:
    """BASELINE configs 2-4 (paced producers) and the unpaced overload, in this process. The
    producer is native and GIL-free (ops.bench_native.paced_write); these run before the headline initialises
    HIP, so nothing but the consumer and its reader thread competes for this process."""
    from beholder_amd.bench import harness
    from beholder_amd.bench.generator import Workload
    from beholder_amd.utils.hostinfo import cgroup_cpu_stat, cgroup_delta, host_busy_pct, host_cpu_times
    w = Workload(n_media=10000, seed=a.seed)
    out = {}
    # unmeasured: 0.3 s at 10k/s through a fresh service first, so the paced configs do not also
    # measure this process's first paced run (first-touch page faults of the ring and the heap,
    # the exited all-process consumers' memory being reclaimed)
    asyncio.run(harness._run_inproc(w.events(3000), 10000, media=w.media))
    cg0 = cgroup_cpu_stat()
    h0 = host_cpu_times()
    r = asyncio.run(harness._run_inproc(w.events(1000), 1000, media=w.media))  # config 2: 1 s at 1k/s
    out.update({"rate_1k_events_per_sec": _r(r["ingest_rate_eps"], 1), **_paced("rate_1k", r)})
    r = asyncio.run(harness._run_inproc(w.events(10000), 10000, media=w.media))  # config 3: 1 s at 10k/s
    out.update(_paced("rate_10k", r))
    # config 4: 1 s paced at 100k/s into the small ring, drop_newest (backpressure + drop accounting)
    r = asyncio.run(harness._run_inproc(w.events(100_000), 100_000, policy="drop_newest", capacity_events=4096,
                                        media=w.media))
    out.update({"rate_100k_offered": r["offered"], "rate_100k_accepted": r["accepted"],
                "rate_100k_dropped": r["dropped"],
                "rate_100k_offered_per_sec": _r(r["offered_rate_eps"], 1), **_paced("rate_100k", r)})
    out.update(_cg("paced", cgroup_delta(cg0, cgroup_cpu_stat())))
    out["paced_host_cpu_busy_pct"] = host_busy_pct(h0, host_cpu_times())
    r = asyncio.run(harness._run_inproc(w.events(200_000), 0, policy="drop_newest", capacity_events=4096,
                                        media=w.media))
    out.update({"burst_offered": r["offered"], "burst_accepted": r["accepted"],
                "burst_dropped": r["dropped"]})
    return out


def soak_extras(a) -> dict:
    """BASELINE config 5 in this process (no child processes: HIP may be initialised now)."""
    import resource

    from beholder_amd.bench import harness
    from beholder_amd.bench.generator import Workload
    w = Workload(n_media=10000, seed=a.seed)
    out = {}
    evs = w.events(a.soak_events)
    probe: list = []
    g = harness.GcPauses()
    r = asyncio.run(harness._run_inproc(evs, 0, media=w.media, rss_probe=probe, gc_probe=g))
    del evs
    gs = g.summary()
    curve = r.get("rss_curve_mb") or []
    out.update({"soak_events": r["acked"], "soak_events_per_sec": _r(r["ingest_rate_eps"], 1),
                "soak_cpu_us_per_event": _r(r.get("cpu_us_per_event")),
                # the service's RSS growth over the run (from after init, with the 1M-event workload
                # already in memory): at the end, and at the highest 0.5 s sample
                "soak_rss_growth_mb": _r(probe[1] - probe[0], 2),
                "soak_rss_peak_growth_mb": _r(max(curve + [probe[1]]) - probe[0], 2),
                "bench_proc_maxrss_mb": _r(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024, 1),
                "soak_gc_pauses": gs.get("count", 0), "soak_gc_max_pause_us": _r(gs.get("max_us")),
                "soak_gc_p99_pause_us": _r(gs.get("p99_us"))})
    return out


# Fixed-work calibrations around the headline, each the minimum of CALIB_REPS runs (ns):
#   calib_ns      bench_native.calib: an L1-resident integer loop (core clock, time-sharing of the core);
#   calib_mem_ns  bench_native.calib_mem: a dependent random walk over 8 MiB (L3 / memory latency, which
#                 other tenants' traffic moves);
#   calib_py_ns   a fixed pure-Python loop (the interpreter: dict, str and int churn, as the
#                 consumer's Python glue does).
# CALIB_REF holds the medians of the same figures over the builder's reference box runs
# (profiles/box_r4_calib1/, 8 runs on one box). value_calibrated = value * calib_ns / CALIB_REF:
# the headline a box with the reference box's core speed would have given. README "Reading the
# headline" explains what the calibrations do and do not account for.
CALIB_ITERS = 4_000_000
CALIB_MEM_BYTES, CALIB_MEM_STEPS = 8 << 20, 500_000
CALIB_REPS = 5
CALIB_REF = {"calib_ns": 6_439_000, "calib_mem_ns": 5_627_000, "calib_py_ns": 2_766_000}


def _calib_py_once() -> int:
    t0 = time.perf_counter_ns()
    d: dict = {}
    for i in range(20_000):
        k = f"m{i % 997}"
        d[k] = d.get(k, 0) + len(str(i * 7))
    return time.perf_counter_ns() - t0


def _thp_mode():
    """The host's transparent-huge-page mode (the bracketed word of the sysfs setting)."""
    try:
        with open("/sys/kernel/mm/transparent_hugepage/enabled") as f:
            t = f.read()
        return t[t.index("[") + 1:t.index("]")]
    except (OSError, ValueError):
        return None


def calibrate() -> dict:
    from beholder_amd.ops.bench_native import calib, calib_mem
    return {"calib_ns": min(calib(CALIB_ITERS)[0] for _ in range(CALIB_REPS)),
            "calib_mem_ns": min(calib_mem(CALIB_MEM_BYTES, CALIB_MEM_STEPS)[0] for _ in range(CALIB_REPS)),
            "calib_py_ns": min(_calib_py_once() for _ in range(CALIB_REPS))}


def _phase(name: str, fn, a) -> dict:
    """One extra phase. A failure there (a fake that would not start on some host) must not cost
    the driver its line: the headline still runs and prints, with ``<phase>_error`` saying what
    went wrong (the contract tests check the extra keys themselves)."""
    try:
        return fn(a)
    except Exception as e:  # noqa: BLE001 - reported on the line, and on stderr in full
        import traceback
        traceback.print_exc(file=sys.stderr)
        return {f"{name}_error": f"{type(e).__name__}: {e}"[:300]}


def _finite(x):
    """The line must be strict JSON for the driver: a NaN or infinity anywhere (an extra key
    computed from an empty phase) becomes null instead of an unparseable token."""
    if isinstance(x, float):
        return x if math.isfinite(x) else None
    if isinstance(x, dict):
        return {k: _finite(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_finite(v) for v in x]
    return x


DATA = ("synthetic telemetry (90% progress / 10% status), 10k-media in-memory store, "
        "Trello/Telegram/Emby stubbed in-process (" + ("h1 stub: each request's bytes built by the H1 client's "
                                                      "builder, a canned 200 parsed by H1Parser into its HttpResponse"
                                                      if STUB == "h1" else "url stub: URL + query built and logged")
        + "; no socket), info logs to /dev/null")

NOTES = ("CPU event-consumer workload (the reference has no device compute; see docs/DESIGN.md). "
         "value = one consumer process per rank; all_procs_* = every CPU of the share busy; "
         "rate_1k/rate_10k/rate_100k/soak = BASELINE configs 2-5 (rate_100k paced into a 4096-event "
         "drop_newest ring; burst = the same ring fed unpaced); tcp_e2e/http_tcp = every dependency "
         "over TCP, tls_e2e = same with HTTPS sinks; tcp_e2e/tls_e2e latencies are receive->ack at "
         "saturation with prefetch 100 in flight (queueing included), warmup_* = the first 5,000 "
         "deliveries (connection pools filling from zero; http.preconnect 0); *_slow_blamed = the "
         "slowest 0.1% of deliveries blamed on the process (consumer / pg / http(s) / broker fake) "
         "whose event-loop or GC stall covered most of their time, 'none' = no stall >= 1 ms "
         "(bench/stallmon.py); rate_*_p99_queue = reader push -> handler start, "
         "rate_*_p99_handle = handler start -> ack; *_dial_max / *_queue_wait_* = the slowest sink "
         "connect (+TLS handshake) and the wait of requests queued for a connection (the warm-up); "
         "*_fakes_cpu_us_per_event = each fake's CPU over the measured window per event; "
         "*_e2e_calib_ns = the calib loop right before that phase; "
         "calib_ns = fixed-work C loop (bench_native.calib) "
         "around the headline, value_calibrated = value * calib_ns / calib_ref_ns; "
         "plumbing_* = BASELINE config 1 through `python -m beholder_amd run --source stdin`, "
         "/metrics scraped before exit")

# The driver keeps the tail of stdout (its `tail` field: the last ~2,000 characters; its
# `stdout_tail`: the last ~8,000), so the one JSON line is built for that:
# the contract keys first, then diagnostics while the line stays within LINE_BUDGET characters,
# then the decision keys, with the headline's own figures last of all. Every key of the run goes
# to the full record (``--full-out``). tests/test_bench_contract.py pins the layout.
LINE_BUDGET = 6000
TAIL_BUDGET = 2000
HEAD_KEYS = ("metric", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data", "config")
# decision keys, in line order: the last one printed is `value`
TAIL_KEYS = (
    "soak_gc_max_pause_us", "soak_rss_growth_mb", "soak_events_per_sec",
    "burst_dropped", "rate_100k_dropped",
    "rate_1k_p99_ingest_latency_us", "rate_10k_p50_ingest_latency_us", "rate_10k_p99_ingest_latency_us",
    "rate_100k_p99_ingest_latency_us",
    "all_procs_events_per_sec",
    "shared_queue_events_per_sec", "shared_queue_exactly_once",
    "http_tcp_h1_events_per_sec",
    "tls_e2e_preconnect_warmup_p999_handle_latency_us",
    "tls_e2e_warmup_p999_handle_latency_us", "tls_e2e_p999_handle_latency_us", "tls_e2e_cpu_us_per_event",
    "tls_e2e_events_per_sec",
    "tls_e2e_rate_10k_p50_handle_latency_us", "tls_e2e_rate_10k_p99_handle_latency_us",
    "tcp_e2e_rate_1k_p50_handle_latency_us", "tcp_e2e_rate_1k_p99_handle_latency_us",
    "tcp_e2e_rate_100k_p50_handle_latency_us", "tcp_e2e_rate_100k_p99_handle_latency_us",
    "tcp_e2e_rate_10k_p50_ingest_latency_us", "tcp_e2e_rate_10k_p99_ingest_latency_us",
    "tcp_e2e_rate_10k_p50_handle_latency_us", "tcp_e2e_rate_10k_p99_handle_latency_us",
    "tcp_e2e_warmup_p999_handle_latency_us", "tcp_e2e_p999_handle_latency_us", "tcp_e2e_p99_handle_latency_us",
    "tcp_e2e_sys_cpu_us_per_event", "tcp_e2e_cpu_us_per_event", "tcp_e2e_events_per_sec",
    "calib_ns", "value_calibrated", "handler_errors", "headline_timed_run_delay_ms",
    "cpu_us_per_event", "p99_handle_latency_us", "p50_handle_latency_us", "value",
)
# diagnostics that go on the line first, while it has room (the rest follow in run order)
DIAG_FIRST = (
    "tcp_e2e_calib_ns", "tcp_e2e_minflt", "tcp_e2e_majflt", "tcp_e2e_nivcsw", "tcp_e2e_fakes_cpu_us_per_event",
    "tcp_e2e_host_cpu_busy_pct", "tcp_e2e_nr_throttled", "tcp_e2e_measured_events", "tcp_e2e_slow_blamed",
    "tcp_e2e_runs", "tls_e2e_runs",
    "tls_e2e_calib_ns", "tls_e2e_sys_cpu_us_per_event", "tls_e2e_minflt", "tls_e2e_nivcsw",
    "tls_e2e_fakes_cpu_us_per_event", "tls_e2e_host_cpu_busy_pct", "tls_e2e_slow_blamed", "tls_e2e_consumer_stall_work",
    "tcp_e2e_consumer_stall_work",
    "headline_minflt", "headline_run_delay_ms", "headline_go_run_delay_ms", "headline_timed_pump_run_delay_ms",
    "headline_timed_proc_run_delay_ms", "involuntary_ctx_switches", "headline_host_cpu_busy_pct",
    "tcp_e2e_rate_1k_events_per_sec", "tcp_e2e_rate_10k_events_per_sec", "tcp_e2e_rate_100k_events_per_sec",
    "tcp_e2e_rate_10k_cpu_us_per_event", "tcp_e2e_rate_10k_broker_late_p99_us",
    "tcp_e2e_rate_100k_broker_late_p99_us", "tls_e2e_rate_10k_events_per_sec",
    "calib_mem_ns", "calib_py_ns",
    "shared_queue_broker_cpu_us_per_event", "shared_queue_acked", "shared_queue_published",
    "plumbing_rc", "plumbing_acked", "plumbing_sink_requests", "rate_1k_acked", "rate_10k_acked",
    "rate_100k_offered", "rate_100k_accepted", "burst_offered", "burst_accepted",
    "tcp_e2e_errors", "tls_e2e_errors", "soak_events",
)


def _write_full(path: str, full: dict):
    """Every key of the run as one JSON document (the line carries a subset). Returns the path
    written, or None when it could not be written (the line is still printed)."""
    if not path:
        return None
    try:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(full, f, indent=1, allow_nan=False)
        os.replace(tmp, path)
        return path
    except OSError as e:
        print(f"bench.py: could not write the full record to {path}: {e}", file=sys.stderr)
        return None


def _enc(k, v) -> int:
    return len(json.dumps({k: v}, allow_nan=False))  # '"k": v, ' as it sits inside the line


def compact_line(full: dict, full_path=None) -> dict:
    """The printed line: HEAD_KEYS, a pointer to the full record, diagnostics while they fit in
    LINE_BUDGET, then TAIL_KEYS (which fit in TAIL_BUDGET: the driver's `tail`)."""
    head = {k: full[k] for k in HEAD_KEYS if k in full}
    head["full_record"] = {"path": full_path, "keys": len(full)}
    tail = {k: full[k] for k in TAIL_KEYS if k in full}
    used = len(json.dumps(head)) + len(json.dumps(tail))
    diag: dict = {}
    order = [k for k in DIAG_FIRST if k in full] + [k for k in full if k not in DIAG_FIRST]
    for k in order:
        if k in head or k in tail or k in diag or k == "notes":
            continue
        c = _enc(k, full[k])
        if used + c > LINE_BUDGET:
            continue  # too big for what is left: a smaller later key may still fit
        diag[k] = full[k]
        used += c
    out = {**head, **diag, **tail}
    while diag and len(json.dumps(out, allow_nan=False)) > LINE_BUDGET:  # never reached; a guard
        diag.popitem()
        out = {**head, **diag, **tail}
    return out


def main(argv=None) -> int:
    a = parse(argv)
    dist = _Dist()
    n = dist.world if dist.world > 1 else a.gpus
    if dist.world == 1 and a.gpus > 1:
        print(f"bench.py: --gpus {a.gpus} requires torch.distributed.run; running 1 rank", file=sys.stderr)
        n = 1
    procs = a.procs_per_rank or default_procs(dist.local_world)
    dev = _Device(dist.local_rank)
    extras: dict = {}

    from beholder_amd.utils.hostinfo import (cgroup_cpu_stat, cgroup_delta, host_busy_pct, host_cpu_times,
                                             thread_run_delay_ns)

    # 1. phases that start child processes (before any HIP call in this process)
    if a.extras and dist.rank == 0:
        extras.update(_phase("io_extras", io_extras, a))
    dist.barrier()
    allp = None
    if a.all_procs_steps > 0 and procs > 1:
        allp = run_procs(a, dist, procs, a.all_procs_steps)
    allp_elapsed = dist.max(allp["elapsed"] if allp else 0.0)
    allp_events = sum(dist.gather(allp["events"] if allp else 0))

    # 2. paced BASELINE configs 2-4 (in process, before HIP is initialised)
    if a.extras and dist.rank == 0:
        extras.update(_phase("paced_extras", paced_extras, a))
    dist.barrier()

    # 3. the headline: one consumer per rank, K timed steps, between two calibration runs
    calib0 = calibrate()
    cg0 = cgroup_cpu_stat()
    h0 = host_cpu_times()
    gc.collect()
    rq0 = thread_run_delay_ns()  # the thread that runs the consumer's event loop
    res = run_solo(a, dist, dev)
    rq1 = thread_run_delay_ns()
    dist.barrier()
    cg1 = cgroup_cpu_stat()
    h1 = host_cpu_times()
    calib1 = calibrate()
    elapsed = dist.max(res["elapsed"])
    parts = dist.gather({k: res[k] for k in ("handle_hist", "ingest_hist", "http_calls", "errors", "abandoned",
                                             "events", "cpu_s", "nivcsw", "minflt", "majflt", "timed_run_delay_ms",
                                             "timed_proc_run_delay_ms", "timed_pump_run_delay_ms",
                                             "go_run_delay_ms")})
    calibs = dist.gather((calib0, calib1))
    # the loop thread's time runnable without a CPU over the headline (warm-up steps included); the
    # process total would also hold the reader thread's many short wake-up waits
    run_delays = dist.gather((rq1 - rq0) / 1e6 if rq0 is not None and rq1 is not None else None)

    # 4. BASELINE config 5 (no child processes: HIP may be initialised now)
    if a.extras and dist.rank == 0:
        extras.update(_phase("soak_extras", soak_extras, a))
    dist.barrier()

    if dist.rank == 0:
        from beholder_amd.ops import Histogram
        hh = Histogram()
        for p in parts:
            hh.merge_bytes(p["handle_hist"])
        total_events = sum(p["events"] for p in parts)
        value = total_events / elapsed
        cal = {}
        for k in CALIB_REF:  # the slowest rank's worse side of the headline
            cal[k] = max(max(c0[k], c1[k]) for c0, c1 in calibs)
            cal[k + "_before"] = calib0[k]
            cal[k + "_after"] = calib1[k]
        ref = CALIB_REF["calib_ns"]
        cal.update({"calib_ref": CALIB_REF,
                    # what a box with the reference box's core speed (the C loop) would give
                    "value_calibrated": round(value * cal["calib_ns"] / ref, 1) if ref else None,
                    "headline_host_cpu_busy_pct": host_busy_pct(h0, h1),
                    **_cg("headline", cgroup_delta(cg0, cg1))})
        full = {
            "metric": BASELINE_METRIC,
            "value": round(value, 1),
            "unit": "events/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "protobuf-events (no tensor compute)",
            "data": DATA,
            "config": {
                "model": "beholder telemetry consumer (status+progress handlers, index.js:62-155)",
                "global_batch": a.events_per_step * n,
                "seq_len": None,
                "parallelism": f"dp{n} x 1 consumer proc/rank (BASELINE: single process per consumer)",
            },
            "events_per_proc_per_sec": round(value / n, 1),
            "p50_handle_latency_us": round(hh.percentile(50) / 1e3, 3),
            "p99_handle_latency_us": round(hh.percentile(99) / 1e3, 3),
            "cpu_us_per_event": round(sum(p["cpu_s"] for p in parts) / total_events * 1e6, 3),
            "involuntary_ctx_switches": sum(p["nivcsw"] for p in parts),
            "headline_minflt": sum(p["minflt"] for p in parts),
            "headline_run_delay_ms": (round(max(run_delays), 2) if all(x is not None for x in run_delays)
                                      else None),
            # the same over exactly the K timed steps (after go(), at stop()): the loop thread, every
            # thread alive across them, and the pump threads feeding the pipe (the worst rank)
            "headline_timed_run_delay_ms": _max_or_none(p["timed_run_delay_ms"] for p in parts),
            "headline_timed_proc_run_delay_ms": _max_or_none(p["timed_proc_run_delay_ms"] for p in parts),
            "headline_timed_pump_run_delay_ms": _max_or_none(p["timed_pump_run_delay_ms"] for p in parts),
            "headline_go_run_delay_ms": _max_or_none(p["go_run_delay_ms"] for p in parts),
            "headline_majflt": sum(p["majflt"] for p in parts),
            "thp": _thp_mode(),
            **cal,
            "http_requests": sum(p["http_calls"] for p in parts),
            "handler_errors": sum(p["errors"] for p in parts),
            "all_procs_per_rank": procs if allp is not None else 0,
            "all_procs_events_per_sec": round(allp_events / allp_elapsed, 1) if allp_elapsed else None,
            "cpus_available": available_cpus(),
            "cpu_share": cpu_share(),
            "gpus_on_node": gpus_on_node(),
            **extras,
            "notes": NOTES,
        }
        full = _finite(full)
        full_path = _write_full(a.full_out, full)
        out = compact_line(full, full_path)
        print(json.dumps(out, allow_nan=False), flush=True)
    dist.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
