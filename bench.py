#!/usr/bin/env python3
"""Headline benchmark: metric-events/sec ingested + p50 handle latency (BASELINE.json ``metric``).

One *step* = ``--events-per-step`` synthetic telemetry events (90% progress /
10% status, protobuf-encoded, framed) pushed through the **whole** service
path of each consumer process:

    producer thread -> OS pipe -> native reader thread (framing, ring)
      -> event loop: Delivery batches -> eager handler dispatch
      -> native protobuf decode -> handler logic (index.js:62-155)
      -> media store (in-memory, 10k rows) -> Prometheus counters
      -> Trello/Telegram/Emby request construction (URL + query encoding)
         into an in-process HTTP recorder (no network)
      -> pino JSON log line per reference log call (info level, to /dev/null)
      -> ack (latency recorded natively)

A step ends when every event of the step has been settled. ``W`` warm-up
steps run untimed, then exactly ``K`` steps are timed.

Scale-out is the reference's: competing consumers, one process each
(SURVEY.md §2.3). Each rank runs ``--procs-per-rank`` consumer processes
(default: the CPU share of one GPU slot minus one, at most 16; the same for every N) on
independent streams.
Timing: every consumer finishes its warm-up and reports ready; the rank's
coordinator synchronizes the device, passes a gloo barrier across ranks, then
releases its consumers through a second barrier and starts the clock; it stops the clock when all of its
consumers report their K steps done, then passes another gloo barrier. The
elapsed time is the MAX over ranks and ``value`` is whole-job events/s.
Per-consumer work is fixed as N grows: weak scaling. The service has no
device work (the reference has none), so nothing runs on the GPU. The
timed region is bracketed by the barriers and by torch.cuda.synchronize()
(no kernel is ever queued). HIP is initialised in a rank process only after
its consumer processes have been spawned.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import asyncio
import gc
import json
import multiprocessing as mp
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

BASELINE_METRIC = "metric_events_ingested_per_sec"


def available_cpus() -> int:
    """CPUs this process may use: affinity mask, capped by a cgroup v2/v1 CPU quota."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return max(1, n)


def cpu_share() -> dict:
    """What the CPU budget is made of: affinity CPUs, the cgroup quota (CPUs, None = no quota)
    and the distinct physical cores behind the affinity CPUs. On the MI355X pool the share is a
    16-CPU quota over all 256 hardware threads, so consumers run next to other tenants' work and
    the all-process number moves with host load (profiles/box_r1_share/)."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = list(range(os.cpu_count() or 1))
    cores = set()
    for c in aff:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            with open(base + "physical_package_id") as f1, open(base + "core_id") as f2:
                cores.add((f1.read().strip(), f2.read().strip()))
        except OSError:
            cores.add(("?", str(c)))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"affinity_cpus": len(aff), "quota_cpus": quota, "physical_cores": len(cores)}


def gpus_on_node() -> int:
    """GPUs visible on this node, counted without initialising HIP (0 if torch is unavailable)."""
    try:
        import torch
        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001 — CPU-only environments
        return 0


def default_procs(local_world: int) -> int:
    """Consumer processes per rank: the CPU share of one GPU slot minus one, at most 16.

    The share is the node's CPUs divided by the number of GPU slots on the node (at least the
    local world size). It does not depend on how many ranks run, so per-rank work stays fixed
    as N grows (weak scaling): on an 8-GPU node with 16 CPUs per GPU, N=1 and N=8 both run 15
    consumers per rank.
    """
    slots = max(1, local_world, gpus_on_node())
    return max(1, min(16, available_cpus() // slots - 1))


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1, help="number of ranks (one process group member per GPU slot)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--events-per-step", type=int, default=65536, help="events per step per consumer process")
    ap.add_argument("--procs-per-rank", type=int, default=0,
                    help="consumer processes per rank (0 = min(16, CPUs per GPU slot - 1))")
    ap.add_argument("--media", type=int, default=10000)
    ap.add_argument("--log-level", default="info")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--ordering", default="none", choices=["none", "per_media"])
    ap.add_argument("--pin", action="store_true",
                    help="pin each consumer process to its own CPU of the rank's affinity mask")
    return ap.parse_args(argv)


class _Device:
    """``torch.cuda.synchronize()`` around the timed region, as the driver contract asks.

    The service queues no device work, so this only orders the (empty) stream. HIP is
    initialised lazily on the first :meth:`sync`. Callers make that happen only after every
    consumer process has been spawned, because a process that initialised the GPU must not start
    programs (spawn = fork + exec).
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


async def run_consumer(a, seed: int, go, stop=None) -> dict:
    """One consumer process: build the service, warm up, ``go()``, time K steps, ``stop()``."""
    from beholder_amd.bench.generator import Workload, bench_config
    from beholder_amd.config import Config
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    from beholder_amd.store import MemoryStore
    from beholder_amd.transport.ingest import FdSource
    from beholder_amd.utils.log import Logger

    E = a.events_per_step
    total_steps = a.warmup + a.steps
    w = Workload(n_media=a.media, seed=seed)
    step_bytes = [w.framed(E) for _ in range(total_steps)]

    rfd, wfd = os.pipe()
    cfg_d = bench_config()
    cfg_d["service"]["log"]["level"] = a.log_level
    cfg_d["service"]["ordering"] = a.ordering
    cfg = Config.from_dict(cfg_d)
    log_sink = open(os.devnull, "w", buffering=1 << 16)
    http = RecordingHttpClient(keep=16)
    svc = Service(cfg, source=FdSource(fd=rfd, batch=512), store=MemoryStore(w.media), http=http,
                  logger=Logger(stream=log_sink, level=a.log_level), serve_metrics=False)
    await svc.init()
    run_task = asyncio.ensure_future(svc.run())
    settler = svc.source.settler

    def write_step(i: int) -> threading.Thread:
        def pump(data=step_bytes[i]):
            mv = memoryview(data)
            while mv:
                n = os.write(wfd, mv[:1 << 20])
                mv = mv[n:]
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
    for i in range(total_steps):
        if i == a.warmup:
            settler.reset_latency()
            go()
            t0 = time.perf_counter()
        th = write_step(i)
        await wait_settled((i + 1) * E)
        th.join()
    if stop is not None:
        stop()
    elapsed = time.perf_counter() - t0
    os.close(wfd)
    await run_task
    await svc.close()
    log_sink.close()
    st = svc.stats()
    return {
        "elapsed": elapsed,
        "events": E * a.steps,
        "handle_hist": settler.handle_latency.to_bytes(),
        "ingest_hist": settler.ingest_latency.to_bytes(),
        "http_calls": http.count,
        "errors": sum(st.get("handler_errors", {}).values()),
        "abandoned": st["source"]["abandoned"],
    }


def _consumer_entry(a, seed, ready, go, results, cpu=None):
    """Spawned consumer process: warm up, report ready, wait for the go signal, time K steps."""
    if cpu is not None:
        try:
            os.sched_setaffinity(0, {cpu})
        except OSError:
            pass

    def start():
        ready.wait()  # warmed up
        go.wait()     # released by the coordinator, which starts its clock at the same moment

    try:
        res = asyncio.run(run_consumer(a, seed, start))
        results.put(res)
    except BaseException as e:  # report, never hang the coordinator
        for b in (ready, go):
            try:
                b.abort()
            except Exception:  # noqa: BLE001
                pass
        results.put({"error": f"{type(e).__name__}: {e}"})
        raise


def run_rank(a, dist: _Dist, procs: int) -> dict:
    """Coordinator for one rank's consumer processes; returns the rank's merged result."""
    base_seed = a.seed + 7919 * dist.rank
    dev = _Device(dist.local_rank)
    if procs == 1:  # the consumer runs in this process, which starts no other program
        def go():
            dev.sync()
            dist.barrier()
        res = asyncio.run(run_consumer(a, base_seed, go, dev.sync))
        res["procs"] = 1
        return res
    ctx = mp.get_context("spawn")
    ready = ctx.Barrier(procs + 1)
    go = ctx.Barrier(procs + 1)
    results = ctx.Queue()
    cpus = sorted(os.sched_getaffinity(0)) if a.pin and hasattr(os, "sched_getaffinity") else []
    first = dist.local_rank * procs

    def cpu_for(i):
        return cpus[(first + i) % len(cpus)] if cpus else None
    children = [ctx.Process(target=_consumer_entry, args=(a, base_seed + 104729 * i, ready, go, results, cpu_for(i)),
                            daemon=True) for i in range(procs)]
    for c in children:
        c.start()
    ready.wait()            # every consumer has warmed up (all spawned: HIP may be initialised now)
    dev.sync()              # nothing is timed yet: the consumers wait at `go`
    dist.barrier()          # every rank is ready (after its device init, so ranks start together)
    go.wait()               # releases the consumers; the clock starts with them
    t0 = time.perf_counter()
    got = [results.get() for _ in range(procs)]
    dev.sync()
    t1 = time.perf_counter()
    for c in children:
        c.join(60)
    errs = [g["error"] for g in got if "error" in g]
    if errs:
        raise RuntimeError("consumer failed: " + "; ".join(errs))
    from beholder_amd.ops import Histogram
    hh, ih = Histogram(), Histogram()
    for g in got:
        hh.merge_bytes(g["handle_hist"])
        ih.merge_bytes(g["ingest_hist"])
    # each consumer also clocks its own K steps from the go signal; the rank's elapsed time is never
    # shorter than the slowest consumer's (guards against any head start before t0)
    elapsed = max(t1 - t0, max(g["elapsed"] for g in got))
    return {"elapsed": elapsed, "coordinator_elapsed": t1 - t0, "events": sum(g["events"] for g in got), "handle_hist": hh.to_bytes(),
            "ingest_hist": ih.to_bytes(), "http_calls": sum(g["http_calls"] for g in got),
            "errors": sum(g["errors"] for g in got), "abandoned": sum(g["abandoned"] for g in got),
            "procs": procs, "max_consumer_elapsed": max(g["elapsed"] for g in got)}


def main(argv=None) -> int:
    a = parse(argv)
    dist = _Dist()
    n = dist.world if dist.world > 1 else a.gpus
    if dist.world == 1 and a.gpus > 1:
        print(f"bench.py: --gpus {a.gpus} requires torch.distributed.run; running 1 rank", file=sys.stderr)
        n = 1
    procs = a.procs_per_rank or default_procs(dist.local_world)
    gc.collect()
    res = run_rank(a, dist, procs)
    dist.barrier()
    elapsed = dist.max(res["elapsed"])
    parts = dist.gather({k: res[k] for k in ("handle_hist", "ingest_hist", "http_calls", "errors", "abandoned",
                                             "events", "procs")})
    if dist.rank == 0:
        from beholder_amd.ops import Histogram
        hh, ih = Histogram(), Histogram()
        for p in parts:
            hh.merge_bytes(p["handle_hist"])
            ih.merge_bytes(p["ingest_hist"])
        total_events = sum(p["events"] for p in parts)
        total_procs = sum(p["procs"] for p in parts)
        value = total_events / elapsed
        out = {
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
            "data": "synthetic telemetry (90% progress / 10% status), 10k-media in-memory store, "
                    "Trello/Telegram/Emby stubbed in-process, info logs to /dev/null",
            "config": {
                "model": "beholder telemetry consumer (status+progress handlers, index.js:62-155)",
                "global_batch": a.events_per_step * total_procs,
                "seq_len": None,
                "parallelism": f"dp{n} x {procs} consumer procs/rank (competing consumers)",
            },
            "procs_per_rank": procs,
            "cpus_available": available_cpus(),
            "cpu_share": cpu_share(),
            "gpus_on_node": gpus_on_node(),
            "events_per_proc_per_sec": round(value / total_procs, 1),
            "p50_handle_latency_us": round(hh.percentile(50) / 1e3, 3),
            "p99_handle_latency_us": round(hh.percentile(99) / 1e3, 3),
            "p50_ingest_latency_us": round(ih.percentile(50) / 1e3, 3),
            "http_requests": sum(p["http_calls"] for p in parts),
            "handler_errors": sum(p["errors"] for p in parts),
            "notes": "CPU event-consumer workload (the reference has no device compute; see docs/DESIGN.md); "
                     "each consumer process runs the full service path on its own synthetic stream",
        }
        print(json.dumps(out), flush=True)
    dist.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
