"""Cold-start probe: where the first seconds of the HTTP sink path go.

1. ``burst``: 100 concurrent requests on a fresh H1Client against the bench's fake endpoints
   (3 processes): wall time, this process's CPU, per-connect durations.
2. ``http_tcp``: the ``http_tcp`` bench config with every H1Client._connect timed: when the
   connects start and how long each takes, next to the warm-up handle latency.

Prints one JSON object."""
import asyncio
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from beholder_amd.bench import harness  # noqa: E402
from beholder_amd.bench.generator import Workload  # noqa: E402
from beholder_amd.sinks import h1  # noqa: E402

rec = []
_orig = h1.H1Client._connect


async def _timed_connect(self, o, deadline):
    t = time.perf_counter()
    try:
        return await _orig(self, o, deadline)
    finally:
        rec.append((t, time.perf_counter() - t))


h1.H1Client._connect = _timed_connect


def summary(xs):
    xs = sorted(xs)
    return {"n": len(xs), "p50_ms": round(xs[len(xs) // 2] * 1e3, 2), "max_ms": round(xs[-1] * 1e3, 2)} if xs else {}


async def burst(port):
    c = h1.H1Client(timeout_s=30)
    r0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    await asyncio.gather(*[c.request("GET", f"http://127.0.0.1:{port}/x") for _ in range(100)])
    wall = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_SELF)
    await c.close()
    return {"wall_ms": round(wall * 1e3, 2),
            "cpu_ms": round((r1.ru_utime + r1.ru_stime - r0.ru_utime - r0.ru_stime) * 1e3, 2)}


def main():
    out = {}
    port, procs = harness._spawn("beholder_amd.bench.http_sink_server", 3)
    try:
        rec.clear()
        out["burst"] = asyncio.run(burst(port))
        out["burst"]["connect"] = summary([d for _, d in rec])
    finally:
        harness._reap(procs)
    rec.clear()
    r = harness._http_tcp(Workload(n_media=10000, seed=0), 50000, clients=("h1",))["h1"]
    t0 = min(t for t, _ in rec) if rec else 0
    out["http_tcp"] = {"connect": summary([d for _, d in rec]),
                       "connect_start_spread_ms": round((max(t for t, _ in rec) - t0) * 1e3, 2) if rec else None,
                       "warmup_handle_latency_us": r["warmup_handle_latency_us"],
                       "handle_latency_us": r["handle_latency_us"], "ingest_rate_eps": r["ingest_rate_eps"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
