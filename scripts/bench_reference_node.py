#!/usr/bin/env python3
"""Same-machine A/B: the reference's own ``index.js`` on Node vs this service's ``bench.py``.

The reference publishes no numbers, so this measures one. It runs
``/root/reference/index.js`` unmodified on the image's Node (v12) with in-process stand-ins
for its dependencies (``scripts/reference_node/stubs``: pino, trello, request-promise-native,
triton-core/{config,dynamics,amqp,db,proto,prom}). The stand-ins do the same work as this
repo's bench fakes: protobuf decode, the JSON log line per log call, URL + query-string
construction per sink request, label-hashed counters, an in-memory media table. Each is
at most as expensive as the real library (the log sink is buffered, where pino@5 writes
synchronously; ``--pino-sync`` adds a run with that behaviour). The buffered Node number is
therefore an upper bound for the reference, and ``speedup`` is taken against it.

Both sides consume identical event streams: the same generator and seeds as bench.py, one
stream per process. They use the same step size and warm-up, and the same number of
competing-consumer processes. The Node processes start together (ready/go handshake).
Whole-job events/s = total events / wall time from "go" to the last result.

The reference is not in the repository (copying it is not allowed), so this runs where
``--index`` exists: in the build container, not on the GPU box.

    python scripts/bench_reference_node.py --procs 1 --steps 10 --warmup 2 --out profiles/x.json
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HERE = os.path.join(ROOT, "scripts", "reference_node")


def write_inputs(d: str, i: int, seed: int, a) -> dict:
    from beholder_amd.bench.generator import Workload, bench_config
    w = Workload(n_media=a.media, seed=seed)
    paths = {k: os.path.join(d, f"{k}{i}") for k in ("config", "media", "events")}
    with open(paths["config"], "w") as f:
        json.dump(bench_config(), f)
    with open(paths["media"], "w") as f:
        json.dump([{"id": m.id, "name": m.name, "creator": m.creator, "creatorId": m.creatorId,
                    "metadataId": m.metadataId, "status": m.status} for m in w.media], f)
    with open(paths["events"], "wb") as f:
        for _ in range(a.warmup + a.steps):  # bench.py generates one w.framed(E) per step, in order
            f.write(w.framed(a.events_per_step))
    return paths


def run_node(a, pino_sync: bool = False) -> dict:
    env = dict(os.environ, NODE_PATH=os.path.join(HERE, "stubs"))
    env.pop("NO_TRELLO", None)
    with tempfile.TemporaryDirectory() as d:
        procs = []
        for i in range(a.procs):
            p = write_inputs(d, i, a.seed + 104729 * i, a)
            cmd = [a.node, os.path.join(HERE, "harness.js"), "--index", a.index, "--config", p["config"],
                   "--media", p["media"], "--events", p["events"], "--events-per-step", str(a.events_per_step),
                   "--warmup", str(a.warmup), "--steps", str(a.steps), "--wait-go"] + (["--pino-sync"] if pino_sync else [])
            procs.append(subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=env, text=True))
        for p in procs:
            line = p.stdout.readline()
            if line.strip() != "ready":
                raise RuntimeError(f"node harness failed to start: {line!r}")
        t0 = time.perf_counter()
        for p in procs:
            p.stdin.write("go\n")
            p.stdin.close()
        results = [json.loads(p.stdout.readline()) for p in procs]
        t1 = time.perf_counter()
        for p in procs:
            p.wait(60)
    lat = sorted(r["p50_handle_latency_us"] for r in results)
    events = sum(r["events"] for r in results)
    return {"events_per_sec": events / (t1 - t0), "events": events, "procs": a.procs,
            "events_per_proc_per_sec": events / (t1 - t0) / a.procs,
            "p50_handle_latency_us_median_over_procs": lat[len(lat) // 2],
            "handler_errors": sum(r["handler_errors"] for r in results),
            "http_requests": sum(r["http_requests"] for r in results), "node": results[0]["node"],
            "per_proc": results}


def run_ours(a) -> dict:
    """bench.py on the same streams. One process: the headline (``value``, one consumer). N
    processes: the all-process phase (``all_procs_*``), whose consumer i uses seed
    ``--seed + 1 + 104729 * i``, hence ``--seed`` one lower than the Node side's."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(a.steps), "--warmup", str(a.warmup),
           "--events-per-step", str(a.events_per_step), "--media", str(a.media), "--no-extras"]
    if a.procs == 1:
        cmd += ["--procs-per-rank", "1", "--all-procs-steps", "0", "--seed", str(a.seed)]
    else:
        cmd += ["--procs-per-rank", str(a.procs), "--all-procs-steps", str(a.steps), "--seed", str(a.seed - 1)]
    out = json.loads(subprocess.run(cmd, check=True, capture_output=True, text=True).stdout.strip().splitlines()[-1])
    if a.procs > 1:
        out["value"] = out["all_procs_events_per_sec"]
        out["events_per_proc_per_sec"] = round(out["value"] / a.procs, 1)
    out["procs"] = a.procs
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--index", default="/root/reference/index.js")
    ap.add_argument("--node", default="node")
    ap.add_argument("--procs", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--events-per-step", type=int, default=65536)
    ap.add_argument("--media", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--skip-ours", action="store_true")
    ap.add_argument("--pino-sync", action="store_true",
                    help="also run the reference with one write(2) per log line (pino@5's default destination)")
    ap.add_argument("--out")
    a = ap.parse_args()
    if not os.path.exists(a.index):
        print(f"reference index.js not found at {a.index}", file=sys.stderr)
        return 2
    res = {"reference_node": run_node(a)}
    if a.pino_sync:
        res["reference_node_pino_sync"] = run_node(a, pino_sync=True)
    if not a.skip_ours:
        ours = run_ours(a)
        res["ours"] = {k: ours[k] for k in ("value", "events_per_proc_per_sec", "p50_handle_latency_us",
                                            "p99_handle_latency_us", "http_requests", "handler_errors", "procs")}
        res["speedup"] = round(ours["value"] / res["reference_node"]["events_per_sec"], 2)
    res["config"] = {"procs": a.procs, "steps": a.steps, "warmup": a.warmup, "events_per_step": a.events_per_step,
                     "media": a.media, "seed": a.seed, "cpu": _cpu_model()}
    text = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    print(text)
    return 0


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    raise SystemExit(main())
