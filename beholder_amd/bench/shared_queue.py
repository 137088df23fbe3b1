"""Competing consumers on one shared queue: the reference's only scaling mode (N replicas of the
service on the same RabbitMQ queues, each with prefetch 100; index.js:43,62,127, SURVEY.md §2.3
"horizontal scaling"), measured the way this service scales it: ``run --workers N``
(parallel/workers.py supervisor, one worker process per CPU).

One measurement (:func:`run_shared`):

* a broker process holds ``events`` pre-encoded telemetry messages (the bench workload) and
  starts delivering once all N connections have subscribed: the native ``SharedBroker``
  (ops/csrc_bench/shared_broker.cpp, the default) or the asyncio
  :class:`~beholder_amd.bench.replay_broker.SharedQueueBroker` (``broker="python"``, whose own
  CPU capped the curve at about 2.2M events/s);
* ``python -m beholder_amd.bench.shared_worker run --workers N --source amqp ...`` is the
  service's ``run`` command with its supervisor; each worker has the 10k-media table in memory
  (``--media-fixture``) and the headline's in-process sink stub (no Trello/Telegram/Emby);
* the broker clocks the run from its first delivery to the ack that settles the last event,
  counts every ack per event (``acked`` = events acked at least once, ``dup_acks``, ``lost``)
  and reports its own CPU over that span; then the supervisor gets SIGTERM and must drain and
  exit 0.

``events_per_sec`` is events / broker span. ``broker_cpu_us_per_event`` (the broker loop's CPU
over the span) next to the rate says when the broker, not the workers, is the limit.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import tempfile
import threading
import time
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _parse_kv(line: str) -> Dict[str, object]:
    out: Dict[str, object] = {}
    for kv in line.split()[1:]:
        k, _, v = kv.partition("=")
        try:
            out[k] = int(v)
        except ValueError:
            try:
                out[k] = float(v)
            except ValueError:
                out[k] = v
    return out


def run_shared(workers: int, events: int, *, media: int = 10000, seed: int = 0, timeout_s: float = 120.0,
               log_level: str = "info", kill_one_after: int = 0, broker: str = "native") -> dict:
    """One shared-queue run with ``workers`` competing consumers; see the module docstring.

    ``kill_one_after``: once the broker reports that many events acked, one worker process gets
    SIGKILL (a crash in the middle of the stream): the supervisor restarts it, the broker requeues
    what the dead connection had un-acked (``redelivered``), and every event must still be acked
    exactly once at the broker (tests/test_workers.py)."""
    import yaml

    from .generator import Workload, bench_config
    from .harness import _die_with_parent, _spawn

    if broker not in ("native", "python"):
        raise ValueError("broker must be 'native' or 'python'")
    port, bprocs = _spawn("beholder_amd.bench.replay_broker", 1,
                          ("--events", str(events), "--media", str(media), "--seed", str(seed), "--shared",
                           "--consumers", str(workers), "--progress-every", str(kill_one_after), "--hold",
                           *(("--python",) if broker == "python" else ())))
    broker_proc = bprocs[0]
    lines: List[str] = []
    got_done = threading.Event()
    progress = threading.Event()

    def read_broker():
        for ln in broker_proc.stdout:
            lines.append(ln.strip())
            if ln.startswith("PROGRESS "):
                progress.set()
            if ln.startswith("FINAL "):
                got_done.set()
        got_done.set()
    threading.Thread(target=read_broker, daemon=True).start()
    sup = None
    out: dict = {"workers": workers, "events": events, "broker": broker}
    try:
        with tempfile.TemporaryDirectory(prefix="beholder-shared-") as td:
            w = Workload(n_media=media, seed=seed)
            cfgd = bench_config()
            cfgd["service"]["log"]["level"] = log_level
            cfgd["service"]["metrics"] = {"enabled": False}
            cp = os.path.join(td, "events.yaml")
            with open(cp, "w") as f:
                yaml.safe_dump(cfgd, f)
            mp = os.path.join(td, "media.json")
            with open(mp, "w") as f:
                json.dump([m._asdict() for m in w.media], f)
            del w
            env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
            sup = subprocess.Popen([sys.executable, "-m", "beholder_amd.bench.shared_worker", "run", "--config", cp,
                                    "--source", "amqp", "--url", f"amqp://guest:guest@127.0.0.1:{port}/",
                                    "--media-fixture", mp, "--workers", str(workers), "--metrics-port", "-1"],
                                   env=env, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                   preexec_fn=_die_with_parent())
            err: List[bytes] = []
            threading.Thread(target=lambda: err.append(sup.stderr.read()), daemon=True).start()
            if kill_one_after:
                def kill_one():
                    import psutil
                    if not progress.wait(timeout_s):
                        return
                    kids = psutil.Process(sup.pid).children()
                    if kids:
                        out["killed_worker_pid"] = kids[0].pid
                        kids[0].kill()
                threading.Thread(target=kill_one, daemon=True).start()
            if not got_done.wait(timeout_s):
                raise RuntimeError(f"shared queue run with {workers} workers did not finish in {timeout_s:.0f} s")
            sup.send_signal(signal.SIGTERM)
            try:
                rc = sup.wait(60)
            except subprocess.TimeoutExpired:
                sup.kill()
                rc = sup.wait()
            out["supervisor_rc"] = rc
            if rc != 0:
                time.sleep(0.1)
                out["supervisor_stderr"] = b"".join(err).decode(errors="replace")[-2000:]
    finally:
        if sup is not None and sup.poll() is None:
            sup.kill()
        if broker_proc.poll() is None:
            broker_proc.terminate()
        try:
            broker_proc.wait(10)
        except subprocess.TimeoutExpired:
            broker_proc.kill()
    done = next((ln for ln in lines if ln.startswith("FINAL ")), None) or \
        next((ln for ln in lines if ln.startswith("DONE ")), None)
    if done is None:
        raise RuntimeError(f"shared queue broker reported no result: {lines[-5:]}")
    d = _parse_kv(done)
    span = float(d.get("broker_s") or 0.0)
    acked = int(d.get("acked", 0))
    per_conn = [int(x) for x in str(d.get("per_conn", "")).split(",") if x]
    out.update({
        "published": d.get("published"), "acked": acked, "dup_acks": d.get("dup_acks"),
        "unknown_acks": d.get("unknown_acks"), "lost": d.get("lost"), "redelivered": d.get("redelivered"),
        "connections": d.get("connections"), "per_connection_delivered": per_conn,
        "broker_s": span, "events_per_sec": acked / span if span > 0 else None,
        "broker_cpu_us_per_event": float(d.get("cpu_s", 0.0)) / acked * 1e6 if acked else None,
        "exactly_once": acked == d.get("published") and d.get("dup_acks") == 0 and d.get("lost") == 0
                        and d.get("unknown_acks") == 0,
    })
    return out


def sweep(ns, events_per_worker: int, *, media: int = 10000, seed: int = 0) -> Dict[int, dict]:
    """:func:`run_shared` for each N in ``ns`` (the same per-worker load: weak scaling)."""
    return {n: run_shared(n, events_per_worker * n, media=media, seed=seed) for n in ns}


def main(argv: Optional[List[str]] = None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description="competing consumers on one shared queue")
    ap.add_argument("--workers", default="1,2,4")
    ap.add_argument("--events-per-worker", type=int, default=100_000)
    a = ap.parse_args(argv)
    res = sweep([int(x) for x in a.workers.split(",")], a.events_per_worker)
    for n, r in res.items():
        print(json.dumps(r), flush=True)
    return 0 if all(r["exactly_once"] and r["supervisor_rc"] == 0 for r in res.values()) else 1


if __name__ == "__main__":
    raise SystemExit(main())
