"""Command line: ``python -m beholder_amd <command>`` (reference entry: ``node index.js``, package.json:5).

Commands
--------
run      start the service (``--source amqp|stdin|file``); the reference's only mode.
config   validate and print the effective config (secrets masked).
gen      write synthetic framed telemetry to stdout/a file (+ optional media fixture).
decode   turn a framed stream into NDJSON (debugging).
seed     load a media fixture into a sqlite/postgres store.
bench    run the BASELINE.json measurement configs (see ``beholder_amd.bench.harness``).
publish  publish a framed stream to an AMQP broker.

Exit codes: 0 ok, 1 runtime failure, 2 usage/config error (startup failures are
fatal — the documented fix of quirk Q10).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import sys
from typing import List, Optional

from .config import Config, ConfigError


def _load_fixture(path: str):
    from .store import Media
    with open(path, "r", encoding="utf-8") as f:
        rows = json.load(f)
    return [Media(**r) for r in rows]


WORKER_MODULE_ENV = "BEHOLDER_WORKER_MODULE"


def worker_command() -> List[str]:
    """How ``run --workers N`` starts each worker: ``python -m beholder_amd`` with the run
    arguments. A wrapper entry module that must be in force in every worker (the bench's
    ``beholder_amd.bench.shared_worker``) opts in by naming itself in ``BEHOLDER_WORKER_MODULE``;
    the supervisor never guesses it from ``__main__`` (a launcher or test runner hosting ``run``
    would otherwise be restarted in its place)."""
    name = os.environ.get(WORKER_MODULE_ENV, "").strip() or "beholder_amd"
    return [sys.executable, "-m", name]


def cmd_run(a: argparse.Namespace) -> int:
    if a.workers and a.workers > 1:
        if a.source in ("stdin", "file"):
            print("beholder: --workers needs a shared broker transport (amqp)", file=sys.stderr)
            return 2
        from .parallel.workers import Supervisor, strip_workers_arg
        argv = strip_workers_arg(sys.argv[1:] if a.argv is None else a.argv)
        if a.metrics_port is not None:
            argv = strip_opt(argv, "--metrics-port")
        try:
            scfg = Config.load("events", path=a.config, env=dict(os.environ)).data["service"]
        except ConfigError as e:
            print(f"beholder: config error: {e}", file=sys.stderr)
            return 2
        mcfg, wcfg = scfg["metrics"], scfg.get("workers") or {}
        port = a.metrics_port if a.metrics_port is not None else (
            int(mcfg.get("port", 3000)) if mcfg.get("enabled", True) else -1)
        return Supervisor(argv, a.workers, metrics_port=port, metrics_host=str(mcfg.get("host", "0.0.0.0")),
                          command=worker_command(),
                          max_restarts=int(wcfg.get("max_restarts", 10)),
                          restart_window_s=float(wcfg.get("restart_window_s", 300.0)),
                          healthy_s=float(wcfg.get("healthy_s", 60.0)),
                          log=lambda m: print(f"beholder supervisor: {m}", file=sys.stderr)).run()
    env = dict(os.environ)
    try:
        cfg = Config.load("events", path=a.config, env=env)
    except ConfigError as e:
        print(f"beholder: config error: {e}", file=sys.stderr)
        return 2
    svc_cfg = cfg.data["service"]
    if a.source:
        svc_cfg["transport"]["kind"] = a.source
    if a.path:
        svc_cfg["transport"]["path"] = a.path
    if a.url:
        svc_cfg["transport"]["url"] = a.url
    if a.policy:
        svc_cfg["transport"]["policy"] = a.policy
    if a.dead_letter:
        svc_cfg["transport"]["dead_letter"] = a.dead_letter
    if a.format:
        svc_cfg["transport"]["format"] = a.format
    if a.log_level:
        svc_cfg["log"]["level"] = a.log_level
    if a.metrics_port is not None:
        svc_cfg["metrics"]["port"] = a.metrics_port
        svc_cfg["metrics"]["enabled"] = a.metrics_port >= 0
    if a.store:
        svc_cfg["store"]["backend"] = a.store
    elif a.media_fixture:
        svc_cfg["store"]["backend"] = "memory"  # a fixture preloads the in-memory store
    if a.dsn:
        svc_cfg["store"]["dsn"] = a.dsn
    if a.ordering:
        svc_cfg["ordering"] = a.ordering

    from .service import Service
    store = None
    if a.media_fixture:
        from .store import MemoryStore
        store = MemoryStore(_load_fixture(a.media_fixture)) if svc_cfg["store"]["backend"] == "memory" else None

    async def main() -> int:
        svc = Service(cfg, store=store)
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGINT, signal.SIGTERM):
            try:
                loop.add_signal_handler(sig, svc.request_stop)
            except (NotImplementedError, RuntimeError):
                pass
        try:
            await svc.init()
            stats = await svc.run()
        finally:
            await svc.close()
        if a.stats:
            print(json.dumps(stats, default=str), file=sys.stderr)
        return 1 if svc.source_error else 0

    try:
        return asyncio.run(main())
    except ConfigError as e:
        print(f"beholder: config error: {e}", file=sys.stderr)
        return 2
    except KeyboardInterrupt:
        return 130
    except Exception as e:  # startup failure is fatal (Q10 fix)
        print(f"beholder: fatal: {type(e).__name__}: {e}", file=sys.stderr)
        return 1


_SECRET_KEYS = ("token", "key", "password", "secret", "dsn", "url")


def redact_config(obj, parent: str = ""):
    """Copy of the config with credentials masked (keys.*, tokens, passwords, DSN/URL userinfo)."""
    import re
    if isinstance(obj, dict):
        return {k: redact_config(v, k) for k, v in obj.items()}
    if isinstance(obj, list):
        return [redact_config(v, parent) for v in obj]
    if isinstance(obj, str) and any(s in parent.lower() for s in _SECRET_KEYS):
        if parent.lower() in ("dsn", "url"):
            return re.sub(r"//([^:/@]+):([^@]+)@", r"//\1:***@", obj)
        return "***" if obj else obj
    return obj


def cmd_config(a: argparse.Namespace) -> int:
    """Validate the config and print the effective (merged, env-overridden) result, secrets masked."""
    try:
        cfg = Config.load("events", path=a.config, env=dict(os.environ))
    except ConfigError as e:
        print(f"beholder: config error: {e}", file=sys.stderr)
        return 2
    out = {"source": cfg.source, "no_trello": cfg.no_trello, "config": redact_config(cfg.data)}
    print(json.dumps(out, indent=2, default=str))
    return 0


def cmd_gen(a: argparse.Namespace) -> int:
    import time

    from .bench.generator import Workload
    w = Workload(n_media=a.media, seed=a.seed, progress_fraction=a.progress_fraction,
                 unknown_media_fraction=a.unknown_fraction)
    if a.media_out:
        with open(a.media_out, "w", encoding="utf-8") as f:
            json.dump([m._asdict() for m in w.media], f)
    out = open(a.out, "wb") if a.out else sys.stdout.buffer
    try:
        if a.ndjson:
            import base64
            from .topics import TOPIC_NAMES_BY_ID
            for t, p in w.events(a.events):
                out.write((json.dumps({"topic": TOPIC_NAMES_BY_ID[t], "b64": base64.b64encode(p).decode()})
                           + "\n").encode())
            return 0
        if a.rate <= 0:
            chunk = 65536
            left = a.events
            while left > 0:
                n = min(chunk, left)
                out.write(w.framed(n))
                left -= n
            return 0
        # paced producer: emit in 1 ms slices
        from .ops import frames
        evs = w.events(a.events)
        t0 = time.perf_counter()
        sent = 0
        per_ms = max(1, int(a.rate / 1000))
        while sent < len(evs):
            due = int((time.perf_counter() - t0) * a.rate) + per_ms
            if due > sent:
                out.write(frames(evs[sent:min(due, len(evs))]))
                out.flush()
                sent = min(due, len(evs))
            else:
                time.sleep(0.0005)
        return 0
    except BrokenPipeError:
        return 0
    finally:
        if a.out:
            out.close()
        else:
            try:
                out.flush()
            except BrokenPipeError:
                pass


def cmd_decode(a: argparse.Namespace) -> int:
    from .models import proto
    from .topics import PROGRESS_ID, STATUS_ID, TOPIC_NAMES_BY_ID
    from .transport.framing import iter_frames
    data = open(a.input, "rb").read() if a.input else sys.stdin.buffer.read()
    types = {STATUS_ID: proto.load("api.TelemetryStatus"), PROGRESS_ID: proto.load("api.TelemetryProgress")}
    from google.protobuf import json_format
    for t, p in iter_frames(data):
        rec = {"topic": TOPIC_NAMES_BY_ID[t] if t < len(TOPIC_NAMES_BY_ID) else t}
        try:
            rec["json"] = json_format.MessageToDict(proto.decode(types[t], p), preserving_proto_field_name=True)
        except Exception as e:  # noqa: BLE001
            rec["error"] = str(e)
        print(json.dumps(rec))
    return 0


def cmd_seed(a: argparse.Namespace) -> int:
    from .store import open_store

    async def main():
        st = open_store(a.store, a.dsn)
        await st.connect()
        try:
            await st.upsert_many(_load_fixture(a.fixture))
            print(await st.count())
        finally:
            await st.close()
    asyncio.run(main())
    return 0


def cmd_bench(a: argparse.Namespace) -> int:
    from .bench import harness
    return harness.main(a.rest)


def cmd_broker(a: argparse.Namespace) -> int:
    from .transport.amqp.broker import serve_forever
    try:
        asyncio.run(serve_forever(a.host, a.port))
    except KeyboardInterrupt:
        pass
    return 0


def cmd_publish(a: argparse.Namespace) -> int:
    from .transport.amqp import publish_frames
    data = open(a.input, "rb").read() if a.input else sys.stdin.buffer.read()
    n = asyncio.run(publish_frames(a.url, data))
    print(n)
    return 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="beholder", description="Beholder telemetry events service")
    sub = ap.add_subparsers(dest="cmd", required=True)

    r = sub.add_parser("run", help="run the service")
    r.add_argument("--config", help="config file (default: search for 'events')")
    r.add_argument("--source", choices=["amqp", "stdin", "file"])
    r.add_argument("--path", help="input file for --source file")
    r.add_argument("--url", help="AMQP URL (default: dyn('rabbitmq'))")
    r.add_argument("--policy", choices=["block", "drop_newest"], help="ingest backpressure policy")
    r.add_argument("--format", choices=["binary", "ndjson"], help="stdin/file framing (default binary)")
    r.add_argument("--dead-letter", help="append never-acked frames to this file")
    r.add_argument("--log-level", choices=["trace", "debug", "info", "warn", "error", "fatal", "silent"])
    r.add_argument("--metrics-port", type=int, help="metrics port (-1 disables the exposer)")
    r.add_argument("--store", choices=["memory", "sqlite", "postgres"])
    r.add_argument("--dsn")
    r.add_argument("--ordering", choices=["none", "per_media"])
    r.add_argument("--media-fixture", help="JSON list of media rows to preload (implies --store memory)")
    r.add_argument("--stats", action="store_true", help="print final stats JSON to stderr")
    r.add_argument("--workers", type=int, default=0,
                   help="N competing-consumer processes on the same queues (amqp); one merged /metrics")
    r.set_defaults(fn=cmd_run)

    c = sub.add_parser("config", help="validate and print the effective config (secrets masked)")
    c.add_argument("--config")
    c.set_defaults(fn=cmd_config)

    g = sub.add_parser("gen", help="generate synthetic framed telemetry")
    g.add_argument("--events", type=int, default=100)
    g.add_argument("--media", type=int, default=1000)
    g.add_argument("--seed", type=int, default=0)
    g.add_argument("--rate", type=float, default=0.0, help="events/s (0 = as fast as possible)")
    g.add_argument("--progress-fraction", type=float, default=0.9)
    g.add_argument("--unknown-fraction", type=float, default=0.0)
    g.add_argument("--ndjson", action="store_true")
    g.add_argument("--media-out", help="write the media fixture JSON here")
    g.add_argument("--out", help="output file (default stdout)")
    g.set_defaults(fn=cmd_gen)

    d = sub.add_parser("decode", help="framed stream -> NDJSON")
    d.add_argument("input", nargs="?")
    d.set_defaults(fn=cmd_decode)

    s = sub.add_parser("seed", help="load a media fixture into a store")
    s.add_argument("fixture")
    s.add_argument("--store", default="sqlite")
    s.add_argument("--dsn", required=True)
    s.set_defaults(fn=cmd_seed)

    b = sub.add_parser("bench", help="BASELINE.json measurement configs")
    b.add_argument("rest", nargs=argparse.REMAINDER)
    b.set_defaults(fn=cmd_bench)

    k = sub.add_parser("broker", help="run the built-in AMQP test broker (local development)")
    k.add_argument("--host", default="127.0.0.1")
    k.add_argument("--port", type=int, default=5672)
    k.set_defaults(fn=cmd_broker)

    p = sub.add_parser("publish", help="publish a framed stream to AMQP")
    p.add_argument("--url", required=True)
    p.add_argument("input", nargs="?")
    p.set_defaults(fn=cmd_publish)
    return ap


def strip_opt(argv: List[str], name: str) -> List[str]:
    out, skip = [], False
    for x in argv:
        if skip:
            skip = False
            continue
        if x == name:
            skip = True
            continue
        if x.startswith(name + "="):
            continue
        out.append(x)
    return out


def main(argv: Optional[List[str]] = None) -> int:
    a = build_parser().parse_args(argv)
    a.argv = argv
    return a.fn(a)
