"""Repeat the production-shaped e2e phases in one process and print every run's rate, CPU per
event, system time, events per NetPoller callback and core speed (bench.py ``*_e2e_runs``), to see
what moves CPU per event between runs of one line. One JSON line per run, with each fake
process's CPU share of the window.

    python scripts/e2e_runs.py [--repeats 6] [--events 250000] [--tls]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--repeats", type=int, default=6)
    ap.add_argument("--events", type=int, default=250_000)
    ap.add_argument("--tls", action="store_true")
    a = ap.parse_args(argv)
    import bench
    from beholder_amd.bench import harness
    harness._tcp_e2e(20_000)  # the bench's unmeasured warm-up pass
    kw = {"http_servers": 4, "tls": True} if a.tls else {}
    prefix = "tls_e2e" if a.tls else "tcp_e2e"
    runs = []
    for _ in range(a.repeats):
        e = harness._tcp_e2e(a.events, **kw)
        runs.append({"events_per_sec": bench._r(e.get("ingest_rate_eps"), 1),
                     "cpu_us_per_event": bench._r(e.get("cpu_us_per_event")),
                     "sys_cpu_us_per_event": bench._r(e.get("sys_cpu_us_per_event")),
                     "events_per_poll_run": bench._events_per_poll(e),
                     "fakes_util": e.get("fakes_util"), "run_delay_ms": e.get("run_delay_ms"),
                     "server_side": e.get("server_side"), "calib_ns": e.get("calib_ns")})
        print(json.dumps({prefix: runs[-1]}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
