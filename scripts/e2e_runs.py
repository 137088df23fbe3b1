"""Repeat the production-shaped e2e phases in one process and print every run's rate, CPU per
event, system time, events per NetPoller callback and core speed (bench.py ``*_e2e_runs``), to see
what moves CPU per event between runs of one line.

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
    out = bench._e2e_keys(prefix, harness._tcp_e2e, a.events, repeats=a.repeats, **kw)
    print(json.dumps({"runs": out[f"{prefix}_runs"], "median_io_per_event": out[f"{prefix}_io_per_event"]}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
