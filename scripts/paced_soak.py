"""The production path held at one of BASELINE's rates for minutes: ``tcp_e2e`` / ``tls_e2e``
(AMQP + Postgres + HTTP(S) sinks, every dependency over sockets) with the replay broker pacing
its sends, measured in windows of ``--window-s`` seconds. Each window reports handler
start->ack and receive->ack p50 / p99 / p999 / max, RSS and the loop stalls seen, so a drift
(a pool that grows, a histogram or trace that slows the loop, a leak) shows as a trend rather
than disappearing into one whole-run percentile.

    python scripts/paced_soak.py --rate 10000 --seconds 600 --window-s 60 [--tls] --out soak.json

Writes the whole ``_tcp_e2e`` result (``windows`` included) as JSON and prints one line per
window while it runs (stderr).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--rate", type=float, default=10000.0, help="events per second the broker sends")
    ap.add_argument("--seconds", type=float, default=600.0, help="length of the measured phase")
    ap.add_argument("--window-s", type=float, default=60.0)
    ap.add_argument("--tls", action="store_true", help="HTTPS sinks (tls_e2e)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    from beholder_amd.bench import harness
    if a.rate <= 0 or a.seconds <= 0 or a.window_s <= 0:
        ap.error("--rate, --seconds and --window-s must be > 0")
    measured = int(a.rate * a.seconds)
    n = measured + measured // 9  # paced runs warm up on a tenth of all events
    r = harness._tcp_e2e(n, http_servers=4 if a.tls else 2, tls=a.tls, rate=a.rate,
                         window_events=max(1, int(a.rate * a.window_s)))
    r["config"] = "tls_e2e" if a.tls else "tcp_e2e"
    with open(a.out, "w") as f:
        json.dump(r, f, indent=1, default=str)
    ws = r.get("windows") or []
    hl = r.get("handle_latency_us") or {}
    print(json.dumps({"config": r["config"], "rate": a.rate, "measured_events": r.get("measured_events"),
                      "acked": r.get("acked"), "errors": r.get("errors"),
                      "handle_p50_us": hl.get("p50"), "handle_p99_us": hl.get("p99"), "handle_p999_us": hl.get("p999"),
                      "cpu_us_per_event": r.get("cpu_us_per_event"), "rss_growth_mb": r.get("rss_growth_mb"),
                      "window_p99_us": [w.get("handle_p99_us") for w in ws],
                      "window_rss_mb": [w.get("rss_mb") for w in ws]}), flush=True)
    return 0 if r.get("errors") == 0 and r.get("acked") == n else 1


if __name__ == "__main__":
    raise SystemExit(main())
