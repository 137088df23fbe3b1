#!/usr/bin/env python3
"""A/B of ``service.http.max_connecting`` on the production-shaped TCP configs (box tier).

Interleaves ``tls_e2e`` (and ``tcp_e2e``) runs with the connect admission cap at its default
(8) and effectively off (``max_connecting`` = prefetch, 100: every first request of the burst
starts its own handshake, the round-2 behaviour). Prints one JSON line per run; the number to
read is the warm-up p999 (the first 5,000 events). Usage:
``python scripts/connect_ab.py --reps 3 --events 100000 --out gpurun_out/x``
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from beholder_amd.bench import harness  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--events", type=int, default=100_000)
    ap.add_argument("--caps", default="8,100")
    ap.add_argument("--tcp", action="store_true", help="also run tcp_e2e")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = []
    for rep in range(a.reps):
        for tls in ((True, False) if a.tcp else (True,)):
            for cap in (int(x) for x in a.caps.split(",")):
                r = harness._tcp_e2e(a.events, http_servers=4 if tls else 2, tls=tls, max_connecting=cap)
                w, s = r["warmup_handle_latency_us"], r["handle_latency_us"]
                row = {"config": "tls_e2e" if tls else "tcp_e2e", "max_connecting": cap, "rep": rep,
                       "events_per_sec": round(r["ingest_rate_eps"] or 0, 1),
                       "cpu_us_per_event": round(r["cpu_us_per_event"] or 0, 3),
                       "warmup_p50_us": round(w.get("p50", 0), 1), "warmup_p99_us": round(w.get("p99", 0), 1),
                       "warmup_p999_us": round(w.get("p999", 0), 1), "steady_p999_us": round(s.get("p999", 0), 1),
                       "http_connections": r["http"].get("connections"),
                       "connecting_peak": r["http"].get("connecting_peak"), "errors": r["errors"]}
                rows.append(row)
                print(json.dumps(row), flush=True)
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, "connect_ab.json"), "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
