"""One paced production-path measurement for an A/B: tcp_e2e (or tls_e2e with --tls) at each of
the bench's paced rates (bench.E2E_RATES), in this process, after the bench's unmeasured warm-up
pass. Prints one JSON line per rate: handler start->ack p50/p99 and the consumer's CPU per event.

Run from the root of the tree to measure (PYTHONPATH=that root): scripts/box_r6_direct_ab.sh.
"""
import argparse
import json
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tls", action="store_true")
    ap.add_argument("--scale", type=float, default=1.0, help="events per rate times this")
    ap.add_argument("--stall-period", type=float, default=0.001,
                    help="the stall monitor's tick on the consumer's loop, seconds")
    a = ap.parse_args()
    from beholder_amd.bench import harness
    kw = dict(http_servers=4, tls=True) if a.tls else {}
    kw["stall_period_s"] = a.stall_period
    harness._tcp_e2e(20000, **kw)  # unmeasured: first-touch pages, lazily opened connections
    for name, rate, n in (("1k", 1000, 3000), ("10k", 10000, 20000), ("100k", 100000, 100000)):
        e = harness._tcp_e2e(max(200, int(n * a.scale)), rate=rate, **kw)
        h = e.get("handle_latency_us") or {}
        print(json.dumps({"rate": name, "cpu_us": round(e["cpu_us_per_event"], 2),
                          "sys_us": round(e.get("sys_cpu_us_per_event", 0.0), 2),
                          "p50": h.get("p50"), "p99": h.get("p99")}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
