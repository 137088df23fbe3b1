"""Long production-shaped runs (memory and latency over many events): tcp_e2e and tls_e2e with
N events each (default 1.5M). Prints one JSON object."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from beholder_amd.bench import harness  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_500_000
out = {}
for c in ("tcp_e2e", "tls_e2e"):
    r = harness.run_config(c, events=n)
    out[c] = {k: r[k] for k in ("acked", "errors", "ingest_rate_eps", "cpu_us_per_event", "rss_growth_mb",
                                "handle_latency_us", "http")}
    att = r.get("attribution_steady") or {}
    out[c]["slow_blamed"] = att.get("blamed")
    out[c]["processes"] = {name: {k: p.get(k) for k in ("loop_lag_max_us", "loop_stalls", "gc_max_pause_us")}
                           for name, p in (att.get("processes") or {}).items()}
    print(f"{c}: {json.dumps(out[c])}", file=sys.stderr, flush=True)  # progress for long runs
print(json.dumps(out))
