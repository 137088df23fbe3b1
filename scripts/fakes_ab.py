import json, sys
sys.path.insert(0, ".")
from beholder_amd.bench import harness
out = []
for i in range(3):
    for n in ((4, 8) if i % 2 == 0 else (8, 4)):
        x = harness._tcp_e2e(100000, http_servers=n, tls=True)
        r = {"servers": n, "eps": round(x["ingest_rate_eps"]), "warm_p999": x["warmup_handle_latency_us"].get("p999"),
             "warm_p99": x["warmup_handle_latency_us"].get("p99"), "p999": x["handle_latency_us"].get("p999"),
             "dial_max": (x.get("http") or {}).get("dial_max_us"), "qwait_max": (x.get("http") or {}).get("queue_wait_max_us")}
        print(json.dumps(r), flush=True)
