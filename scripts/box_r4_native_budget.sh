#!/bin/bash
# Round-4 native-I/O budget: tcp_e2e / tls_e2e (warm-up and steady p999),
# interleaved, current tree (A) against the tree with handshakes on the loop thread and no
# continuation-first queueing (B: BEHOLDER_AB_HS_THREADS=0 BEHOLDER_AB_FRONT=0; max_connecting
# stays 8). RUNS pairs; one JSON line per run under gpurun_out/$OUT/.
# Historical: the BEHOLDER_AB_* switches were removed after this A/B (profiles/box_r4_native_budget/),
# so arms B and C now run the same code as A.
set -o pipefail
out=gpurun_out/${OUT:-box_r4_native_budget}
mkdir -p "$out"
runs=${RUNS:-8}
probe='import json, sys
sys.path.insert(0, ".")
from beholder_amd.bench import harness
r = {}
for name, kw in (("tcp", {}), ("tls", {"http_servers": 4, "tls": True})):
    x = harness._tcp_e2e(50000, **kw)
    r[name] = {"eps": x["ingest_rate_eps"], "p999": x["handle_latency_us"].get("p999"),
               "warm_p999": x["warmup_handle_latency_us"].get("p999"), "warm_p99": x["warmup_handle_latency_us"].get("p99"),
               "cpu": x["cpu_us_per_event"], "errors": x["errors"], "http": x.get("http"),
               "blamed": (x.get("attribution_steady") or {}).get("blamed"),
               "warm_blamed": (x.get("attribution_warmup") or {}).get("blamed")}
print(json.dumps(r))'
arms=${ARMS:-AB}  # A = current; B = no handshake threads, no continuation-first; C = no continuation-first only
for i in $(seq 1 "$runs"); do
  for arm in $(echo "$arms" | fold -w1); do
    case $arm in
      A) env=() ;;
      B) env=(BEHOLDER_AB_HS_THREADS=0 BEHOLDER_AB_FRONT=0) ;;
      C) env=(BEHOLDER_AB_FRONT=0) ;;
    esac
    env "${env[@]}" timeout -k 10 120 python3 -c "$probe" > "$out/${arm}_$i.json" 2> "$out/${arm}_$i.err" || exit $?
    echo "run $i arm $arm: $(cut -c1-150 "$out/${arm}_$i.json")"
  done
done
