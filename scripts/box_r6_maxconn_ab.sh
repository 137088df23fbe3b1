#!/bin/bash
# tls_e2e's warm-up tail (the first wave of TLS handshakes) against service.http.max_connecting
# (connects + handshakes in flight per origin): 8 (the default) against 32, interleaved, fresh
# fakes per run. One JSON line per run in gpurun_out/$OUT/ab.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-maxconn_ab}
mkdir -p "$out"
for i in $(seq 1 "${RUNS:-4}"); do
  for mc in ${ORDER:-8 32}; do
    timeout -k 10 120 python -c "
import json
from beholder_amd.bench import harness
r = harness._tcp_e2e(250000, http_servers=4, tls=True, max_connecting=$mc)
w, h = r['warmup_handle_latency_us'], r['handle_latency_us']
print(json.dumps({'max_connecting': $mc, 'pair': $i, 'eps': round(r['ingest_rate_eps']), 'cpu_us': round(r['cpu_us_per_event'], 3),
                  'warm_p99': w.get('p99'), 'warm_p999': w.get('p999'), 'p999': h.get('p999'),
                  'connections': r['http'].get('connections'), 'dial_max_us': r['http'].get('dial_max_us'),
                  'queue_wait_max_us': r['http'].get('queue_wait_max_us')}))" >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit 1
    tail -n 1 "$out/ab.jsonl"
  done
done
