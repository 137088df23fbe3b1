#!/bin/bash
# A/B of service.http.preconnect on the production-shaped configs: tcp_e2e / tls_e2e against
# their *_preconnect variants (100 sink connections opened at init), interleaved. The number to
# read is warmup_handle_latency_us (the first 5,000 events); the steady state should not move.
# Output under gpurun_out/$1.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-preconnect_ab}
mkdir -p "$out"
for r in 1 2 3; do
  for c in tcp_e2e tcp_e2e_preconnect tls_e2e tls_e2e_preconnect; do
    timeout -k 10 150 python -m beholder_amd bench $c --out $out/${c}_r$r.json > $out/${c}_r$r.log 2>&1
    echo "$c r$r done"
  done
done
echo done
