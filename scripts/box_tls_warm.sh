#!/bin/bash
# Where the tls_e2e warm-up tail comes from after the background pool grow: tls_e2e with the grow
# on and off, and tls_e2e_preconnect, interleaved. Output under gpurun_out/$1.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-tls_warm}
mkdir -p "$out"
for r in 1 2 3; do
  timeout -k 10 150 python -m beholder_amd bench tls_e2e --out $out/grow_on_r$r.json > $out/grow_on_r$r.log 2>&1
  BEHOLDER_PG_BACKGROUND_GROW=0 timeout -k 10 150 python -m beholder_amd bench tls_e2e --out $out/grow_off_r$r.json > $out/grow_off_r$r.log 2>&1
  timeout -k 10 150 python -m beholder_amd bench tls_e2e_preconnect --out $out/preconnect_r$r.json > $out/preconnect_r$r.log 2>&1
  echo "r$r done"
done
echo done
