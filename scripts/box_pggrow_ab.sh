#!/bin/bash
# A/B of the Postgres pool's background grow (BEHOLDER_PG_BACKGROUND_GROW) on tcp_e2e: with it
# off, the query that finds every connection busy waits for the new connection's startup and
# authentication. The number to read is warmup_handle_latency_us. Output under gpurun_out/$1.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-pggrow_ab}
mkdir -p "$out"
for r in 1 2 3 4; do
  for v in on off; do
    if [ $v = on ]; then f=1; else f=0; fi
    BEHOLDER_PG_BACKGROUND_GROW=$f timeout -k 10 150 python -m beholder_amd bench tcp_e2e --out $out/tcp_e2e_${v}_r$r.json > $out/tcp_e2e_${v}_r$r.log 2>&1
    echo "$v r$r done"
  done
done
echo done
