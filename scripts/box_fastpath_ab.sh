#!/bin/bash
# A/B of the native H1 request path and Postgres pool pick (BEHOLDER_NATIVE_H1 / BEHOLDER_NATIVE_POOL)
# on the production-shaped configs, interleaved. Output under gpurun_out/$1.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-fastpath_ab}
mkdir -p "$out"
for r in 1 2 3; do
  for v in on off; do
    if [ $v = on ]; then f=1; else f=0; fi
    BEHOLDER_NATIVE_H1=$f BEHOLDER_NATIVE_POOL=$f timeout -k 10 150 python -m beholder_amd bench tcp_e2e --out $out/tcp_e2e_${v}_r$r.json > $out/tcp_e2e_${v}_r$r.log 2>&1
    BEHOLDER_NATIVE_H1=$f BEHOLDER_NATIVE_POOL=$f timeout -k 10 150 python -m beholder_amd bench http_tcp --out $out/http_tcp_${v}_r$r.json > $out/http_tcp_${v}_r$r.log 2>&1
    echo "$v r$r done"
  done
done
timeout -k 10 300 python -u scripts/profile_e2e.py 100000 > "$out/cprofile_tcp_e2e.txt"
echo done
