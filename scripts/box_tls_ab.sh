#!/bin/bash
# A/B of the native TLS path (BEHOLDER_NATIVE_TLS) on tls_e2e (HTTPS sinks), interleaved, plus
# tcp_e2e for reference. Output under gpurun_out/$1.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-tls_ab}
mkdir -p "$out"
for r in 1 2 3; do
  for v in on off; do
    if [ $v = on ]; then f=1; else f=0; fi
    BEHOLDER_NATIVE_TLS=$f timeout -k 10 150 python -m beholder_amd bench tls_e2e --out $out/tls_e2e_${v}_r$r.json > $out/tls_e2e_${v}_r$r.log 2>&1
    echo "$v r$r done"
  done
  timeout -k 10 150 python -m beholder_amd bench tcp_e2e --out $out/tcp_e2e_r$r.json > $out/tcp_e2e_r$r.log 2>&1
done
echo done
