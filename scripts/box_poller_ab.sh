#!/bin/bash
# A/B of the shared epoll set (BEHOLDER_NATIVE_POLLER) on tcp_e2e and tls_e2e, interleaved.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-poller_ab}
mkdir -p "$out"
for r in ${REPS:-1 2 3}; do
  for v in on off; do
    if [ $v = on ]; then f=1; else f=0; fi
    for cfg in ${CFGS:-tcp_e2e tls_e2e}; do
      BEHOLDER_NATIVE_POLLER=$f timeout -k 10 150 python -m beholder_amd bench $cfg --out $out/${cfg}_${v}_r$r.json > $out/${cfg}_${v}_r$r.log 2>&1
    done
    echo "$v r$r done"
  done
done
echo done
