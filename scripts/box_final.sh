#!/bin/bash
# End-of-round check on one box: the driver's sequence (scripts/box_round.sh), then five
# tcp_e2e and five tls_e2e runs for medians. Output under gpurun_out/$1.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-final}
bash scripts/box_round.sh "${1:-final}"
for r in 1 2 3 4 5; do
  for c in tcp_e2e tls_e2e; do
    timeout -k 10 150 python -m beholder_amd bench $c --out $out/${c}_r$r.json > $out/${c}_r$r.log 2>&1
    echo "$c r$r done"
  done
done
echo done
