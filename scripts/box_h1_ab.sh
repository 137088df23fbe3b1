#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/h1ab
mkdir -p $O
for r in 1 2 3; do
  for v in old new; do
    d=$GRAFT_REPO_ROOT; [ $v = old ] && d=$GRAFT_REPO_ROOT/_ab_old
    (cd $d && timeout -k 10 150 python -m beholder_amd bench http_tcp --out $O/http_tcp_${v}_r$r.json > $O/http_tcp_${v}_r$r.log 2>&1) || exit 1
    (cd $d && timeout -k 10 150 python -m beholder_amd bench tcp_e2e --out $O/tcp_e2e_${v}_r$r.json > $O/tcp_e2e_${v}_r$r.log 2>&1) || exit 1
    echo "$v r$r done"
  done
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
