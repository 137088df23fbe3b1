#!/bin/bash
# The production path held at 10k events/s for minutes, in one-minute windows
# (scripts/paced_soak.py): tcp_e2e for 8 minutes, then tls_e2e for 5. Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-paced_soak}
mkdir -p "$out"
timeout -k 10 600 python -u scripts/paced_soak.py --rate 10000 --seconds 480 --window-s 60 \
  --out "$out/tcp_10k.json" > "$out/tcp_10k.log" 2>&1 &&
timeout -k 10 420 python -u scripts/paced_soak.py --rate 10000 --seconds 300 --window-s 60 --tls \
  --out "$out/tls_10k.json" > "$out/tls_10k.log" 2>&1
rc=$?
echo "rc=$rc" >> "$out/tls_10k.log"
exit $rc
