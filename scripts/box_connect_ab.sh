#!/bin/bash
# Round-3 box sequence: GPU tier + smoke + the default bench line, then the
# service.http.max_connecting A/B (tls_e2e / tcp_e2e, cap 8 vs 100). Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-connect_ab}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as e; e.smoke()" > "$out/smoke.log" 2>&1 &&
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" &&
timeout -k 10 900 python -u scripts/connect_ab.py --reps 3 --events 100000 --tcp --out "$out" > "$out/connect_ab.log" 2>&1
rc=$?
echo "rc=$rc" >> "$out/bench.err"
exit $rc
