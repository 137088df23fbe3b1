#!/bin/bash
# What the driver runs at round end, on one box: GPU-tier tests, smoke(), the default bench line.
# Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-round}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as e; e.smoke()" > "$out/smoke.log" 2>&1 &&
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --full-out "$out/bench_full.json" > "$out/bench.json" 2> "$out/bench.err"
rc=$?
echo "rc=$rc" >> "$out/bench.err"
exit $rc
