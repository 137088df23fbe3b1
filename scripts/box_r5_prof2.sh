#!/bin/bash
# Shared-queue sweep (after the broker's speed-up) and call-stack profiles of tcp_e2e and the
# headline on the box. Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r5_prof2}
mkdir -p "$out"
timeout -k 10 300 python -m beholder_amd.bench.shared_queue --workers 1,2,4,8 --events-per-worker 100000 > "$out/shared_queue.jsonl" 2> "$out/shared_queue.err" &&
timeout -k 10 240 python scripts/cprof.py --workload tcp_e2e --events 1500000 --top 80 --depth 24 > "$out/tcp_e2e.txt" 2> "$out/tcp_e2e.err" &&
timeout -k 10 180 python scripts/cprof.py --workload headline --steps 60 --top 80 --depth 24 > "$out/headline.txt" 2> "$out/headline.err"
