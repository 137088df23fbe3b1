#!/bin/bash
# Call-stack profiles of the headline and tcp_e2e on the final tree. Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r5_prof4}
mkdir -p "$out"
timeout -k 10 180 python scripts/cprof.py --workload headline --steps 120 --top 90 --depth 24 > "$out/headline.txt" 2> "$out/headline.err" &&
timeout -k 10 240 python scripts/cprof.py --workload tcp_e2e --events 1500000 --top 90 --depth 24 > "$out/tcp_e2e.txt" 2> "$out/tcp_e2e.err"
