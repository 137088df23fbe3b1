#!/bin/bash
# Where the paced production path's CPU goes at 100k events/s (the consumer near one core there,
# 10 us/event, against 3.3 at saturation): call-stack profiles of tcp_e2e paced at 100k/s and
# 30k/s. Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-box_r6_rate100k}
mkdir -p "$out"
timeout -k 10 300 python scripts/cprof.py --workload tcp_e2e --events 400000 --rate 100000 --depth 16 --top 60 > "$out/tcp_e2e_100k.txt" 2>&1 &&
timeout -k 10 300 python scripts/cprof.py --workload tcp_e2e --events 150000 --rate 30000 --depth 16 --top 60 > "$out/tcp_e2e_30k.txt" 2>&1
