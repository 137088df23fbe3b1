#!/bin/bash
# Round-6 box session: where the production path's CPU goes at BASELINE's rates (paced tcp_e2e),
# against saturation. Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-box_r6_lowrate}
mkdir -p "$out"
timeout -k 10 300 python scripts/cprof.py --workload tcp_e2e --events 30000 --rate 10000 --depth 16 --top 50 > "$out/tcp_e2e_10k.txt" 2>&1 &&
timeout -k 10 300 python scripts/cprof.py --workload tcp_e2e --events 3000 --rate 1000 --depth 16 --top 50 > "$out/tcp_e2e_1k.txt" 2>&1 &&
timeout -k 10 300 python scripts/cprof.py --workload tcp_e2e --events 200000 --depth 16 --top 50 > "$out/tcp_e2e_sat.txt" 2>&1
