#!/bin/bash
# Native CPU profiles (scripts/cprof.py, SIGPROF sampler of _native_bench) of the headline
# consumer and of tcp_e2e, then the shared-queue sweep on its own. Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r5_prof}
mkdir -p "$out"
timeout -k 10 180 python scripts/cprof.py --workload headline --top 90 > "$out/headline.txt" 2> "$out/headline.err" &&
timeout -k 10 180 python scripts/cprof.py --workload tcp_e2e --events 400000 --top 90 > "$out/tcp_e2e.txt" 2> "$out/tcp_e2e.err" &&
timeout -k 10 300 python -m beholder_amd.bench.shared_queue --workers 1,2,4,8 --events-per-worker 100000 > "$out/shared_queue.jsonl" 2> "$out/shared_queue.err"
rc=$?
echo "rc=$rc" >> "$out/shared_queue.err"
exit $rc
