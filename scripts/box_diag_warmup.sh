#!/bin/bash
# Warm-up tail diagnosis on the GPU box (scripts/diag_warmup.py): TLS and TCP, three runs each in
# one process, with loop stalls, GC pauses, dial times and cgroup CPU throttling per run.
set -o pipefail
out=gpurun_out/${1:-diag_warmup}
mkdir -p "$out"
cat /proc/self/cgroup > "$out/cgroup.txt" 2>&1; nproc >> "$out/cgroup.txt"
timeout -k 10 300 python -u scripts/diag_warmup.py --tls --reps 3 > "$out/tls.jsonl" 2> "$out/tls.err" &&
timeout -k 10 300 python -u scripts/diag_warmup.py --reps 3 > "$out/tcp.jsonl" 2> "$out/tcp.err"
