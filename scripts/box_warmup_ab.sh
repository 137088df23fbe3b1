#!/bin/bash
# Interleaved warm-up tail A/B on one box (scripts/diag_warmup.py): an older build checked out
# under _ab/<name> (built in-tree on the CPU container, not committed) against this tree.
# Usage: bash scripts/box_warmup_ab.sh <out-name> [ab-dir] [rounds] [--tls]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-warmup_ab}
other=${2:-_ab/head0}
rounds=${3:-3}
flag=${4:---tls}
mkdir -p "$out"
for i in $(seq 1 "$rounds"); do
  for side in other head; do
    if [ "$side" = other ]; then dir=$other; else dir=.; fi
    (cd "$dir" && timeout -k 10 300 python -u scripts/diag_warmup.py $flag --reps 2) \
      >> "$out/$side.jsonl" 2>> "$out/$side.err" || exit $?
    echo "round $i $side done"
  done
done
