#!/bin/bash
# Interleaved headline A/B on one box: an older build checked out under _ab/<name> (built in-tree
# on the CPU container, not committed) against this tree. Headline phase only: no extras, no
# all-process phase. Usage: bash scripts/box_headline_ab.sh <out-name> [ab-dir] [runs]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-headline_ab}
other=${2:-_ab/r2}
runs=${3:-4}
mkdir -p "$out"
for i in $(seq 1 "$runs"); do
  for side in other head; do
    if [ "$side" = other ]; then dir=$other; else dir=.; fi
    (cd "$dir" && timeout -k 10 300 python bench.py --no-extras --all-procs-steps 0 --steps 20 --warmup 5) \
      >> "$out/$side.jsonl" 2>> "$out/$side.err" || exit $?
    echo "run $i $side done"
  done
done
