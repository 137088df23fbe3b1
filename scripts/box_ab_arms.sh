#!/bin/bash
# Interleaved headline A/B/n on one box: ARMS="name:dir name:dir ..." (each dir a tree with its
# extensions built in place; "." is this tree). RUNS rounds, the arms in turn within each round;
# one JSON line per run under gpurun_out/$OUT/, and "arm round value cpu_us_per_event" on stdout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-ab_arms}
mkdir -p "$out"
runs=${RUNS:-6}
for i in $(seq 1 "$runs"); do
  for arm in $ARMS; do
    name=${arm%%:*}
    dir=${arm#*:}
    (cd "$dir" && timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --all-procs-steps 0 \
        --full-out "") > "$out/${name}_$i.json" 2> "$out/${name}_$i.err" || exit 1
    echo "$name $i $(python -c "import json; d=json.load(open('$out/${name}_$i.json')); print(d['value'], d['cpu_us_per_event'])")"
  done
done
