#!/bin/bash
# Interleaved headline A/B: this tree (new) against ab_old/ (an older tree built in place, made
# by `git archive <rev> beholder_amd bench.py | tar -x -C ab_old`). RUNS pairs; one JSON line per
# run under gpurun_out/$OUT/.
set -o pipefail
out=gpurun_out/${OUT:-ab_tree}
mkdir -p "$out"
runs=${RUNS:-6}
for i in $(seq 1 "$runs"); do
  for arm in new old; do
    if [ "$arm" = old ]; then b=ab_old/bench.py; else b=bench.py; fi
    timeout -k 10 120 python "$b" --steps 20 --warmup 5 --no-extras --all-procs-steps 0 > "$out/${arm}_$i.json" 2> "$out/${arm}_$i.err" || exit 1
    echo "$arm $i $(python -c "import json,sys; d=json.load(open('$out/${arm}_$i.json')); print(d['value'], d['cpu_us_per_event'])")"
  done
done
