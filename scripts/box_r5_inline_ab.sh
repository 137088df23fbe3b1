#!/bin/bash
# Is the bench line's headline (run after every extra phase, in the same process) slower than
# the same headline in a fresh process? Alternates `bench.py --no-extras` and the full default
# bench.py on one box. One JSON line per run in gpurun_out/$OUT/runs.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-r5_inline_ab}
mkdir -p "$out"
for i in $(seq 1 "${RUNS:-3}"); do
  for arm in fresh full; do
    if [ "$arm" = fresh ]; then extra="--no-extras"; else extra=""; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 $extra --full-out "$out/full_$arm$i.json" > "$out/line.json" 2>> "$out/err.log" || exit 1
    python -c "import json; d=json.load(open('$out/full_$arm$i.json')); print(json.dumps({'arm': '$arm', 'pair': $i, 'value': d['value'], 'cpu_us': d['cpu_us_per_event'], 'p50': d['p50_handle_latency_us'], 'calib_ns': d['calib_ns'], 'minflt': d.get('headline_minflt')}))" >> "$out/runs.jsonl"
  done
  tail -2 "$out/runs.jsonl"
done
