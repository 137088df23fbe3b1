#!/bin/bash
# Interleaved A/B of the headline consumer alone (bench.py run_consumer, 20 steps): this tree
# ("new") against ab_old/ (an older tree built in place, as scripts/box_r5_e2e_ab.sh describes).
# One JSON line per measurement in gpurun_out/$OUT/ab.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-r5_head_ab}
mkdir -p "$out"
root=$PWD
probe='import asyncio, json, sys
import bench
a = bench.parse(["--steps", "20", "--warmup", "5", "--no-extras"])
r = asyncio.run(bench.run_consumer(a, 0, lambda: None, None))
print(json.dumps({"eps": r["events"] / r["elapsed"], "cpu_us": r["cpu_s"] / r["events"] * 1e6}))'
for i in $(seq 1 "${RUNS:-8}"); do
  for arm in new old; do
    if [ "$arm" = old ]; then dir=$root/ab_old; else dir=$root; fi
    (cd "$dir" && PYTHONPATH=$dir timeout -k 10 120 python -c "$probe") > "$out/tmp.json" 2>> "$out/ab.err" || exit 1
    python -c "import json,sys; d=json.load(open('$out/tmp.json')); d.update(arm='$arm', cfg='headline', pair=$i); print(json.dumps(d))" >> "$out/ab.jsonl"
  done
  tail -2 "$out/ab.jsonl"
done
