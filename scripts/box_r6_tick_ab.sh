#!/bin/bash
# What the bench's stall monitor costs the paced production path: paced tcp_e2e (1k/10k/100k
# events/s) with the monitor ticking every 1 ms (the bench's default) against every 50 ms,
# interleaved, this tree. One JSON line per rate and run in gpurun_out/$OUT/ab.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-tick_ab}
mkdir -p "$out"
for i in $(seq 1 "${RUNS:-4}"); do
  for arm in 0.001 0.05; do
    PYTHONPATH=$PWD timeout -k 10 120 python scripts/paced_ab.py --stall-period "$arm" > "$out/tmp.jsonl" 2>> "$out/ab.err" || exit 1
    python -c "
import json
for ln in open('$out/tmp.jsonl'):
    r = json.loads(ln); r.update(tick_s=$arm, pair=$i); print(json.dumps(r))" >> "$out/ab.jsonl" || exit 1
  done
  tail -n 6 "$out/ab.jsonl"
done
