#!/bin/bash
# Does anything before the headline in bench.py (TCP extras, the 15-process phase) move the
# single-process value? Full default runs interleaved with headline-only runs on one box; each
# line carries cpu_us_per_event and involuntary_ctx_switches of the timed steps. Output under
# gpurun_out/$1.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-headline_ab}
mkdir -p "$out"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $out/full.jsonl 2>> $out/full.err
  echo "full r$r done"
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --all-procs-steps 0 >> $out/headline.jsonl 2>> $out/headline.err
  echo "headline r$r done"
done
echo done
