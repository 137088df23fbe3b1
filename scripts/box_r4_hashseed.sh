#!/bin/bash
# Does the headline's run-to-run spread follow the string-hash seed? Headline + calibrations only,
# PYTHONHASHSEED fixed per run (two seeds, interleaved), then unset.
set -o pipefail
out=gpurun_out/${OUT:-r4_hashseed}
mkdir -p "$out"
for i in 1 2 3 4; do
  for seed in 0 1; do
    PYTHONHASHSEED=$seed timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-extras --all-procs-steps 0 \
      > "$out/seed${seed}_$i.json" 2> "$out/seed${seed}_$i.err" || exit $?
    echo "seed $seed run $i: $(head -c 120 "$out/seed${seed}_$i.json")"
  done
done
