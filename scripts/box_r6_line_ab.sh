#!/bin/bash
# Interleaved A/B of the whole bench line (every phase, in the driver's order): this tree ("new")
# against ab_old/ (an older tree built in place). One line per run: headline value, CPU per event,
# tcp_e2e and the paced 10k/s CPU per event. Output under gpurun_out/$OUT/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-line_ab}
mkdir -p "$out"
root=$PWD
for i in $(seq 1 "${RUNS:-3}"); do
  for arm in new old; do
    if [ "$arm" = old ]; then dir=$root/ab_old; else dir=$root; fi
    (cd "$dir" && timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --full-out "$root/$out/${arm}_$i.json" > "$root/$out/${arm}_$i.line" 2> "$root/$out/${arm}_$i.err") || exit 1
    python -c "
import json
d = json.load(open('$out/${arm}_$i.json'))
print('$arm', $i, d['value'], d['cpu_us_per_event'], d.get('tcp_e2e_events_per_sec'), d.get('tcp_e2e_rate_10k_cpu_us_per_event'), d.get('calib_py_ns'))" | tee -a "$out/summary.txt"
  done
done
