#!/bin/bash
# Round-4 box run: the driver's bench command, RUNS times, each line kept (gpurun_out/$OUT/);
# ARGS adds bench.py flags (e.g. ARGS="--no-extras --all-procs-steps 0" for headline + calibration only).
set -o pipefail
out=gpurun_out/${OUT:-box_r4_bench}
mkdir -p "$out"
runs=${RUNS:-2}
for i in $(seq 1 "$runs"); do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 $ARGS > "$out/bench_$i.json" 2> "$out/bench_$i.err" || exit $?
  echo "run $i done: $(head -c 200 "$out/bench_$i.json")"
done
