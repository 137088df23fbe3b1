#!/bin/bash
# Interleaved headline A/B of one environment setting: arm "env" runs bench.py with $AB_ENV
# exported (e.g. AB_ENV="GLIBC_TUNABLES=glibc.malloc.trim_threshold=268435456"), arm "base"
# without. RUNS pairs; one JSON line per run under gpurun_out/$OUT/.
set -o pipefail
out=gpurun_out/${OUT:-env_ab}
mkdir -p "$out"
runs=${RUNS:-6}
for i in $(seq 1 "$runs"); do
  for arm in env base; do
    if [ "$arm" = env ]; then
      timeout -k 10 120 env $AB_ENV python bench.py --steps 20 --warmup 5 --no-extras > "$out/${arm}_$i.json" 2> "$out/${arm}_$i.err" || exit 1
    else
      timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras > "$out/${arm}_$i.json" 2> "$out/${arm}_$i.err" || exit 1
    fi
    echo "$arm $i $(python -c "import json; d=json.load(open('$out/${arm}_$i.json')); print(d['value'], d['cpu_us_per_event'])")"
  done
done
