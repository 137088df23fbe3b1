#!/bin/bash
# Headline-only A/B of the allocator (interleaved): pymalloc (default), PYTHONMALLOC=malloc, and
# malloc with glibc's transparent-huge-page tunable. One JSON line per run in gpurun_out/$OUT/.
set -o pipefail
out=gpurun_out/${OUT:-r4_alloc_ab}
mkdir -p "$out"
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > "$out/thp.txt" 2>&1
for i in $(seq 1 "${RUNS:-4}"); do
  for m in default malloc hugetlb; do
    case $m in
      default) env=() ;;
      malloc) env=(PYTHONMALLOC=malloc) ;;
      hugetlb) env=(PYTHONMALLOC=malloc GLIBC_TUNABLES=glibc.malloc.hugetlb=1) ;;
    esac
    env "${env[@]}" timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-extras --all-procs-steps 0 \
      > "$out/${m}_$i.json" 2> "$out/${m}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], d['value'], d['cpu_us_per_event'], d['headline_minflt'], d['calib_ns'])" "$out/${m}_$i.json" $m
  done
done
