#!/bin/bash
# Box A/B: consumer processes pinned to CPUs vs free, interleaved three times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py > gpurun_out/pin_r${rep}_off.json 2> gpurun_out/pin_r${rep}_off.err || exit 1
  timeout -k 10 300 python bench.py --pin > gpurun_out/pin_r${rep}_on.json 2> gpurun_out/pin_r${rep}_on.err || exit 1
done
nproc > gpurun_out/nproc.txt; python -c "import os; print(sorted(os.sched_getaffinity(0)))" > gpurun_out/affinity.txt
