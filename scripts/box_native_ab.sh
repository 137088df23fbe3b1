#!/bin/bash
# GPU-box A/B: compiled handlers (default) vs the Python handlers (service.native_handlers: false), one consumer
# process, three interleaved repetitions; then the default bench (all consumer processes) and the
# production-shaped tcp_e2e config both ways. Every step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/native_ab
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --procs-per-rank 1 > gpurun_out/native_ab/p1_native_r$r.json 2>&1 || exit 1
  BEHOLDER_CFG__service__native_handlers=false timeout -k 10 120 python bench.py --procs-per-rank 1 \
    > gpurun_out/native_ab/p1_python_r$r.json 2>&1 || exit 1
done
timeout -k 10 200 python bench.py > gpurun_out/native_ab/bench_native.json 2>&1 || exit 1
BEHOLDER_CFG__service__native_handlers=false timeout -k 10 200 python bench.py > gpurun_out/native_ab/bench_python.json 2>&1 || exit 1
timeout -k 10 200 python -m beholder_amd bench tcp_e2e --out gpurun_out/native_ab/tcp_e2e_native.json \
  > gpurun_out/native_ab/tcp_e2e_native.log 2>&1 || exit 1
BEHOLDER_CFG__service__native_handlers=false timeout -k 10 200 python -m beholder_amd bench tcp_e2e \
  --out gpurun_out/native_ab/tcp_e2e_python.json > gpurun_out/native_ab/tcp_e2e_python.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/native_ab/pytest_gpu.log 2>&1
