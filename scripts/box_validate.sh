#!/bin/bash
# GPU-box validation run: build check, box-tier tests, bench, BASELINE configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
lscpu > gpurun_out/lscpu.txt 2>&1
nproc > gpurun_out/nproc.txt
python -c "import sys; print(sys.version)" > gpurun_out/python.txt
timeout -k 10 300 python __graft_entry__.py > gpurun_out/entry.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 600 python -m beholder_amd bench all --out gpurun_out/baseline_configs.json > gpurun_out/baseline.log 2>&1
