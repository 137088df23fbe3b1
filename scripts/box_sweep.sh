#!/bin/bash
# Box run: consumer-process sweep per rank (twice, interleaved, to expose box noise), then
# the transport configs (AMQP ingest, all-TCP production shape) and the box-tier tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for p in 1 8 12 14 15 16; do
    timeout -k 10 300 python bench.py --procs-per-rank $p > gpurun_out/sweep_r${rep}_p$p.json 2> gpurun_out/sweep_r${rep}_p$p.err || exit 1
  done
done
timeout -k 10 300 python -m beholder_amd bench amqp --events 400000 > gpurun_out/amqp.json 2>&1 &&
timeout -k 10 300 python -m beholder_amd bench tcp_e2e --events 200000 > gpurun_out/tcp_e2e.json 2>&1 &&
timeout -k 10 300 python -m beholder_amd bench http_tcp > gpurun_out/http_tcp.json 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
