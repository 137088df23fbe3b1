#!/bin/bash
# Box A/B: native IOFuture (synchronous Driver wake-up) vs plain asyncio futures for I/O replies.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2 3; do
  BEHOLDER_IOFUTURE=0 timeout -k 10 300 python -m beholder_amd bench tcp_e2e --events 150000 > gpurun_out/iof_r${rep}_off.json 2>&1 || exit 1
  BEHOLDER_IOFUTURE=1 timeout -k 10 300 python -m beholder_amd bench tcp_e2e --events 150000 > gpurun_out/iof_r${rep}_on.json 2>&1 || exit 1
done
timeout -k 10 600 python -m pytest tests -x -q -m "not gpu" > gpurun_out/pytest_cpu.log 2>&1
