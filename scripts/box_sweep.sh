#!/bin/bash
# Box run: consumer-process sweep per rank + AMQP ingest + consumer profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for p in 1 4 8 12 15; do
  timeout -k 10 300 python bench.py --procs-per-rank $p > gpurun_out/sweep_p$p.json 2> gpurun_out/sweep_p$p.err || exit 1
done
timeout -k 10 300 python -m beholder_amd bench amqp --events 400000 > gpurun_out/amqp.json 2>&1 &&
timeout -k 10 300 python scripts/profile_consumer.py > gpurun_out/cprofile_consumer.txt 2>&1
