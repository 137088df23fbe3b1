#!/bin/bash
# Box run: long soak (RSS curve, GC pauses), production-shaped profile, validation tier.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m beholder_amd bench soak --events 10000000 > gpurun_out/soak10m.json 2> gpurun_out/soak10m.err &&
timeout -k 10 300 python scripts/profile_e2e.py 80000 > gpurun_out/cprofile_e2e.txt 2>&1 &&
timeout -k 10 300 python -m beholder_amd bench amqp tcp_e2e http_tcp > gpurun_out/transports.json 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
