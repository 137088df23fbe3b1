#!/bin/bash
# Production-shaped path on the box: tcp_e2e and http_tcp (every dependency over TCP), steady
# state after a warm-up, then a cProfile of tcp_e2e. Output under gpurun_out/$1.
set -euo pipefail
out=gpurun_out/${1:-io_profile}
mkdir -p "$out"
nproc > "$out/nproc.txt"
for i in 1 2; do
  timeout -k 10 240 python -u -c "
import json, sys
from beholder_amd.bench import harness
r = harness.run_config('tcp_e2e', events=100000)
print(json.dumps(r))" > "$out/tcp_e2e_$i.json"
done
timeout -k 10 240 python -u -c "
import json
from beholder_amd.bench import harness
r = harness.run_config('http_tcp', events=100000)
print(json.dumps(r))" > "$out/http_tcp.json"
timeout -k 10 300 python -u scripts/profile_e2e.py 100000 > "$out/cprofile_tcp_e2e.txt"
echo done
