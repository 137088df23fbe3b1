#!/bin/bash
# The soak on the final tree: the bench's own in-process soak at 1M and 3M events (RSS growth
# from after init), and the CLI's 10M-event soak. Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r5_soak_final}
mkdir -p "$out"
probe='import sys, json
sys.path.insert(0, ".")
import bench
a = bench.parse(["--soak-events", sys.argv[1]])
r = bench.soak_extras(a)
print(json.dumps(r))'
timeout -k 10 120 python -c "$probe" 1000000 > "$out/soak1m.json" 2> "$out/soak1m.err" &&
timeout -k 10 180 python -c "$probe" 3000000 > "$out/soak3m.json" 2> "$out/soak3m.err" &&
timeout -k 10 400 python -m beholder_amd bench soak --events 10000000 > "$out/soak10m.json" 2> "$out/soak10m.err"
