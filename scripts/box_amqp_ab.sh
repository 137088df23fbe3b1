#!/bin/bash
# A/B of the amqp config: this tree against the round-1 tree copied to _ab_old/ (not committed).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-amqp_ab}
mkdir -p "$out"
for r in 1 2 3; do
  for v in old new; do
    d=$GRAFT_REPO_ROOT; [ $v = old ] && d=$GRAFT_REPO_ROOT/_ab_old
    (cd $d && timeout -k 10 120 python -c "
import json
from beholder_amd.bench import harness
r = harness.run_config('amqp', events=300000)
print(json.dumps({k: r.get(k) for k in ('ingest_rate_eps', 'cpu_us_per_event', 'acked')}))") > $out/amqp_${v}_r$r.json
  done
done
echo done
