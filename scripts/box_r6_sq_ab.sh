#!/bin/bash
# Interleaved A/B of the shared-queue phase (run --workers N on one queue, N = 1, 2, 4, 8): this
# tree ("new") against ab_old/ (an older tree built in place). One JSON line per run and N in
# gpurun_out/$OUT/ab.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-sq_ab}
mkdir -p "$out"
root=$PWD
for i in $(seq 1 "${RUNS:-3}"); do
  for arm in new old; do
    if [ "$arm" = old ]; then dir=$root/ab_old; else dir=$root; fi
    (cd "$dir" && PYTHONPATH=$dir timeout -k 10 240 python -m beholder_amd.bench.shared_queue --workers "${NS:-1,2,4,8}") > "$out/tmp.jsonl" 2>> "$out/ab.err" || exit 1
    python -c "
import json
for ln in open('$out/tmp.jsonl'):
    try:
        r = json.loads(ln)
    except ValueError:
        continue
    print(json.dumps({'arm': '$arm', 'pair': $i, 'workers': r.get('workers'), 'eps': r.get('events_per_sec'),
                      'exactly_once': r.get('exactly_once'), 'per_worker': r.get('per_worker_delivered')}))" >> "$out/ab.jsonl" || exit 1
  done
  tail -n 8 "$out/ab.jsonl" | cut -c1-160
done
