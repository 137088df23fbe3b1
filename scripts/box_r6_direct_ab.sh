#!/bin/bash
# Interleaved A/B of the paced production path (tcp_e2e at 1k/10k/100k events/s): this tree
# ("new", AMQP deliveries handed to the waiting consumer from the read callback) against ab_old/
# (the tree before it, built in place: git archive b1c3122^ beholder_amd bench.py scripts).
# One JSON line per rate and run in gpurun_out/$OUT/ab.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-direct_ab}
mkdir -p "$out"
root=$PWD
for i in $(seq 1 "${RUNS:-4}"); do
  for arm in new old; do
    if [ "$arm" = old ]; then dir=$root/ab_old; else dir=$root; fi
    (cd "$dir" && PYTHONPATH=$dir timeout -k 10 120 python "$root/scripts/paced_ab.py" ${TLS:+--tls}) > "$out/tmp.jsonl" 2>> "$out/ab.err" || exit 1
    python -c "
import json, sys
for ln in open('$out/tmp.jsonl'):
    r = json.loads(ln); r.update(arm='$arm', pair=$i, tls=bool('${TLS:-}')); print(json.dumps(r))" >> "$out/ab.jsonl" || exit 1
  done
  tail -n 6 "$out/ab.jsonl"
done
