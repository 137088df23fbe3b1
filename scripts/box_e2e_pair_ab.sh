#!/bin/bash
# Interleaved A/B of tcp_e2e in fresh processes: this tree ("new") against ab_old/ (an older tree
# built in place, as scripts/box_r5_e2e_ab.sh describes). Each measurement: scripts/e2e_runs.py
# (the bench's unmeasured warm-up pass, then one 250k-event run). One JSON line per measurement
# in gpurun_out/$OUT/ab.jsonl. HEADLINE=1 adds the headline consumer alone per arm and pair.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-e2e_pair_ab}
mkdir -p "$out"
root=$PWD
probe='import asyncio, json
import bench
a = bench.parse(["--steps", "20", "--warmup", "5", "--no-extras"])
r = asyncio.run(bench.run_consumer(a, 0, lambda: None, None))
print(json.dumps({"eps": r["events"] / r["elapsed"], "cpu_us": r["cpu_s"] / r["events"] * 1e6}))'
for i in $(seq 1 "${RUNS:-8}"); do
  for arm in new old; do
    if [ "$arm" = old ]; then dir=$root/ab_old; else dir=$root; fi
    (cd "$dir" && PYTHONPATH=$dir timeout -k 10 120 python scripts/e2e_runs.py --repeats "${REPEATS:-2}" ${TLS:+--tls}) > "$out/tmp.jsonl" 2>> "$out/ab.err" || exit 1
    python - "$arm" "$i" "$out/tmp.jsonl" >> "$out/ab.jsonl" <<'PY'
import json, sys
for ln in open(sys.argv[3]):
    k, r = next(iter(json.loads(ln).items()))
    r.update(arm=sys.argv[1], pair=int(sys.argv[2]), cfg=k)
    print(json.dumps(r))
PY
    if [ -n "${HEADLINE:-}" ]; then  # and the headline consumer alone (bench.py run_consumer)
      (cd "$dir" && PYTHONPATH=$dir timeout -k 10 120 python -c "$probe") > "$out/tmp.json" 2>> "$out/ab.err" || exit 1
      python -c "import json; d=json.load(open('$out/tmp.json')); d.update(arm='$arm', cfg='headline', pair=$i); print(json.dumps(d))" >> "$out/ab.jsonl"
    fi
  done
  tail -n 6 "$out/ab.jsonl" | cut -c1-200
done
