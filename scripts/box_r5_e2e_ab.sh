#!/bin/bash
# Interleaved A/B of the production-shaped path: this tree ("new") against
# ab_old/ (an older tree built in place: `git archive <rev> beholder_amd bench.py scripts | tar -x
# -C ab_old`, then `python -m beholder_amd._build --no-hip` inside it). Per pair and arm:
# tcp_e2e and tls_e2e (250k events, harness defaults) and the headline consumer alone.
# One JSON line per measurement in gpurun_out/$OUT/ab.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-r5_e2e_ab}
mkdir -p "$out"
root=$PWD
probe='import asyncio, json, sys
import bench
a = bench.parse(["--steps", "20", "--warmup", "5", "--no-extras"])
r = asyncio.run(bench.run_consumer(a, 0, lambda: None, None))
print(json.dumps({"eps": r["events"] / r["elapsed"], "cpu_us": r["cpu_s"] / r["events"] * 1e6}))'
for i in $(seq 1 "${RUNS:-5}"); do
  for arm in new old; do
    if [ "$arm" = old ]; then dir=$root/ab_old; else dir=$root; fi
    for cfg in tcp_e2e tls_e2e; do
      (cd "$dir" && PYTHONPATH=$dir timeout -k 10 150 python -m beholder_amd bench $cfg --events 250000) > "$out/tmp.json" 2>> "$out/ab.err" || exit 1
      python - "$arm" "$cfg" "$out/tmp.json" >> "$out/ab.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(json.dumps({"arm": sys.argv[1], "cfg": sys.argv[2], "eps": d["ingest_rate_eps"], "cpu_us": d["cpu_us_per_event"],
                  "sys_us": d.get("sys_cpu_us_per_event"), "p999_us": d["handle_latency_us"].get("p999"),
                  "warm_p999_us": d["warmup_handle_latency_us"].get("p999"), "fakes": d.get("fakes_cpu_us_per_event")}))
PY
    done
    (cd "$dir" && PYTHONPATH=$dir timeout -k 10 120 python -c "$probe") > "$out/tmp.json" 2>> "$out/ab.err" || exit 1
    python -c "import json,sys; d=json.load(open('$out/tmp.json')); d.update(arm='$arm', cfg='headline'); print(json.dumps(d))" >> "$out/ab.jsonl"
  done
  tail -6 "$out/ab.jsonl"
done
