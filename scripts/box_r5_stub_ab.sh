#!/bin/bash
# Headline A/B (interleaved, one box) of the in-process sink stub:
#   h1   each request's bytes built by the H1 client's builder, a canned 200 parsed by H1Parser
#        into the H1 client's HttpResponse (the default from round 5)
#   url  round 4's stub: URL + query built and logged, one shared response
# Output: $out/ab.jsonl, one line per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${OUT:-r5_stub_ab}
mkdir -p "$out"
probe='import asyncio, json, os, sys
sys.path.insert(0, ".")
import bench
a = bench.parse(["--steps", "20", "--warmup", "5", "--no-extras"])
r = asyncio.run(bench.run_consumer(a, 0, lambda: None, None))
print(json.dumps({"side": os.environ["BEHOLDER_BENCH_STUB"], "eps": r["events"] / r["elapsed"],
                  "cpu_us": r["cpu_s"] / r["events"] * 1e6, "http_calls": r["http_calls"]}))'
for i in $(seq 1 "${RUNS:-6}"); do
  for side in url h1; do
    BEHOLDER_BENCH_STUB=$side timeout -k 10 120 python3 -c "$probe" >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit $?
  done
  tail -2 "$out/ab.jsonl"
done
