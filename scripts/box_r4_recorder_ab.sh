#!/bin/bash
# Headline A/B (interleaved, one box): the compiled handlers calling the recorder's native core
# (A, native_record) against the recorder's Python coroutine (B, native_record = None).
set -o pipefail
out=gpurun_out/${OUT:-r4_recorder_ab}
mkdir -p "$out"
probe='import asyncio, json, sys
sys.path.insert(0, ".")
import bench
from beholder_amd.sinks import http as H
if sys.argv[1] == "B":
    init = H.RecordingHttpClient.__init__
    def no_fast(self, *a, **k):
        init(self, *a, **k)
        self.native_record = None
    H.RecordingHttpClient.__init__ = no_fast
a = bench.parse(["--steps", "20", "--warmup", "5", "--no-extras"])
r = asyncio.run(bench.run_consumer(a, 0, lambda: None, None))
print(json.dumps({"side": sys.argv[1], "eps": r["events"] / r["elapsed"], "cpu_us": r["cpu_s"] / r["events"] * 1e6}))'
for i in $(seq 1 "${RUNS:-5}"); do
  for side in A B; do
    timeout -k 10 120 python3 -c "$probe" $side >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit $?
  done
  tail -2 "$out/ab.jsonl"
done
