#!/bin/bash
# Heap-setting A/B across the headline and the production-shaped path, interleaved:
#   pymalloc (default) | malloc+hugetlb | malloc+hugetlb with a fixed mmap threshold and no trim.
set -o pipefail
out=gpurun_out/${OUT:-r4_heap_ab}
mkdir -p "$out"
probe='import asyncio, json, sys
sys.path.insert(0, ".")
import bench
from beholder_amd.bench import harness
a = bench.parse(["--steps", "20", "--warmup", "5", "--no-extras"])
r = asyncio.run(bench.run_consumer(a, 0, lambda: None, None))
out = {"variant": sys.argv[1], "headline": r["events"] / r["elapsed"], "headline_cpu": r["cpu_s"] / r["events"] * 1e6}
for name, kw in (("tcp", {}), ("tls", {"http_servers": 4, "tls": True})):
    x = harness._tcp_e2e(50000, **kw)
    out[name] = {"eps": round(x["ingest_rate_eps"]), "p999": x["handle_latency_us"].get("p999"),
                 "warm_p999": x["warmup_handle_latency_us"].get("p999"), "cpu": round(x["cpu_us_per_event"], 3),
                 "blamed": (x.get("attribution_steady") or {}).get("blamed")}
print(json.dumps(out))'
for i in $(seq 1 "${RUNS:-3}"); do
  for v in pymalloc huge huge_fixed; do
    case $v in
      pymalloc) env=(BEHOLDER_HEAP_REEXEC=0) ;;
      huge) env=(PYTHONMALLOC=malloc GLIBC_TUNABLES=glibc.malloc.hugetlb=1) ;;
      huge_fixed) env=(PYTHONMALLOC=malloc GLIBC_TUNABLES=glibc.malloc.hugetlb=1:glibc.malloc.mmap_threshold=33554432:glibc.malloc.trim_threshold=1073741824) ;;
    esac
    env "${env[@]}" timeout -k 10 200 python3 -c "$probe" $v >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit $?
    tail -1 "$out/ab.jsonl" | cut -c1-230
  done
done
