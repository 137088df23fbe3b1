#!/usr/bin/env python3
"""Native-level flat CPU profile of the headline consumer (no `perf` on these hosts).

Samples instruction pointers with the bench extension's SIGPROF sampler (``ops/csrc_bench/prof.cpp``)
while one consumer runs the bench's timed steps (``bench.run_consumer``), then resolves every
sample to ``object:function`` through ``/proc/self/maps``, the objects' ELF load segments and
their symbol tables (``nm``: our extension's full table, the interpreter's exported symbols).
Prints the top functions by self samples, and the split by object.

    python scripts/cprof.py [--steps 20] [--hz 2000] [--top 60] [--tid main|all]
    python scripts/cprof.py --workload tcp_e2e|tls_e2e [--events 200000] [--rate 10000]   # the production-shaped path
    python scripts/cprof.py ... --depth 24 [--focus send,recv]   # + inclusive cost and callers
"""
from __future__ import annotations

import argparse
import asyncio
import bisect
import collections
import os
import subprocess
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def maps():
    out = []
    with open("/proc/self/maps") as f:
        for ln in f:
            parts = ln.split()
            if len(parts) < 6 or "x" not in parts[1]:
                continue
            a, b = (int(x, 16) for x in parts[0].split("-"))
            out.append((a, b, int(parts[2], 16), parts[5]))
    out.sort()
    return out


_segs_cache: dict = {}
_syms_cache: dict = {}


def load_segments(path):
    """[(p_offset, p_vaddr, p_filesz)] of the LOAD segments."""
    if path in _segs_cache:
        return _segs_cache[path]
    segs = []
    try:
        txt = subprocess.run(["readelf", "-lW", path], capture_output=True, text=True, timeout=30).stdout
        for ln in txt.splitlines():
            p = ln.split()
            if p and p[0] == "LOAD":
                segs.append((int(p[1], 16), int(p[2], 16), int(p[4], 16)))
    except (OSError, subprocess.SubprocessError):
        pass
    _segs_cache[path] = segs
    return segs


def symbols(path):
    """Sorted (vaddr, name) of the function symbols (static table, else dynamic)."""
    if path in _syms_cache:
        return _syms_cache[path]
    syms = []
    for args in (["nm", "-n", "--defined-only", "-C", path], ["nm", "-D", "-n", "--defined-only", "-C", path]):
        try:
            txt = subprocess.run(args, capture_output=True, text=True, timeout=60).stdout
        except (OSError, subprocess.SubprocessError):
            continue
        for ln in txt.splitlines():
            p = ln.split(" ", 2)
            if len(p) == 3 and p[1] in "tTwWiI":
                syms.append((int(p[0], 16), p[2]))
        if syms:
            break
    syms.sort()
    _syms_cache[path] = (syms, [a for a, _ in syms])
    return _syms_cache[path]


def resolve(ip, mp, starts):
    i = bisect.bisect_right(starts, ip) - 1
    if i < 0 or ip >= mp[i][1]:
        return ("?", "?")
    a, _, off, path = mp[i]
    foff = ip - a + off
    vaddr = foff
    for so, sv, sz in load_segments(path):
        if so <= foff < so + sz:
            vaddr = foff - so + sv
            break
    syms, addrs = symbols(path)
    j = bisect.bisect_right(addrs, vaddr) - 1
    name = syms[j][1] if j >= 0 else f"+{vaddr:#x}"
    return (os.path.basename(path), name)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--hz", type=int, default=2000)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--tid", default="main", choices=["main", "all"])
    ap.add_argument("--workload", default="headline", choices=["headline", "tcp_e2e", "tls_e2e"])
    ap.add_argument("--events", type=int, default=200_000, help="tcp_e2e / tls_e2e events")
    ap.add_argument("--rate", type=float, default=0.0,
                    help="tcp_e2e / tls_e2e: the broker paces its sends at this many events/s (0 = saturation)")
    ap.add_argument("--depth", type=int, default=0,
                    help="also unwind this many frames per sample: inclusive cost per function and each "
                         "top leaf's callers")
    ap.add_argument("--focus", default="",
                    help="with --depth: comma-separated substrings of leaf functions whose callers are listed "
                         "(default: the top 8 leaves)")
    a = ap.parse_args(argv)
    import bench
    from beholder_amd.ops import bench_native as native

    ba = bench.parse(["--steps", str(a.steps), "--warmup", str(a.warmup), "--no-extras"])
    main_tid = threading.get_native_id()

    def go():
        native.prof_start(a.hz, a.depth)

    def stop():
        res["samples"], res["lost"] = native.prof_stop()

    res: dict = {}
    if a.workload == "headline":
        r = asyncio.run(bench.run_consumer(ba, 0, go, stop))
    else:
        from beholder_amd.bench import harness
        tls = a.workload == "tls_e2e"
        x = harness._tcp_e2e(a.events, http_servers=4 if tls else 2, tls=tls, hooks=(go, stop), rate=a.rate)
        r = {"events": x["measured_events"], "elapsed": x["elapsed_s"],
             "cpu_s": x["cpu_us_per_event"] * x["measured_events"] / 1e6}
    mp = maps()
    starts = [m[0] for m in mp]
    samples = res["samples"]
    if a.tid == "main":
        samples = [s for s in samples if s[1] == main_tid]
    fn = collections.Counter()
    obj = collections.Counter()
    incl = collections.Counter()
    callers = collections.defaultdict(collections.Counter)
    for smp in samples:
        ip = smp[0]
        o, f = resolve(ip, mp, starts)
        fn[(o, f)] += 1
        obj[o] += 1
        if len(smp) > 2:
            # return addresses: the call instruction is just before each one
            frames = [(o, f)] + [resolve(r - 1, mp, starts) for r in smp[2][1:]]
            for x in set(frames):
                incl[x] += 1
            chain = " <- ".join(g for _, g in frames[1:4])
            callers[(o, f)][chain] += 1
    n = max(1, len(samples))
    print(f"events/s {r['events'] / r['elapsed']:.0f}  cpu us/event {r['cpu_s'] / r['events'] * 1e6:.3f}  "
          f"samples {len(samples)} ({a.tid} thread), lost {res['lost']}")
    print("\n-- by object --")
    for o, c in obj.most_common():
        print(f"{100 * c / n:6.2f}%  {o}")
    print("\n-- by function (self) --")
    for (o, f), c in fn.most_common(a.top):
        print(f"{100 * c / n:6.2f}%  {o:28s} {f}")
    if incl:
        print("\n-- by function (inclusive: on the stack) --")
        for (o, f), c in incl.most_common(a.top):
            print(f"{100 * c / n:6.2f}%  {o:28s} {f}")
        focus = [x for x in a.focus.split(",") if x]
        leaves = [k for k, _ in fn.most_common(8)] if not focus else \
            [k for k in fn if any(x in k[1] for x in focus)]
        for k in leaves:
            print(f"\n-- callers of {k[1]} ({100 * fn[k] / n:.2f}% self) --")
            for chain, c in callers[k].most_common(8):
                print(f"{100 * c / n:6.2f}%  {chain}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
