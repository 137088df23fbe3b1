#!/usr/bin/env python3
"""Does thread placement move the single-process headline? Interleaved A/B, one child per run.

The headline consumer is three threads: the pump writing each step into a pipe, the native
reader thread (pipe -> framer -> ring) and the event loop (ring -> handlers). Two runs with the
same calibrations can differ by 25% in CPU per event (``profiles/box_r4_fresh3/``), which points
at where those threads land on a 256-thread, 16-L3 host. Arms (the child sets its mask before it
starts any thread; threads inherit it):

* ``none``  - the inherited mask (what ``bench.py`` does);
* ``l3``    - 4 CPUs on distinct cores of one L3 domain (the least busy one right now);
* ``cross`` - 2 CPUs on distinct cores of each of two L3 domains.

    python scripts/pin_ab.py [--rounds 6] [--steps 20]        # prints one JSON line per run
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _read(path: str) -> str:
    with open(path) as f:
        return f.read().strip()


def l3_domains(allowed) -> list:
    """Allowed CPUs grouped by shared L3, one CPU per physical core in each group."""
    groups: dict = {}
    for c in sorted(allowed):
        base = f"/sys/devices/system/cpu/cpu{c}"
        l3 = None
        for idx in range(8):
            d = f"{base}/cache/index{idx}"
            try:
                if _read(f"{d}/level") == "3":
                    l3 = _read(f"{d}/shared_cpu_list")
                    break
            except OSError:
                break
        try:
            core = _read(f"{base}/topology/thread_siblings_list")
        except OSError:
            core = str(c)
        g = groups.setdefault(l3 or "?", {})
        g.setdefault(core, c)  # first allowed CPU of each core
    return [sorted(g.values()) for g in groups.values()]


def cpu_idle(cpus, dt: float = 0.2) -> dict:
    def snap():
        out = {}
        with open("/proc/stat") as f:
            for ln in f:
                p = ln.split()
                if p[0].startswith("cpu") and p[0] != "cpu":
                    v = [int(x) for x in p[1:9]]
                    out[int(p[0][3:])] = (v[3] + v[4], sum(v))
        return out
    a = snap()
    time.sleep(dt)
    b = snap()
    return {c: (b[c][0] - a[c][0]) / max(1, b[c][1] - a[c][1]) for c in cpus if c in a and c in b}


def pick(arm: str) -> list:
    allowed = os.sched_getaffinity(0)
    if arm == "none":
        return sorted(allowed)
    doms = [d for d in l3_domains(allowed) if len(d) >= 4]
    idle = cpu_idle(allowed)
    doms.sort(key=lambda d: -sum(sorted((idle.get(c, 0) for c in d), reverse=True)[:4]))
    if arm == "l3":
        d = doms[0]
        return sorted(sorted(d, key=lambda c: -idle.get(c, 0))[:4])
    if len(doms) < 2:
        raise SystemExit("cross: fewer than two L3 domains with 4 cores in the mask")
    a, b = doms[0], doms[1]
    return sorted(sorted(a, key=lambda c: -idle.get(c, 0))[:2] + sorted(b, key=lambda c: -idle.get(c, 0))[:2])


def child(arm: str, cpus: list, steps: int) -> None:
    os.sched_setaffinity(0, cpus)
    import asyncio

    import bench
    a = bench.parse(["--steps", str(steps), "--warmup", "5", "--no-extras"])
    r = asyncio.run(bench.run_consumer(a, 0, lambda: None))
    print(json.dumps({"arm": arm, "cpus": cpus, "events_per_sec": round(r["events"] / r["elapsed"], 1),
                      "cpu_us_per_event": round(r["cpu_s"] / r["events"] * 1e6, 3), "nivcsw": r["nivcsw"]}),
          flush=True)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--arms", default="none,l3,cross")
    ap.add_argument("--child", default=None)
    ap.add_argument("--cpus", default=None)
    a = ap.parse_args(argv)
    if a.child:
        child(a.child, [int(x) for x in a.cpus.split(",")], a.steps)
        return 0
    arms = a.arms.split(",")
    print(json.dumps({"l3_domains": l3_domains(os.sched_getaffinity(0))[:16]}), flush=True)
    for i in range(a.rounds):
        for arm in (arms if i % 2 == 0 else arms[::-1]):
            cpus = pick(arm)
            r = subprocess.run([sys.executable, __file__, "--child", arm, "--cpus", ",".join(map(str, cpus)),
                                "--steps", str(a.steps)], capture_output=True, text=True, timeout=300)
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else json.dumps(
                {"arm": arm, "rc": r.returncode, "err": r.stderr[-500:]})
            print(line, flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
