#!/usr/bin/env python3
"""Summary table of an interleaved native-budget A/B (scripts/box_r4_native_budget.sh output)."""
import glob
import json
import os
import statistics
import sys


def main(d):
    rows = {s: [] for s in "ABC" if glob.glob(os.path.join(d, f"{s}_*.json"))}
    for side in rows:
        for p in sorted(glob.glob(os.path.join(d, f"{side}_*.json")), key=lambda x: int(x.rsplit("_", 1)[1][:-5])):
            with open(p) as f:
                rows[side].append(json.loads(f.read()))
    for ph in ("tcp", "tls"):
        for k in ("eps", "p999", "warm_p99", "warm_p999", "cpu"):
            fmt = (lambda x: f"{x / 1e3:.0f}k") if k == "eps" else (lambda x: f"{x:.2f}" if k == "cpu" else f"{x / 1e3:.2f}")
            for j, (side, rs) in enumerate(rows.items()):
                v = [r[ph][k] for r in rs]
                label = f"{ph}_{k}" if j == 0 else ""
                print(f"{label:14s} {side} median {fmt(statistics.median(v)):>8s}  [{', '.join(fmt(x) for x in v)}]")
    print("(p999 / warm_* in ms; eps = events/s; cpu = us/event)")


if __name__ == "__main__":
    main(sys.argv[1])
