#!/usr/bin/env python3
"""Summary of an interleaved production-path A/B (scripts/box_r5_e2e_ab.sh: ab.jsonl)."""
import json
import statistics
import sys


def main(path: str) -> int:
    rows = [json.loads(x) for x in open(path) if x.strip()]
    for cfg in ("tcp_e2e", "tls_e2e", "headline"):
        for key, fmt in (("eps", lambda v: f"{v / 1e3:.1f}k"), ("cpu_us", lambda v: f"{v:.3f}"),
                         ("sys_us", lambda v: f"{v:.3f}"), ("p999_us", lambda v: f"{v / 1e3:.2f}ms"),
                         ("warm_p999_us", lambda v: f"{v / 1e3:.2f}ms")):
            for arm in ("new", "old"):
                v = [r[key] for r in rows if r["cfg"] == cfg and r["arm"] == arm and r.get(key) is not None]
                if not v:
                    continue
                print(f"{cfg:9s} {key:13s} {arm:3s} median {fmt(statistics.median(v)):>9s}  "
                      f"[{', '.join(fmt(x) for x in v)}]")
    return 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1]))
