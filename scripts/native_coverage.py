"""Line and branch coverage of the native runtime (``ops/csrc``) under the CPU test suite.

Builds ``_native`` and ``_native_bench`` with gcov instrumentation (``ops.build --coverage``: -O0,
objects, ``.gcno`` and ``.gcda`` kept under ``build/coverage/``), runs ``pytest -m "not gpu"``
against that build (``BEHOLDER_ALLOW_BUILD=0``: nothing rebuilds it underneath), then asks
``gcov`` for each source's line, branch and function counts and writes

* ``<out>/summary.txt``  per source (headers merged over every unit that includes them): lines,
  branches taken, functions called; the functions and the lines never executed;
* ``<out>/summary.json`` the same numbers.

Afterwards the optimised build is restored (``ops.build --force``).

    python scripts/native_coverage.py [--out profiles/native_coverage] [--jobs 6] [-- pytest args]

``make coverage`` runs it. Host code only; no GPU is involved.
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from beholder_amd import _build  # noqa: E402

# tests that rebuild the in-tree extension with the default flags (they would replace the
# instrumented one mid-run) or only drive copies of the tree
SKIP = ("tests/test_packaging.py", "tests/test_oracle_mutations.py")


def run_tests(jobs: int, extra: list) -> int:
    env = dict(os.environ, BEHOLDER_ALLOW_BUILD="0")
    cmd = [sys.executable, "-m", "pytest", "tests", "-q", "-p", "no:cacheprovider", "-m", "not gpu"]
    cmd += [f"--ignore={p}" for p in SKIP]
    if jobs > 1:
        cmd += ["-n", str(jobs)]
    cmd += extra
    print(" ".join(cmd), flush=True)
    return subprocess.run(cmd, cwd=ROOT, env=env).returncode


def gcov_json(src: str, objdir: str, workdir: str) -> dict:
    """gcov's JSON intermediate format for one translation unit."""
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    subprocess.run(["gcov", "-j", "-b", "-o", obj, src], cwd=workdir, capture_output=True, text=True, check=True)
    path = os.path.join(workdir, os.path.splitext(os.path.basename(src))[0] + ".gcov.json.gz")
    with gzip.open(path) as f:
        data = json.load(f)
    os.unlink(path)
    return data


def collect() -> dict:
    """Per project source (translation units and the headers they include, merged over every
    unit): executed lines, branches taken, and the functions defined there with their calls."""
    files: dict = {}
    ours = (os.path.abspath(_build.CSRC), os.path.abspath(_build.CSRC_BENCH))
    work = os.path.join(_build.COVERAGE_DIR, "gcov-work")
    os.makedirs(work, exist_ok=True)
    for target, csrc in ((_build.TARGET, _build.CSRC), (_build.BENCH_TARGET, _build.CSRC_BENCH)):
        objdir = _build.coverage_objdir(target)
        for src in _build.sources(csrc):
            for f in gcov_json(src, objdir, work)["files"]:
                path = os.path.abspath(f["file"])
                if not path.startswith(ours):
                    continue
                rel = os.path.relpath(path, ROOT)
                e = files.setdefault(rel, {"lines": {}, "branches": {}, "functions": {}})
                for ln in f["lines"]:
                    n = ln["line_number"]
                    e["lines"][n] = e["lines"].get(n, 0) + ln["count"]
                    br = [b["count"] for b in ln["branches"]]
                    if br:
                        old = e["branches"].get(n)
                        e["branches"][n] = br if old is None or len(old) != len(br) else [a + b for a, b in zip(old, br)]
                for fn in f["functions"]:
                    key = (fn["start_line"], fn["demangled_name"])
                    e["functions"][key] = e["functions"].get(key, 0) + fn["execution_count"]
    return files


def _ranges(nums: list) -> str:
    out, i = [], 0
    while i < len(nums):
        j = i
        while j + 1 < len(nums) and nums[j + 1] == nums[j] + 1:
            j += 1
        out.append(str(nums[i]) if i == j else f"{nums[i]}-{nums[j]}")
        i = j + 1
    return ",".join(out)


def report(files: dict) -> dict:
    res = {}
    for rel, e in sorted(files.items()):
        lines = e["lines"]
        hit = sum(1 for c in lines.values() if c)
        br = [c for v in e["branches"].values() for c in v]
        unc_fn = sorted((ln, name) for (ln, name), c in e["functions"].items() if not c)
        res[rel] = {
            "lines": [round(100.0 * hit / max(len(lines), 1), 1), len(lines)],
            "branches_taken": [round(100.0 * sum(1 for c in br if c) / max(len(br), 1), 1), len(br)],
            "functions": [len(e["functions"]) - len(unc_fn), len(e["functions"])],
            "uncovered_functions": [f"{ln}: {name}" for ln, name in unc_fn],
            "uncovered_lines": _ranges(sorted(n for n, c in lines.items() if not c)),
        }
    return res


def write_summary(res: dict, out: str, rc: int) -> None:
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump({"pytest_rc": rc, "files": res}, f, indent=1, sort_keys=True)
    rows = []
    tl = tn = tb = tbn = 0.0
    for rel, s in sorted(res.items()):
        lp, ln = s["lines"]
        bp, bn = s["branches_taken"]
        tl += lp * ln / 100
        tn += ln
        tb += bp * bn / 100
        tbn += bn
        rows.append(f"{rel:48s} {lp:6.1f}% of {ln:5d}   {bp:6.1f}% of {bn:5d}   "
                    f"{s['functions'][0]:3d}/{s['functions'][1]:3d}")
    head = (f"native coverage under pytest -m 'not gpu' (gcov {_gcov_version()}, -O0; pytest rc {rc})\n"
            f"{'source':48s} {'lines':>15s}   {'branches taken':>15s}   functions\n")
    total = (f"{'TOTAL':48s} {100 * tl / max(tn, 1):6.1f}% of {int(tn):5d}   "
             f"{100 * tb / max(tbn, 1):6.1f}% of {int(tbn):5d}\n")
    unc = ["", "functions with no executed line:"]
    for rel, s in sorted(res.items()):
        for name in s["uncovered_functions"]:
            unc.append(f"  {rel}:{name}")
    unl = ["", "lines not executed:"] + [f"  {rel}: {s['uncovered_lines']}" for rel, s in sorted(res.items())]
    with open(os.path.join(out, "summary.txt"), "w") as f:
        f.write(head + "\n".join(rows) + "\n" + total + "\n".join(unc) + "\n" + "\n".join(unl) + "\n")
    print(head + "\n".join(rows) + "\n" + total + "\n".join(unc))


def _gcov_version() -> str:
    r = subprocess.run(["gcov", "--version"], capture_output=True, text=True)
    return r.stdout.split("\n")[0].split()[-1] if r.returncode == 0 else "?"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "native_coverage"))
    ap.add_argument("--jobs", type=int, default=6)
    ap.add_argument("--report-only", action="store_true", help="gcov over the counts already collected")
    ap.add_argument("pytest_args", nargs="*")
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    rc = 0
    if not a.report_only:
        _build.build(force=True, coverage=True)
        _build.build_bench(force=True, coverage=True)
        try:
            rc = run_tests(a.jobs, a.pytest_args)
        finally:
            write_summary(report(collect()), a.out, rc)
            _build.build(force=True)
            _build.build_bench(force=True)
    else:
        write_summary(report(collect()), a.out, rc)
    return rc


if __name__ == "__main__":
    raise SystemExit(main())
