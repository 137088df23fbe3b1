"""Minimal lint for environments without pyflakes: unused imports.

    python scripts/lint.py beholder_amd tests bench.py

An import is unused when its bound name never appears as a Name (load), as the base of
an attribute, in ``__all__``, or inside a string annotation. The check skips re-export
modules (``__init__.py``), lines marked ``# noqa`` and ``from __future__``. The exit
status is non-zero when anything is reported.
"""
from __future__ import annotations

import ast
import os
import sys
from typing import Iterator, List, Tuple


def _files(paths: List[str]) -> Iterator[str]:
    for p in paths:
        if os.path.isdir(p):
            for root, dirs, files in os.walk(p):
                dirs[:] = [d for d in dirs if d not in ("__pycache__", ".git", "gpurun_out")]
                for f in sorted(files):
                    if f.endswith(".py"):
                        yield os.path.join(root, f)
        elif p.endswith(".py"):
            yield p


def check(path: str) -> List[Tuple[int, str]]:
    src = open(path, encoding="utf-8").read()
    tree = ast.parse(src, path)
    lines = src.splitlines()
    imported = {}  # name -> lineno
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            if "noqa" in lines[node.lineno - 1]:
                continue
            for a in node.names:
                if a.name == "*":
                    continue
                name = a.asname or a.name.split(".")[0]
                imported.setdefault(name, node.lineno)
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Constant) and isinstance(node.value, str):
            # string annotations / __all__ entries
            for tok in node.value.replace("[", " ").replace("]", " ").replace(",", " ").replace(".", " ").split():
                used.add(tok.strip("\"'"))
    problems = [(ln, f"'{name}' imported but unused") for name, ln in imported.items() if name not in used]
    return sorted(problems)


def main(argv: List[str]) -> int:
    bad = 0
    for f in _files(argv or ["beholder_amd", "tests", "bench.py"]):
        if os.path.basename(f) == "__init__.py":
            continue
        for ln, msg in check(f):
            print(f"{f}:{ln}: {msg}")
            bad += 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
