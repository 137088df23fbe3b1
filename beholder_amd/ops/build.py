"""CLI: ``python -m beholder_amd.ops.build`` — build the native runtime in-tree (see :mod:`beholder_amd._build`)."""
from .._build import TARGET, build, main  # noqa: F401

if __name__ == "__main__":
    raise SystemExit(main())
