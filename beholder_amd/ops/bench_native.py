"""Loader of ``_native_bench``: the bench, test and diagnostic natives, kept out of the service's
extension. The runtime image does not build or ship it (Dockerfile
``--no-bench``); the service never imports this module.

Exports ``Recorder`` (the in-process sink stub's core, sinks/http.py RecordingHttpClient),
``paced_write`` (the paced producer of BASELINE configs 2-4), ``calib`` / ``calib_mem`` (the bench
line's fixed-work calibrations) and ``prof_start`` / ``prof_stop`` (the SIGPROF sampler of
scripts/cprof.py), ``SharedBroker`` (the shared-queue bench's broker fake) and ``PgFake`` (the e2e
bench's Postgres fake). Like :mod:`beholder_amd.ops`, a missing or stale module is built on import
when a compiler is there (``BEHOLDER_ALLOW_BUILD=0`` forbids it), and the import fails loudly otherwise.
"""
from __future__ import annotations

import importlib
import os
import subprocess

from . import native as _service_native  # noqa: F401  (_native first: this module imports its _C_API)


def _load():
    from .. import _build
    if os.environ.get("BEHOLDER_ALLOW_BUILD", "1") != "0":
        try:
            _build.build_bench()
        except (OSError, subprocess.CalledProcessError) as e:
            if not os.path.exists(_build.BENCH_TARGET):
                raise ImportError(f"cannot build the beholder bench natives: {e}") from e
    try:
        return importlib.import_module("beholder_amd.ops._native_bench")
    except ImportError as first:
        raise ImportError("beholder bench natives are not built; run `python -m beholder_amd.ops.build`") from first


native_bench = _load()

Recorder = native_bench.Recorder
paced_write = native_bench.paced_write
calib = native_bench.calib
calib_mem = native_bench.calib_mem
prof_start = native_bench.prof_start
prof_stop = native_bench.prof_stop
SharedBroker = native_bench.SharedBroker
PgFake = native_bench.PgFake

__all__ = ["native_bench", "Recorder", "paced_write", "calib", "calib_mem", "prof_start", "prof_stop", "SharedBroker",
           "PgFake"]
