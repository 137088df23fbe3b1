"""Transparent huge pages for the interpreter's heap (a process-start setting).

A consumer process touches a few hundred MB of small Python objects (deliveries, decoded
messages, strings) scattered over its heap; with 4 KiB pages that is a TLB miss on most of them.
The MI355X hosts run THP in ``madvise`` mode, so only memory that asks for huge pages gets them,
and CPython's own small-object allocator (pymalloc) hands out 256 KiB arenas that never could.
``PYTHONMALLOC=malloc`` routes those objects through glibc malloc, and glibc 2.35's
``glibc.malloc.hugetlb=1`` tunable makes malloc ``madvise(MADV_HUGEPAGE)`` its heap.

Measured on the box (``profiles/box_r4_alloc_ab/``, headline only, interleaved): the default
heap gave 779-1,183k events/s, slow in the box's first minute; with both settings 1,071-1,153k
from the first run on, with 5-9 page faults in the timed steps instead of 55-72.

Both are read when the interpreter starts. The production image sets them (``Dockerfile``);
``bench.py`` re-executes itself with them before anything touches the GPU (:func:`reexec_with_hugepage_heap`).
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional

HEAP_ENV = {"PYTHONMALLOC": "malloc", "GLIBC_TUNABLES": "glibc.malloc.hugetlb=1"}
_GUARD = "BEHOLDER_HEAP_REEXEC"


def thp_mode() -> Optional[str]:
    try:
        with open("/sys/kernel/mm/transparent_hugepage/enabled") as f:
            t = f.read()
        return t[t.index("[") + 1:t.index("]")]
    except (OSError, ValueError):
        return None


def heap_tuned(env=None) -> bool:
    env = os.environ if env is None else env
    return env.get("PYTHONMALLOC") == "malloc" and "glibc.malloc.hugetlb=1" in env.get("GLIBC_TUNABLES", "")


def reexec_with_hugepage_heap(argv: List[str]) -> None:
    """Replace this process with the same command under :data:`HEAP_ENV`, once, when THP can
    back the heap (mode ``always`` or ``madvise``) and the settings are not in effect yet.
    Call it first thing: before torch is imported or any GPU call (a process that has
    initialised the GPU must never exec). ``BEHOLDER_HEAP_REEXEC=0`` opts out. Returns (doing
    nothing) when the settings are in effect, not applicable, or the exec is refused."""
    if heap_tuned() or os.environ.get(_GUARD) is not None or thp_mode() not in ("always", "madvise"):
        return
    if "torch" in sys.modules:  # too late to be sure nothing touched the GPU
        return
    env = dict(os.environ)
    env[_GUARD] = "1"
    env["PYTHONMALLOC"] = HEAP_ENV["PYTHONMALLOC"]
    tun = env.get("GLIBC_TUNABLES")
    env["GLIBC_TUNABLES"] = f"{tun}:{HEAP_ENV['GLIBC_TUNABLES']}" if tun else HEAP_ENV["GLIBC_TUNABLES"]
    sys.stdout.flush()
    sys.stderr.flush()
    try:
        os.execve(sys.executable, [sys.executable, *argv], env)
    except OSError:
        return  # refused: run on the default heap
