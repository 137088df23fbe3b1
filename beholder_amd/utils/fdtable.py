"""Grow the process's file-descriptor table at startup, not in the middle of a connect burst.

Linux sizes a process's descriptor table on demand: when a new descriptor number passes the
table's size, ``socket(2)`` / ``accept(2)`` / ``dup(2)`` doubles it. In a process with more than
one thread (this service always has some: the native reader, the TLS handshake threads) that
grow waits for an RCU grace period before it frees the old table, while the calling thread is
blocked. On the MI355X box (256 hardware threads, other tenants) one such wait took
**140–160 ms**. It hit the loop thread in the ``socket()`` of a sink connect, during the first
burst of HTTPS connects: every delivery in flight waited behind it. The profile is in
``profiles/box_r3_fdtable/summary.txt`` (``scripts/diag_warmup.py``, measured per call).

The table never shrinks, so growing it once at startup, before the first delivery, removes the
stall for the life of the process: one ``F_DUPFD`` to a high descriptor number, then close.
``F_DUPFD`` takes the lowest free number at or above the target, so no open descriptor is
touched.
"""
from __future__ import annotations

import fcntl
import os
import resource

_reserved = 0


def reserve_fd_table(n: int = 1024) -> int:
    """Make the descriptor table hold at least ``n`` descriptors (capped by the soft
    ``RLIMIT_NOFILE``). Returns the size now reserved; 0 if it could not. Cheap when the table
    is already that large."""
    global _reserved
    try:
        soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
    except (OSError, ValueError):
        return 0
    if soft != resource.RLIM_INFINITY:
        n = min(n, soft)
    if n <= _reserved:
        return _reserved
    if n < 8:
        return 0
    r, w = os.pipe()
    try:
        high = fcntl.fcntl(r, getattr(fcntl, "F_DUPFD_CLOEXEC", fcntl.F_DUPFD), n - 1)
        os.close(high)
    except OSError:  # every number from n-1 up is taken (or the limit is lower than it says)
        return 0
    finally:
        os.close(r)
        os.close(w)
    _reserved = n
    return n
