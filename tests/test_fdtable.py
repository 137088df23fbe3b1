"""utils/fdtable.py: the startup descriptor-table grow leaves every open descriptor alone."""
import os
import resource

from beholder_amd.utils import fdtable


def _fresh(monkeypatch):
    monkeypatch.setattr(fdtable, "_reserved", 0)


def test_reserve_returns_size_and_keeps_low_numbers(monkeypatch):
    _fresh(monkeypatch)
    soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = min(512, soft)
    assert fdtable.reserve_fd_table(want) == want
    r, w = os.pipe()  # new descriptors still take the lowest free numbers
    try:
        assert r < 256 and w < 256
    finally:
        os.close(r)
        os.close(w)
    assert fdtable.reserve_fd_table(want) == want  # once grown: a no-op


def test_reserve_does_not_touch_an_open_descriptor_at_the_target(monkeypatch):
    _fresh(monkeypatch)
    soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
    n = min(300, soft)
    r, w = os.pipe()
    os.dup2(w, n - 1)  # something already lives at the number the grow aims at
    try:
        assert fdtable.reserve_fd_table(n) == n
        os.write(n - 1, b"x")  # still open, still the pipe
        assert os.read(r, 1) == b"x"
    finally:
        os.close(n - 1)
        os.close(r)
        os.close(w)


def test_reserve_is_capped_by_the_soft_limit(monkeypatch):
    _fresh(monkeypatch)
    soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
    got = fdtable.reserve_fd_table(soft * 4 if soft != resource.RLIM_INFINITY else 1 << 20)
    assert got in (0, soft) or soft == resource.RLIM_INFINITY
