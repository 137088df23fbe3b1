"""The event path's clock (ops/csrc/gil_clock.hpp): CLOCK_MONOTONIC / CLOCK_REALTIME extrapolated
from the TSC between anchors where the kernel's clocksource is the TSC. Every value must sit
between two time.monotonic_ns() reads around it (within a tolerance for a preempted test
process), never go backwards, stay right across idle gaps longer than an anchor interval, and
give Date.now()-compatible milliseconds for log lines; BEHOLDER_TSC_CLOCK=0 turns it off."""
import os
import time

import pytest

from beholder_amd.ops import _native as m

TOL_NS = 2000  # a preempted read on a loaded CI host


@pytest.fixture
def clock(monkeypatch):
    m.gil_clock_reset()
    yield m
    monkeypatch.delenv("BEHOLDER_TSC_CLOCK", raising=False)
    m.gil_clock_reset()


def _check(n):
    prev = 0
    bad = 0
    for _ in range(n):
        t0 = time.monotonic_ns()
        g, _ = m.gil_clock()
        t1 = time.monotonic_ns()
        assert g >= prev
        prev = g
        if not (t0 - TOL_NS <= g <= t1 + TOL_NS):
            bad += 1
    return bad


def test_values_sit_between_monotonic_reads(clock):
    # the first reads calibrate (1 ms of baseline); the rest are extrapolated
    assert _check(200_000) == 0
    info = m.gil_clock_info()
    with open("/sys/devices/system/clocksource/clocksource0/current_clocksource") as f:
        tsc = f.read().strip() == "tsc"
    assert info["mode"] == ("tsc" if tsc else "clock_gettime")
    if tsc:
        assert info["ns_per_tick"] > 0 and info["anchors"] >= 2


def test_idle_gaps_longer_than_an_anchor(clock):
    _check(20_000)
    for gap in (0.0003, 0.002, 0.02):
        time.sleep(gap)
        assert _check(2_000) == 0


def test_wall_ms_matches_time_time(clock):
    for _ in range(2_000):
        a = time.time_ns() // 1_000_000
        _, w = m.gil_clock()
        b = time.time_ns() // 1_000_000
        assert a - 1 <= w <= b + 1


def test_env_turns_it_off(clock, monkeypatch):
    monkeypatch.setenv("BEHOLDER_TSC_CLOCK", "0")
    m.gil_clock_reset()
    assert m.gil_clock_info()["mode"] == "clock_gettime"
    assert _check(5_000) == 0


def test_builds_without_a_tsc():
    """Off x86: no <x86intrin.h>, no rdtsc, mode 0 only. BEHOLDER_NO_TSC takes the
    path other architectures take; the clock's translation unit must compile on it."""
    import shutil
    import subprocess
    import sysconfig

    from beholder_amd import _build
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no C++ compiler")
    src = os.path.join(_build.CSRC, "gil_clock.cpp")
    r = subprocess.run([cxx, "-std=c++17", "-fsyntax-only", "-DBEHOLDER_NO_TSC", f"-I{_build.CSRC}",
                        f"-I{sysconfig.get_paths()['include']}", src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    with open(os.path.join(_build.CSRC, "gil_clock.hpp")) as f:
        text = f.read()
    assert "#include <x86intrin.h>" in text.split("#else")[0] and "BEHOLDER_HAVE_TSC 0" in text
