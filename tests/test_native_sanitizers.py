"""Race / memory-safety checks of the native ingest ring and the TLS handshake completion channel
(SURVEY.md §5 "race detection").

Compiles tests/native/ring_stress.cpp with ThreadSanitizer and with
AddressSanitizer+UBSan (host code only) and runs it: multi-producer ring
integrity under contention, drop accounting, random-chunk framing, shutdown
wake-ups.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("target", ["ring_stress_tsan", "ring_stress_asan"])
def test_ring_stress_under_sanitizer(target):
    b = subprocess.run(["make", "-s", target], cwd=HERE, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([os.path.join(HERE, target)], capture_output=True, text=True, timeout=300, env=env)
    if "unexpected memory mapping" in r.stderr:
        # TSan's shadow layout clashes with some kernels' mmap randomisation (seen on the GPU
        # box image): an environment limit, not a finding
        pytest.skip("ThreadSanitizer cannot map its shadow memory on this kernel")
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "ALL OK" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("target", ["hs_wake_stress_tsan", "hs_wake_stress_asan",
                                    "hs_reactor_stress_tsan", "hs_reactor_stress_asan"])
def test_handshake_completion_channel_under_sanitizer(target):
    """The TLS handshake threads' completion channel (ops/csrc/hs_wake.hpp) with the job
    ownership protocol of py_netconn.cpp around it: workers post or free, the loop drains,
    orphans connections and closes the channel while posts race it; every job is freed once.
    hs_reactor_stress: the same protocol on the real reactor (ops/csrc/hs_reactor.hpp) with
    socketpairs, jobs stepped by whichever thread takes their readiness, orphaned by shutdown(2)
    or expired by the deadline scan."""
    b = subprocess.run(["make", "-s", target], cwd=HERE, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([os.path.join(HERE, target)], capture_output=True, text=True, timeout=300, env=env)
    if "unexpected memory mapping" in r.stderr:
        pytest.skip("ThreadSanitizer cannot map its shadow memory on this kernel")
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "each freed once" in r.stdout
