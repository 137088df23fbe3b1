"""Race / memory-safety checks of the native ingest ring (SURVEY.md §5 "race detection").

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
