"""Shared pytest configuration.

Marker ``gpu``: the driver runs ``pytest -m gpu`` on a real MI355X box at
round end. Beholder has no device kernels (the reference service has none —
SURVEY.md §0/§2.3), so the ``gpu`` tier holds the *box-tier* tests: the native
ingest runtime loaded on the target machine image, the full-scale BASELINE
configs (10k/100k ev/s, 1M soak) and the multi-rank bench launcher. They need
the box's CPU/memory headroom, not the accelerator.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: MI355X-box tier test (native runtime at full scale)")
    config.addinivalue_line("markers", "slow: long-running soak/bench test")
