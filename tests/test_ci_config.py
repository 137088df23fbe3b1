"""CI runs the quality gates, not only the tests (lint, sanitizers, the differential
fuzz with a fixed budget), and the deployment image builds without ROCm."""
import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _steps(job):
    cfg = yaml.safe_load(open(os.path.join(ROOT, ".circleci", "config.yml")))
    out = []
    for st in cfg["jobs"][job]["steps"]:
        if isinstance(st, dict) and "run" in st:
            r = st["run"]
            out.append(r["command"] if isinstance(r, dict) else r)
    return cfg, out


def test_ci_test_job_runs_every_gate():
    cfg, cmds = _steps("test")
    joined = "\n".join(cmds)
    assert "python -m beholder_amd.ops.build" in joined and "--hip" not in joined
    assert "make lint" in cmds
    assert "make tsan" in cmds and "make asan" in cmds
    fuzz = [c for c in cmds if "test_native_handlers.py" in c]
    assert fuzz and "BEHOLDER_FUZZ_EXAMPLES=" in fuzz[0]
    assert int(fuzz[0].split("BEHOLDER_FUZZ_EXAMPLES=")[1].split()[0]) >= 1000
    tests = [c for c in cmds if "pytest tests" in c]
    assert tests and "--ignore" not in tests[0]  # the bench contract runs too
    assert "-m \"not gpu\"" in tests[0]


def test_build_job_requires_tests_and_is_master_only():
    cfg, cmds = _steps("build")
    jobs = cfg["workflows"]["build-push"]["jobs"]
    build = [j for j in jobs if isinstance(j, dict) and "build" in j][0]["build"]
    assert build["requires"] == ["test"] and build["filters"]["branches"]["only"] == ["master"]
    assert any("docker build" in c for c in cmds) and any("docker push tritonmedia/beholder" in c for c in cmds)


def test_dockerfile_builds_without_rocm():
    text = open(os.path.join(ROOT, "Dockerfile")).read()
    assert "FROM python:3.10-slim" in text
    build = [ln for ln in text.splitlines() if "beholder_amd.ops.build" in ln]
    assert build and "--hip " not in build[0] + " "  # the HIP extra is never required in the image


def test_dockerfile_has_the_native_build_dependencies():
    """The native runtime links OpenSSL (ops/csrc/py_tls.cpp): the slim image needs its headers;
    the CI image (python:3.10, buildpack-deps) ships them."""
    from beholder_amd import _build
    text = open(os.path.join(ROOT, "Dockerfile")).read()
    apt = [ln for ln in text.splitlines() if "apt-get install" in ln]
    assert apt and "g++" in apt[0] and "libssl-dev" in apt[0]
    assert "-lssl" in _build.LIBS and "-lcrypto" in _build.LIBS
