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
    build = [ln for ln in text.splitlines() if "beholder_amd._build" in ln]
    assert build and "--hip " not in build[0] + " "  # the HIP extra is never required in the image


def _stages():
    """Dockerfile stages: name -> list of instruction lines (continuations joined)."""
    text = open(os.path.join(ROOT, "Dockerfile")).read().replace("\\\n", " ")
    stages, cur = {}, None
    for ln in text.splitlines():
        ln = ln.strip()
        if not ln or ln.startswith("#"):
            continue
        if ln.upper().startswith("FROM "):
            parts = ln.split()
            cur = parts[3] if len(parts) >= 4 and parts[2].upper() == "AS" else str(len(stages))
            stages[cur] = []
        stages[cur].append(ln)
    return stages


def test_dockerfile_has_the_native_build_dependencies():
    """The native runtime links OpenSSL (ops/csrc/py_tls.cpp): the build stage needs g++ and its
    headers; the CI image (python:3.10, buildpack-deps) ships them."""
    from beholder_amd import _build
    build = _stages()["build"]
    apt = [ln for ln in build if "apt-get install" in ln]
    assert apt and "g++" in apt[0] and "libssl-dev" in apt[0]
    # the build module alone (beholder_amd/__init__ imports nothing): one compile, no protobuf needed
    assert any("python -m beholder_amd._build --force" in ln for ln in build)
    assert "-lssl" in _build.LIBS and "-lcrypto" in _build.LIBS


def test_runtime_stage_has_no_compiler_and_never_rebuilds():
    """The shipped stage (the last one) copies the built tree from the build stage, installs no
    compiler or headers, runs as uid 999 and sets BEHOLDER_ALLOW_BUILD=0, so an import never
    recompiles C++ in production (ops/__init__.py)."""
    stages = _stages()
    assert list(stages)[-1] == "runtime" and len(stages) == 2
    rt = stages["runtime"]
    assert not any(("apt-get" in ln or "g++" in ln or "-dev" in ln or "gcc" in ln) for ln in rt)
    assert any(ln.startswith("COPY --from=build") and "/stack" in ln for ln in rt)
    assert any(ln.startswith("ENV") and "BEHOLDER_ALLOW_BUILD=0" in ln for ln in rt)
    assert any(ln == "USER 999" for ln in rt)
    assert rt[-1].startswith("ENTRYPOINT") and "beholder_amd" in rt[-1]
    ignore = open(os.path.join(ROOT, ".dockerignore")).read().split()
    assert "**/*.so" in ignore and ".git" in ignore  # the image builds its own extension


def test_allow_build_0_loads_without_compiling(tmp_path):
    """With BEHOLDER_ALLOW_BUILD=0 a stale stamp does not trigger a build (no compiler needed)."""
    import shutil
    import subprocess
    import sys
    from beholder_amd import _build
    tree = tmp_path / "tree"
    shutil.copytree(os.path.join(ROOT, "beholder_amd"), tree / "beholder_amd",
                    ignore=shutil.ignore_patterns("__pycache__", "*.lock", "*.tmp", "csrc"))
    with open(tree / "beholder_amd" / "ops" / os.path.basename(_build.STAMP), "w") as f:
        f.write("stale")
    env = dict(os.environ, CXX="/nonexistent/c++", PYTHONPATH=str(tree), BEHOLDER_ALLOW_BUILD="0")
    r = subprocess.run([sys.executable, "-c", "import beholder_amd.ops as o; print(o.native.__file__)"],
                       cwd=str(tree), env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().startswith(str(tree)) and "building" not in r.stderr
