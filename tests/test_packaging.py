"""The shippable artifact: the deployment image and CI have no ROCm, numpy or torch.

Dockerfile and .circleci/config.yml run ``python -m beholder_amd.ops.build --force`` on stock
Python images, then the CPU test tier. The HIP library is an optional extra (the offload probe),
so the build must succeed without ``hipcc``, and every test module must collect without numpy
and torch."""
import os
import subprocess
import sys

import pytest

from beholder_amd import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_build_without_hipcc_succeeds(monkeypatch, capsys):
    monkeypatch.setattr(_build, "hipcc", lambda: "")
    called = []
    monkeypatch.setattr(_build, "build_hip", lambda **k: called.append(k))
    assert _build.main([]) == 0
    assert not called
    assert "skipping the optional gfx950 HIP extension" in capsys.readouterr().err


def test_build_hip_required_fails_without_hipcc(monkeypatch):
    monkeypatch.setattr(_build, "hipcc", lambda: "")
    with pytest.raises(RuntimeError, match="hipcc not found"):
        _build.main(["--hip"])


def test_build_with_hipcc_builds_hip(monkeypatch):
    monkeypatch.setattr(_build, "hipcc", lambda: "/opt/rocm/bin/hipcc")
    called = []
    monkeypatch.setattr(_build, "build_hip", lambda **k: called.append(k) or "lib.so")
    assert _build.main([]) == 0 and len(called) == 1
    called.clear()
    assert _build.main(["--no-hip"]) == 0 and not called


def test_build_cli_without_hipcc_on_path():
    """The module CLI as the Dockerfile runs it, with no ROCm on PATH and HIPCC unset."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from beholder_amd import _build\n"
            "_build.hipcc = lambda: ''\n"
            "sys.exit(_build.main([]))\n") % ROOT
    env = {k: v for k, v in os.environ.items() if k != "HIPCC"}
    env["PATH"] = "/usr/bin:/bin"
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr


def test_collection_without_numpy_and_torch():
    """Every test module collects with numpy and torch unavailable (stock python:3.10 CI image)."""
    # a meta-path finder that refuses the modules (as on an image without them); a None entry in
    # sys.modules would instead look like an imported module to libraries that probe sys.modules
    code = ("import sys\n"
            "class Block:\n"
            "    def find_spec(self, name, path=None, target=None):\n"
            "        if name.split('.')[0] in ('numpy', 'torch'):\n"
            "            raise ModuleNotFoundError(f'No module named {name!r}', name=name)\n"
            "sys.meta_path.insert(0, Block())\n"
            "import pytest\n"
            "sys.exit(pytest.main(['--collect-only', '-q', '-p', 'no:cacheprovider', 'tests']))\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "error" not in r.stdout.lower().split("\n")[-2], r.stdout[-2000:]


FAKE_CXX = r"""#!/bin/sh
# stand-in compiler: logs each call; `-c SRC -o OBJ` writes an empty object, the link copies the
# real extension to its -o target (slowly, so concurrent importers really overlap)
echo "$$ $*" >> "$FAKE_CXX_LOG"
out=""; link=1
while [ $# -gt 0 ]; do
  case "$1" in
    -c) link=0 ;;
    -o) shift; out="$1" ;;
  esac
  shift
done
if [ $link = 1 ]; then sleep 1; cp "$REAL_SO" "$out"; else : > "$out"; fi
"""


def test_concurrent_importers_compile_once(tmp_path):
    """A stale stamp and 6 processes importing the package at once (workers starting together):
    the build lock lets exactly one of them compile; all 6 import the result."""
    import shutil
    tree = tmp_path / "tree"
    shutil.copytree(os.path.join(ROOT, "beholder_amd"), tree / "beholder_amd",
                    ignore=shutil.ignore_patterns("__pycache__", "*.lock", "*.tmp"))
    real_so = tmp_path / "real.so"
    shutil.copy(_build.TARGET, real_so)
    with open(tree / "beholder_amd" / "ops" / os.path.basename(_build.STAMP), "w") as f:
        f.write("stale")
    cxx = tmp_path / "fake-cxx"
    cxx.write_text(FAKE_CXX)
    cxx.chmod(0o755)
    log = tmp_path / "cxx.log"
    env = dict(os.environ, CXX=str(cxx), FAKE_CXX_LOG=str(log), REAL_SO=str(real_so), PYTHONPATH=str(tree))
    env.pop("BEHOLDER_ALLOW_BUILD", None)
    code = "import beholder_amd.ops as o; print(o.native.__file__)"
    procs = [subprocess.Popen([sys.executable, "-c", code], cwd=str(tree), env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for _ in range(6)]
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), [e[-2000:] for _, e in outs]
    assert all(o.strip().startswith(str(tree)) for o, _ in outs)
    calls = log.read_text().splitlines()
    links = [c for c in calls if " -c " not in c]
    assert len(links) == 1, calls
    assert len({c.split()[0] for c in calls}) == len(calls)  # (each call its own compiler process)
    assert sum("building the native runtime" in e for _, e in outs) == 1
    assert not [f for f in os.listdir(tree / "beholder_amd" / "ops") if f.endswith(".tmp")]
