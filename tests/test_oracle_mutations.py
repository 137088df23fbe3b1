"""Source mutations the reference-executed gate must catch.

Each case copies the package to a scratch tree, changes one line of one handler implementation
(``handlers.py`` or its compiled twin ``ops/csrc/py_handlers.cpp``, which the scratch tree then
rebuilds), and runs ``tests/reference_oracle.py`` there against ``/root/reference/index.js`` on
Node: the gate must report a difference. The unmutated copy must pass, so a failure is the
mutation's.

The ``reread`` scenarios are the ones that see Q3 (index.js:94 keys the hooks off the row
``getByID`` re-read, not off the message): there another writer changes the row between the
listener's ``updateStatus`` and its ``getByID`` (index.js:68,76).
"""
import os
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import reference_oracle as ro  # noqa: E402

pytestmark = pytest.mark.skipif(not ro.available(), reason="needs node and /root/reference/index.js")

# (file, original line, mutated line): each a one-line change of behaviour
MUTATIONS = {
    # Q3 (index.js:94): the DEPLOYED hooks keyed off the message's status, not the re-read row's
    "hooks_off_message_status_python": (
        "beholder_amd/handlers.py",
        "            if media.status == self.deployed:",
        "            if status == self.deployed:"),
    "hooks_off_message_status_native": (
        "beholder_amd/ops/csrc/py_handlers.cpp",
        "      PyObject* ms = field(c->media, hs->media_cls, hs->ix_m[2], s_status);",
        "      PyObject* ms = Py_NewRef(c->status);"),
}


def _tree(tmp_path, mutation=None):
    dst = tmp_path / "tree"
    ignore = shutil.ignore_patterns("__pycache__", "*.so", "*.srchash", "*.lock", "*.tmp", "hip")
    shutil.copytree(os.path.join(ROOT, "beholder_amd"), dst / "beholder_amd", ignore=ignore)
    shutil.copytree(os.path.join(ROOT, "scripts", "reference_node"), dst / "scripts" / "reference_node")
    os.makedirs(dst / "tests")
    for f in ("reference_oracle.py", "helpers.py"):
        shutil.copy(os.path.join(HERE, f), dst / "tests" / f)
    if mutation:
        path, old, new = MUTATIONS[mutation]
        with open(dst / path) as f:
            text = f.read()
        assert text.count(old) == 1, f"{mutation}: the line to mutate is not in {path} exactly once"
        with open(dst / path, "w") as f:
            f.write(text.replace(old, new))
    return dst


def _gate(tree, impl: str) -> subprocess.CompletedProcess:
    env = dict(os.environ, BEHOLDER_ALLOW_BUILD="1", PYTHONPATH=str(tree))
    return subprocess.run([sys.executable, "tests/reference_oracle.py", "--seeds", "2", "--events", "400",
                           "--modes", "reread", "--impls", impl], cwd=tree, env=env, capture_output=True,
                          text=True, timeout=600)


def test_unmutated_copy_passes_the_reread_gate(tmp_path):
    r = _gate(_tree(tmp_path), "python,native")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count(" OK ") == 4, r.stdout


@pytest.mark.parametrize("name", sorted(MUTATIONS))
def test_gate_catches_the_mutation(tmp_path, name):
    impl = "native" if name.endswith("_native") else "python"
    r = _gate(_tree(tmp_path, name), impl)
    assert r.returncode == 1 and "DIFF" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    assert "Traceback" not in r.stderr, r.stderr[-3000:]


def test_reread_scenarios_reach_both_directions_of_q3():
    """The reread streams hold status events whose re-read row decides the hooks against the
    message: hooks that run after a non-DEPLOYED message, and hooks skipped after a DEPLOYED one."""
    total = {"hooks_without_deployed_msg": 0, "hooks_skipped_on_deployed_msg": 0}
    for seed in range(2):
        sc = ro.make_scenario(seed, 400, "reread")
        for k, v in ro.reread_coverage(sc, ro.run_node(sc)).items():
            total[k] += v
    assert all(v > 0 for v in total.values()), total
