"""Source mutations the reference-executed gate must catch.

Each case copies the package to a scratch tree, changes one line of one handler implementation
(``handlers.py`` or its compiled twin ``ops/csrc/py_handlers.cpp``, which the scratch tree then
rebuilds), and runs ``tests/reference_oracle.py`` there against ``/root/reference/index.js`` on
Node: the gate must report a difference. The unmutated copy must pass, so a failure is the
mutation's.

The ``reread`` scenarios are the ones that see Q3 (index.js:94 keys the hooks off the row
``getByID`` re-read, not off the message): there another writer changes the row between the
listener's ``updateStatus`` and its ``getByID`` (index.js:68,76). The ``faults`` scenarios run
with ``--suspend`` (every store call and sink request waits, as production's socket clients do)
reach the compiled handlers' resume states, where the two resume mutations live. The
``concurrent`` scenarios (several deliveries in flight, resumed in a scripted order on both sides)
see a per-media serialisation that the reference does not have (Q9). The ``--service`` runs put
each event through the whole consumer (AMQP broker, ``AmqpSource``, the service's dispatch, acks
counted at the broker), where a mutation of the transport's ack flushing shows.
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

# name -> (file, original text, mutated text, the gate's scenario options): each a one-line change
# of behaviour
REREAD = ("--modes", "reread")
FAULTS_SUSPENDED = ("--modes", "faults", "--suspend")
SERVICE = ("--modes", "base", "--service")  # through the whole consumer (run_service)
SOCKETS = ("--modes", "faults", "--service", "--sockets")  # ... with Postgres and the sinks over TCP
MUTATIONS = {
    # Q3 (index.js:94): the DEPLOYED hooks keyed off the message's status, not the re-read row's
    "hooks_off_message_status_python": (
        "beholder_amd/handlers.py",
        "            if media.status == self.deployed:",
        "            if status == self.deployed:", REREAD),
    "hooks_off_message_status_native": (
        "beholder_amd/ops/csrc/py_handlers.cpp",
        "      PyObject* ms = field(c->media, hs->media_cls, hs->ix_m[2], s_status);",
        "      PyObject* ms = Py_NewRef(c->status);", REREAD),
    # Q4 (index.js:92-122): a Telegram failure the status handler resumes with (state 5) falls
    # through to Emby instead of the catch
    "telegram_failure_runs_emby_native": (
        "beholder_amd/ops/csrc/py_handlers.cpp",
        "      value = request_finish(c, value);\n      if (!value) goto hooks_catch;\n      Py_DECREF(value);\n"
        "    emby: {",
        "      value = request_finish(c, value);\n      if (!value) { PyErr_Clear(); goto emby; }\n"
        "      Py_DECREF(value);\n    emby: {", FAULTS_SUSPENDED),
    # index.js:53-57,149-151: a comment POST failure the progress handler resumes with (state 2)
    # counts the comment and skips the warning
    "comment_failure_counted_native": (
        "beholder_amd/ops/csrc/py_handlers.cpp",
        "      value = request_finish(c, value);\n      if (!value) goto catch_;",
        "      value = request_finish(c, value);\n      if (!value) { PyErr_Clear(); goto commented; }",
        FAULTS_SUSPENDED),
    # the consumer path, which the handler-level gate does not run: acks settled by the handlers
    # are never scheduled for a flush over AMQP (they would leave only when the channel closes)
    "acks_never_flushed": (
        "beholder_amd/transport/amqp/source.py",
        "        loop.call_soon(self._flush_acks)",
        "        pass  # loop.call_soon(self._flush_acks)", SERVICE),
    # the NetPoller's batch end: the callables deferred to it (the ack flush of handlers that
    # finished inside the batch) never run; only the socket runs have a NetPoller
    "deferred_acks_never_flushed": (
        "beholder_amd/ops/csrc/py_netpoll.cpp",
        "  flush_all(p);\n  run_deferred(p);",
        "  flush_all(p);\n  (void)run_deferred;", SOCKETS),
    # Q9 (index.js:43,62,127): deliveries of one media serialised by default
    "per_media_ordering_by_default": (
        "beholder_amd/config.py",
        '        "ordering": "none",',
        '        "ordering": "per_media",', ("--modes", "concurrent")),
}
# the mutations tests/test_handlers.py must catch too (its "suspend" cases reach the resume states)
HANDLER_SUITE_CATCHES = ("telegram_failure_runs_emby_native", "comment_failure_counted_native")


def _tree(tmp_path, mutation=None):
    dst = tmp_path / "tree"
    ignore = shutil.ignore_patterns("__pycache__", "*.so", "*.srchash", "*.lock", "*.tmp", "hip")
    shutil.copytree(os.path.join(ROOT, "beholder_amd"), dst / "beholder_amd", ignore=ignore)
    shutil.copytree(os.path.join(ROOT, "scripts", "reference_node"), dst / "scripts" / "reference_node")
    os.makedirs(dst / "tests")
    for f in ("reference_oracle.py", "helpers.py", "conftest.py", "test_handlers.py", "pg_fake.py"):
        shutil.copy(os.path.join(HERE, f), dst / "tests" / f)
    if mutation:
        path, old, new, _ = MUTATIONS[mutation]
        with open(dst / path) as f:
            text = f.read()
        assert text.count(old) == 1, f"{mutation}: the line to mutate is not in {path} exactly once"
        with open(dst / path, "w") as f:
            f.write(text.replace(old, new))
    return dst


def _env(tree):
    return dict(os.environ, BEHOLDER_ALLOW_BUILD="1", PYTHONPATH=str(tree))


def _gate(tree, impl: str, modes=REREAD) -> subprocess.CompletedProcess:
    return subprocess.run([sys.executable, "tests/reference_oracle.py", "--seeds", "2", "--events", "400",
                           *modes, "--impls", impl], cwd=tree, env=_env(tree), capture_output=True,
                          text=True, timeout=600)


@pytest.mark.parametrize("modes", [REREAD, FAULTS_SUSPENDED, ("--modes", "concurrent"), SERVICE, SOCKETS],
                         ids=["reread", "faults_suspend", "concurrent", "service", "sockets"])
def test_unmutated_copy_passes_the_gate(tmp_path, modes):
    r = _gate(_tree(tmp_path), "python,native", modes)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count(" OK ") == 4, r.stdout


@pytest.mark.parametrize("name", sorted(MUTATIONS))
def test_gate_catches_the_mutation(tmp_path, name):
    impl = "native" if name.endswith("_native") else "python" if name.endswith("_python") else "python,native"
    r = _gate(_tree(tmp_path, name), impl, MUTATIONS[name][3])
    assert r.returncode == 1 and "DIFF" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    assert "OK" not in r.stdout, r.stdout[-3000:]  # caught on every seed and implementation
    assert "Traceback" not in r.stderr, r.stderr[-3000:]


@pytest.mark.parametrize("name", HANDLER_SUITE_CATCHES)
def test_handler_suite_catches_the_resume_mutation(tmp_path, name):
    """The branch suite alone catches the resume-state mutations: its suspending cases finish the
    compiled handlers in the states a socket client always leads to."""
    tree = _tree(tmp_path, name)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "tests/test_handlers.py"],
                       cwd=tree, env=_env(tree), capture_output=True, text=True, timeout=600)
    assert r.returncode == 1, r.stdout[-3000:] + r.stderr[-3000:]
    failed = [ln for ln in r.stdout.splitlines() if ln.startswith("FAILED")]
    assert failed and all("[native-suspend]" in ln for ln in failed), r.stdout[-3000:]


def test_reread_scenarios_reach_both_directions_of_q3():
    """The reread streams hold status events whose re-read row decides the hooks against the
    message: hooks that run after a non-DEPLOYED message, and hooks skipped after a DEPLOYED one."""
    total = {"hooks_without_deployed_msg": 0, "hooks_skipped_on_deployed_msg": 0}
    for seed in range(2):
        sc = ro.make_scenario(seed, 400, "reread")
        for k, v in ro.reread_coverage(sc, ro.run_node(sc)).items():
            total[k] += v
    assert all(v > 0 for v in total.values()), total
