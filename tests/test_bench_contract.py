"""bench.py driver contract: one JSON line, required keys, multi-rank launch via torch.distributed.run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _last_json(stdout: str) -> dict:
    lines = [x for x in stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_single_rank_contract():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--events-per-step", "4096",
                        "--procs-per-rank", "1"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = _last_json(r.stdout)
    assert REQUIRED <= set(out) and out["n_gpus"] == 1 and out["steps"] == 2 and out["warmup"] == 1
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(out["config"])
    assert out["value"] > 0 and out["handler_errors"] == 0
    assert out["value"] == pytest.approx(4096 * 2 / (out["ms_per_step"] * 2 / 1000), rel=0.01)


def test_bench_two_ranks_gloo():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29561", "bench.py", "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--events-per-step", "4096", "--procs-per-rank", "1"],
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _last_json(r.stdout)
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 8192
    assert out["config"]["parallelism"].startswith("dp2")


def test_bench_multiprocess_rank():
    """Consumer processes per rank: events add up, value = total events / coordinator time."""
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--events-per-step", "4096",
                        "--procs-per-rank", "2"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _last_json(r.stdout)
    assert out["procs_per_rank"] == 2 and out["config"]["global_batch"] == 8192
    assert out["value"] == pytest.approx(8192 * 2 / (out["ms_per_step"] * 2 / 1000), rel=0.01)
    assert out["handler_errors"] == 0


def test_consumers_get_no_head_start(monkeypatch):
    """Slow device initialisation before the clock must not let consumers start early: the
    coordinator's clock and each consumer's own clock cover the same K steps."""
    import time as _time

    import bench
    calls = []

    def slow_first_sync(self):  # device initialisation happens on the first sync only
        calls.append(1)
        if len(calls) == 1:
            _time.sleep(0.5)
    monkeypatch.setattr(bench._Device, "sync", slow_first_sync)
    a = bench.parse(["--procs-per-rank", "2", "--steps", "2", "--warmup", "1", "--events-per-step", "4096",
                     "--media", "200"])
    res = bench.run_rank(a, bench._Dist(), 2)
    assert res["events"] == 2 * 2 * 4096
    # with a head start the consumers would finish ~0.5 s of work before the coordinator's t0
    assert res["coordinator_elapsed"] >= res["max_consumer_elapsed"] - 0.05, res
    assert res["coordinator_elapsed"] < res["max_consumer_elapsed"] + 1.0, res
    assert len(calls) == 2  # before t0 and before t1
