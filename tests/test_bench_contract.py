"""bench.py driver contract: one JSON line, required keys, multi-rank launch via torch.distributed.run,
the single-process headline (BASELINE.json configs are single process) and the extra keys."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}
EXTRAS = {"all_procs_events_per_sec", "rate_10k_p50_ingest_latency_us", "rate_10k_p99_ingest_latency_us",
          "soak_rss_growth_mb", "soak_gc_max_pause_us", "burst_dropped", "tcp_e2e_events_per_sec",
          "rate_1k_acked", "rate_1k_p50_ingest_latency_us", "rate_1k_p99_ingest_latency_us",
          "rate_100k_offered", "rate_100k_accepted", "rate_100k_dropped", "rate_100k_p99_ingest_latency_us",
          "soak_rss_peak_growth_mb", "bench_proc_maxrss_mb",
          "http_tcp_h1_p999_handle_latency_us", "p50_handle_latency_us", "tls_e2e_events_per_sec",
          "tls_e2e_cpu_us_per_event", "cpu_us_per_event", "involuntary_ctx_switches",
          "tcp_e2e_warmup_p999_handle_latency_us", "tls_e2e_warmup_p999_handle_latency_us",
          # round 4: per-hop paced latency, calibration, config 1, stall attribution, throttling
          "rate_1k_p99_queue_latency_us", "rate_10k_p99_queue_latency_us", "rate_100k_p99_queue_latency_us",
          "rate_1k_p99_handle_latency_us", "rate_10k_p99_handle_latency_us", "rate_100k_p99_handle_latency_us",
          "calib_ns", "calib_ns_before", "calib_ns_after", "value_calibrated", "headline_nr_throttled",
          "plumbing_rc", "plumbing_acked", "plumbing_sink_requests", "plumbing_has_progress_counter",
          "plumbing_has_trello_counter", "tcp_e2e_slow_blamed", "tls_e2e_slow_blamed",
          "tcp_e2e_warmup_slow_blamed", "tls_e2e_warmup_slow_blamed", "tcp_e2e_nr_throttled",
          "tls_e2e_nr_throttled", "tcp_e2e_nivcsw", "soak_cpu_us_per_event", "tls_e2e_dial_max_us",
          "tls_e2e_queue_wait_max_us", "headline_minflt", "thp", "tls_e2e_preconnect_warmup_p999_handle_latency_us",
          "tls_e2e_preconnect_init_ms", "tls_e2e_init_ms", "rate_1k_p99_due_to_ack_us",
          "rate_10k_p99_due_to_ack_us", "rate_100k_p99_due_to_ack_us", "rate_10k_p99_due_to_recv_us",
          # round 6: the production path paced at BASELINE's rates, the timed steps' run-queue waits
          "tcp_e2e_rate_1k_p50_handle_latency_us", "tcp_e2e_rate_10k_p99_handle_latency_us",
          "tcp_e2e_rate_100k_p99_ingest_latency_us", "tls_e2e_rate_10k_p50_handle_latency_us",
          "tls_e2e_rate_100k_p99_handle_latency_us", "tcp_e2e_rate_10k_broker_late_p99_us",
          "headline_timed_run_delay_ms", "headline_timed_proc_run_delay_ms", "headline_timed_pump_run_delay_ms"}
SMALL = ["--steps", "2", "--warmup", "1", "--events-per-step", "4096", "--media", "500", "--full-out", ""]
# the keys the driver's `tail` (the last ~2,000 characters of stdout) must show
DECISION = ("value", "p50_handle_latency_us", "p99_handle_latency_us", "cpu_us_per_event", "calib_ns",
            "value_calibrated", "tcp_e2e_events_per_sec", "tcp_e2e_cpu_us_per_event", "tcp_e2e_sys_cpu_us_per_event",
            "tcp_e2e_p999_handle_latency_us", "tls_e2e_events_per_sec", "tls_e2e_p999_handle_latency_us",
            "rate_1k_p99_ingest_latency_us", "rate_10k_p99_ingest_latency_us", "rate_100k_p99_ingest_latency_us",
            "soak_events_per_sec", "soak_gc_max_pause_us", "all_procs_events_per_sec",
            "tcp_e2e_rate_1k_p50_handle_latency_us", "tcp_e2e_rate_1k_p99_handle_latency_us",
            "tcp_e2e_rate_10k_p50_handle_latency_us", "tcp_e2e_rate_10k_p99_handle_latency_us",
            "tcp_e2e_rate_10k_p50_ingest_latency_us", "tcp_e2e_rate_10k_p99_ingest_latency_us",
            "tcp_e2e_rate_100k_p50_handle_latency_us", "tcp_e2e_rate_100k_p99_handle_latency_us",
            "tls_e2e_rate_10k_p50_handle_latency_us", "tls_e2e_rate_10k_p99_handle_latency_us",
            "headline_timed_run_delay_ms")


def _last_json(stdout: str) -> dict:
    """The driver reads rank 0's stdout: exactly one line, the JSON record (no library chatter
    such as gloo's "[Gloo] Rank r is connected to ..." report)."""
    lines = [x for x in stdout.splitlines() if x.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), stdout
    return json.loads(lines[0])


def test_bench_single_rank_contract(tmp_path):
    full_path = str(tmp_path / "full.json")
    r = subprocess.run([sys.executable, "bench.py", *SMALL, "--procs-per-rank", "2", "--all-procs-steps", "1",
                        "--io-events", "2000", "--e2e-events", "4000", "--soak-events", "20000",
                        "--shared-queue-events", "3000", "--e2e-repeats", "2", "--e2e-paced-scale", "0.1",
                        "--full-out", full_path],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.strip()][-1]
    printed = _last_json(r.stdout)
    # the line the driver keeps: short, and every decision key inside its last 2,000 characters
    import bench
    assert len(line) <= bench.LINE_BUDGET <= 8000, len(line)
    tail = line[-2000:]
    for k in DECISION:
        assert f'"{k}": ' in tail, (k, tail)
    assert REQUIRED <= set(printed)
    assert printed["full_record"] == {"path": full_path, "keys": printed["full_record"]["keys"]}
    with open(full_path) as f:
        out = json.load(f)  # every key of the run
    assert printed["full_record"]["keys"] == len(out)
    for k, v in printed.items():
        if k != "full_record":
            assert out[k] == v, k
    assert REQUIRED <= set(out) and out["n_gpus"] == 1 and out["steps"] == 2 and out["warmup"] == 1
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(out["config"])
    assert EXTRAS <= set(out), EXTRAS - set(out)
    # the headline is ONE consumer process (BASELINE.json configs are single process)
    assert out["config"]["global_batch"] == 4096 and "1 consumer proc/rank" in out["config"]["parallelism"]
    assert out["value"] > 0 and out["handler_errors"] == 0
    assert out["value"] == pytest.approx(4096 * 2 / (out["ms_per_step"] * 2 / 1000), rel=0.01)
    assert out["all_procs_per_rank"] == 2 and out["all_procs_events_per_sec"] > 0
    assert out["rate_10k_acked"] == 10000 and out["soak_events"] == 20000 and out["tcp_e2e_errors"] == 0
    assert out["tls_e2e_errors"] == 0 and out["tls_e2e_preconnect_errors"] == 0
    assert out["tls_e2e_preconnect_handshakes"] >= 1
    assert out["burst_accepted"] + out["burst_dropped"] == out["burst_offered"]
    # BASELINE configs 2 and 4 as specified: 1 s at 1k/s, 1 s paced at 100k/s into the 4096 ring
    assert out["rate_1k_acked"] == 1000
    # due -> ack holds receive -> ack (the event cannot be received before it is due... almost:
    # the producer writes every frame already due in one write, so allow the pacing grain)
    assert out["rate_10k_p99_due_to_ack_us"] + 200 >= out["rate_10k_p99_ingest_latency_us"]
    assert out["rate_100k_offered"] == 100_000
    assert out["rate_100k_accepted"] + out["rate_100k_dropped"] == out["rate_100k_offered"]
    assert out["rate_100k_acked"] == out["rate_100k_accepted"]
    assert "soak_rss_peak_mb" not in out and "overload_offered" not in out
    # BASELINE config 1: the real CLI on stdin, /metrics scraped with both reference counters
    assert out["plumbing_rc"] == 0 and out["plumbing_acked"] == 100 and out["plumbing_sink_requests"] > 0
    assert out["plumbing_has_progress_counter"] and out["plumbing_has_trello_counter"]
    assert out["calib_ns"] >= max(out["calib_ns_before"], out["calib_ns_after"]) > 0
    assert set(out["tcp_e2e_slow_blamed"]) >= {"consumer", "pg", "http", "none"}
    # the e2e phases say what else could have moved them
    # the window starts at the settled count read after the warm-up (a few in-flight deliveries past it)
    assert 4000 - 400 - 300 <= out["tcp_e2e_measured_events"] <= 4000 - 400 and out["tcp_e2e_calib_ns"] > 0
    assert set(out["tcp_e2e_fakes_cpu_us_per_event"]) == {"broker", "pg", "http"}
    assert len(out["tcp_e2e_runs"]["events_per_sec"]) == 2 and out["tcp_e2e_events_per_sec"] in \
        out["tcp_e2e_runs"]["events_per_sec"]
    assert out["tcp_e2e_sys_cpu_us_per_event"] >= 0 and out["tcp_e2e_minflt"] >= 0
    runs = out["tcp_e2e_runs"]
    assert all(len(runs[k]) == 2 for k in ("sys_cpu_us_per_event", "events_per_poll_run", "calib_ns"))
    assert all(x > 0 for x in runs["events_per_poll_run"]), runs
    assert out["tcp_e2e_run_delay_ms"] is None or out["tcp_e2e_run_delay_ms"] >= 0
    assert out["rate_10k_loop_run_delay_us"] is None or out["rate_10k_loop_run_delay_us"] >= 0
    assert out["headline_run_delay_ms"] is None or out["headline_run_delay_ms"] >= 0
    assert out["headline_timed_run_delay_ms"] is None or out["headline_timed_run_delay_ms"] >= 0
    # the paced production path: every event of each rate measured and acked, none failing
    for pre in ("tcp_e2e", "tls_e2e"):
        for name, rate, n in bench.E2E_RATES:
            k = f"{pre}_rate_{name}"
            # a tenth is warm-up, and the warm-up's end is seen at a poll (up to 50 ms of events later)
            assert out[f"{k}_errors"] == 0 and out[f"{k}_measured_events"] >= max(200, int(n * 0.1)) * 0.6, k
            assert out[f"{k}_p50_handle_latency_us"] <= out[f"{k}_p99_handle_latency_us"], k
    # the consumer's socket calls per event: a send per sink request, queries
    # and acks batched, every kind of connection seen
    io = out["tcp_e2e_io_per_event"]
    assert set(io) == {"h1_sends", "h1_recvs", "pg_sends", "pg_recvs", "poll_runs", "poll_ready", "amqp_reads",
                       "amqp_writes"}
    assert 0.2 < io["h1_sends"] < 1.0 and all(io[k] > 0 for k in io), io
    # competing consumers on one queue (run --workers N), every event acked exactly once
    ns = bench.shared_queue_workers(out["cpus_available"])
    assert list(out["shared_queue_events_per_sec"]) == [str(n) for n in ns] and out["shared_queue_exactly_once"]
    assert all(out["shared_queue_acked"][str(n)] == out["shared_queue_published"][str(n)] == 3000 * n for n in ns)


def test_bench_two_ranks_gloo():
    pytest.importorskip("torch")  # torch.distributed.run launches the ranks
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29561", "bench.py", "--gpus", "2",
                        *SMALL, "--procs-per-rank", "2", "--all-procs-steps", "1", "--no-extras"],
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _last_json(r.stdout)
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 8192
    assert out["config"]["parallelism"].startswith("dp2")
    assert out["value"] == pytest.approx(8192 * 2 / (out["ms_per_step"] * 2 / 1000), rel=0.01)
    assert out["all_procs_per_rank"] == 2 and out["all_procs_events_per_sec"] > 0
    assert "tcp_e2e_events_per_sec" not in out


def test_all_procs_phase_adds_up():
    """Consumer processes of the all-process phase: events add up over the spawned consumers."""
    import bench
    a = bench.parse([*SMALL, "--procs-per-rank", "2"])
    res = bench.run_procs(a, bench._Dist(), 2, steps=2)
    assert res["events"] == 2 * 2 * 4096 and res["errors"] == 0 and res["procs"] == 2


def test_consumers_get_no_head_start(monkeypatch):
    """A slow cross-rank barrier before the clock must not let consumers start early: the
    coordinator's clock and each consumer's own clock cover the same steps."""
    import time as _time

    import bench
    calls = []

    def slow_first_barrier(self):
        calls.append(1)
        if len(calls) == 1:
            _time.sleep(0.5)
    monkeypatch.setattr(bench._Dist, "barrier", slow_first_barrier)
    a = bench.parse([*SMALL, "--procs-per-rank", "2"])
    res = bench.run_procs(a, bench._Dist(), 2, steps=2)
    assert res["events"] == 2 * 2 * 4096
    # with a head start the consumers would finish ~0.5 s of work before the coordinator's t0
    assert res["coordinator_elapsed"] >= res["max_consumer_elapsed"] - 0.05, res
    assert res["coordinator_elapsed"] < res["max_consumer_elapsed"] + 1.0, res
    assert len(calls) == 1


def test_no_hip_before_child_processes(monkeypatch, capsys):
    """Every child process (TCP fakes, all-process consumers) starts before the first device
    synchronize, the first HIP call of the coordinator; torch has not initialised HIP then."""
    import bench
    from beholder_amd.bench import harness
    order = []
    orig_sync, orig_spawn, orig_procs = bench._Device.sync, harness._spawn, bench.run_procs

    def spy_sync(self):
        order.append("sync")
        orig_sync(self)

    def spy_spawn(*a, **k):
        torch = sys.modules.get("torch")
        assert torch is None or not torch.cuda.is_initialized()
        order.append("spawn")
        return orig_spawn(*a, **k)

    def spy_procs(*a, **k):
        torch = sys.modules.get("torch")
        assert torch is None or not torch.cuda.is_initialized()
        order.append("procs")
        return orig_procs(*a, **k)
    monkeypatch.setattr(bench._Device, "sync", spy_sync)
    monkeypatch.setattr(harness, "_spawn", spy_spawn)
    monkeypatch.setattr(bench, "run_procs", spy_procs)
    assert bench.main([*SMALL, "--procs-per-rank", "2", "--all-procs-steps", "1", "--io-events", "1000",
                       "--e2e-events", "1000", "--soak-events", "5000", "--shared-queue-events", "0",
                       "--e2e-paced-scale", "0"]) == 0
    out = _last_json(capsys.readouterr().out)
    assert out["value"] > 0
    assert "spawn" in order and "procs" in order and "sync" in order
    first = order.index("sync")
    assert all(x == "sync" for x in order[first:]), order


def test_line_is_strict_json():
    """A NaN or infinity in any extra key would make the driver's JSON parse fail: they print as
    null."""
    import bench
    out = bench._finite({"value": 1.5, "x": float("nan"), "y": [float("inf"), 2], "z": {"w": float("-inf")}})
    assert json.loads(json.dumps(out, allow_nan=False)) == {"value": 1.5, "x": None, "y": [None, 2], "z": {"w": None}}


def test_a_failing_extra_phase_still_leaves_the_line(capsys):
    import bench

    def boom(a):
        raise RuntimeError("fake would not start")
    assert bench._phase("io_extras", boom, None) == {"io_extras_error": "RuntimeError: fake would not start"}
    assert "fake would not start" in capsys.readouterr().err
    assert bench._phase("paced_extras", lambda a: {"k": 1}, None) == {"k": 1}


def test_compact_line_keeps_decision_keys_last_and_fits():
    """However many diagnostic keys a run produces, the printed line stays within LINE_BUDGET and
    the decision keys are its last TAIL_BUDGET characters; oversized diagnostics are left to the
    full record."""
    import bench
    full = {k: 1 for k in bench.HEAD_KEYS}
    full.update({"data": "x" * 300, "config": {"model": "m", "global_batch": 1, "seq_len": None, "parallelism": "dp1"}})
    full.update({f"diag_{i}": {"a": 123456.7, "b": [1, 2, 3]} for i in range(400)})
    full["huge"] = "y" * 9000
    full.update({k: 123456.789 for k in bench.TAIL_KEYS if k not in ("shared_queue_events_per_sec",)})
    full["shared_queue_events_per_sec"] = {"1": 123456.7, "2": 234567.8, "4": 345678.9, "8": 456789.1}
    line = json.dumps(bench.compact_line(full, "/x/full.json"))
    assert len(line) <= bench.LINE_BUDGET
    assert "huge" not in line and '"diag_0"' in line
    tail_keys = [k for k in json.loads(line)][-len(bench.TAIL_KEYS):]
    assert tail_keys == list(bench.TAIL_KEYS)
    assert tail_keys[-1] == "value"
    start = line.index(f'"{bench.TAIL_KEYS[0]}"')
    assert len(line) - start <= bench.TAIL_BUDGET, len(line) - start
