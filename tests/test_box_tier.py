"""Box-tier tests (``-m gpu``): run on the MI355X box at round end.

Beholder has no device kernels (the reference service has none), so these do
not touch the accelerator. They exercise the *native* runtime on the target
machine image at full scale: the in-tree extension must be the one loaded,
the BASELINE.json configs must meet their targets, and the multi-rank bench
launcher must work.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_native_runtime_is_in_tree_and_loaded():
    from beholder_amd import ops
    path = os.path.realpath(ops.native.__file__)
    assert path.startswith(os.path.realpath(os.path.join(ROOT, "beholder_amd", "ops"))), path
    assert ops.native.ABI_VERSION == 1
    # every hot-path entry point is native
    for name in ("MessageCodec", "Ingest", "Delivery", "Settler", "Histogram", "format_line", "encode_query",
                 "AmqpDemux", "H1Parser", "PgReader", "Driver", "IOFuture", "AckBatcher", "Buckets",
                 "dispatch_batch", "pg_bind", "NativeHandlers", "HandlerCall", "SinkStats", "_C_API", "io_counts"):
        assert hasattr(ops.native, name), name
    # bench / diagnostic code is a module of its own, also in-tree
    for name in ("Recorder", "prof_start", "prof_stop", "calib", "calib_mem", "paced_write"):
        assert not hasattr(ops.native, name), name
    from beholder_amd.ops import bench_native
    bpath = os.path.realpath(bench_native.native_bench.__file__)
    assert bpath.startswith(os.path.realpath(os.path.join(ROOT, "beholder_amd", "ops"))), bpath


def test_compiled_handlers_match_python_on_the_box():
    """The compiled handlers are the service default, and they agree with handlers.py on the
    target image: the same 20k-event stream through both gives identical sink requests, counters
    and store contents."""
    import asyncio

    from beholder_amd.bench.generator import Workload, bench_config
    from beholder_amd.config import Config
    from beholder_amd.ops import native
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    from beholder_amd.store import MemoryStore
    from beholder_amd.transport.ingest import BytesSource
    from beholder_amd.utils.log import Logger, MemoryStream

    w = Workload(n_media=500, seed=11, unknown_media_fraction=0.01)
    data = w.framed(20_000)

    def run(native_on):
        cfg = bench_config()
        cfg["service"]["native_handlers"] = native_on
        http, store, stream = RecordingHttpClient(), MemoryStore(w.media), MemoryStream()
        svc = Service(Config.from_dict(cfg), source=BytesSource(data), store=store, http=http,
                      logger=Logger(stream=stream), serve_metrics=False)

        async def go():
            await svc.init()
            st = await svc.run()
            await svc.close()
            return st
        st = asyncio.run(go())
        import gc
        gc.collect()  # un-acked (Q1) deliveries are counted abandoned when freed
        st["source"] = svc.source.settler.stats()
        return svc, st, list(http.calls), sorted(store.snapshot().items()), [
            (r["level"], r["msg"]) for r in stream.records()]

    a = run(True)
    b = run(False)
    assert isinstance(a[0].handler_impl, native.NativeHandlers) and b[0].handler_impl is b[0].handlers
    assert a[1]["source"]["acked"] == b[1]["source"]["acked"] and a[1]["source"]["abandoned"] == b[1]["source"]["abandoned"]
    assert a[1]["progress_updates"] == b[1]["progress_updates"] and a[1]["trello_comments"] == b[1]["trello_comments"]
    assert a[2] == b[2] and a[3] == b[3] and a[4] == b[4]


def test_bench_single_rank_full_path():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "1",
                          "--e2e-repeats", "1", "--e2e-events", "50000", "--shared-queue-events", "20000",
                          "--full-out", ""],
                         capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
    r = json.loads(line)
    assert r["metric"] == "metric_events_ingested_per_sec" and r["n_gpus"] == 1
    assert r["handler_errors"] == 0
    assert r["value"] > 20000, r


def test_baseline_configs_plumbing_and_backpressure():
    """BASELINE configs 1 (100 events on stdin) and 4 (100k ev/s, backpressure + drop accounting)."""
    from beholder_amd.bench import harness
    res = harness.run_config("plumbing")
    assert res["acked"] == 100 and res["errors"] == 0
    res = harness.run_config("backpressure", duration_s=2.0)
    assert res["offered"] == res["accepted"] + res["dropped"], res


def test_soak_1m_events_rss_and_gc():
    """BASELINE config 5: 1M events, report RSS and GC pauses; RSS must stay bounded."""
    from beholder_amd.bench import harness
    res = harness.run_config("soak", events=1_000_000)
    assert res["acked"] == 1_000_000
    assert res["rss_growth_mb"] < 64, res  # the service itself must not grow with traffic


def test_bench_two_ranks_torchrun_on_box():
    """The driver's multi-GPU launch path (torch.distributed.run, gloo barriers, MAX over ranks)."""
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", "29571", os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--steps", "3", "--warmup", "1", "--procs-per-rank", "2", "--no-extras"],
                         capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert r["n_gpus"] == 2 and r["all_procs_per_rank"] == 2 and r["handler_errors"] == 0
    # value = one consumer per rank (BASELINE configs are single process); all_procs_* = 2 per rank
    assert r["config"]["global_batch"] == 2 * 65536


def test_io_bound_concurrency_reaches_prefetch():
    """Sinks with 2 ms latency: up to prefetch (100, index.js:43) handlers in flight."""
    from beholder_amd.bench import harness
    res = harness.run_config("io_bound", events=20000)
    assert res["acked"] == 20000 and res["max_inflight"] == 100


def test_tcp_e2e_every_dependency_over_tcp():
    """Production shape: AMQP broker -> service -> Postgres (pipelined) + HTTP sinks (keep-alive),
    all over real sockets; every event acked, every DB read / sink call answered."""
    from beholder_amd.bench import harness
    res = harness.run_config("tcp_e2e", events=50_000)
    assert res["acked"] == 50_000 and res["errors"] == 0, res
    assert res["server_side"]["queries"] >= 50_000  # one media read per event (index.js:76,140)
    assert res["server_side"]["requests"] == res["http"]["requests"] and res["http"]["errors"] == 0


def test_tls_e2e_https_sinks_on_native_tls():
    """Production shape with HTTPS sinks (Trello / Telegram are HTTPS): every request on a
    native TLS connection (ops TlsContext), certificates verified, every event acked."""
    from beholder_amd.bench import harness
    res = harness.run_config("tls_e2e", events=50_000)
    assert res["tls"] is True and res["acked"] == 50_000 and res["errors"] == 0, res
    assert res["server_side"]["requests"] == res["http"]["requests"] and res["http"]["errors"] == 0
    assert res["http"]["connections"] <= 100  # keep-alive: no reconnect churn


def test_tls_e2e_million_events_memory_flat():
    """1M events over every native socket path (AMQP, Postgres NetConns, HTTPS sinks on native TLS
    with H1Call): the process RSS after the run is within a few MB of the warm start, and within
    a few MB over the run's second half alone (a leak of 8 bytes per event would add 4 MB there;
    box: 1.9 MB and 0.16 MB, profiles/box_r5_rss/)."""
    from beholder_amd.bench import harness
    res = harness.run_config("tls_e2e", events=1_000_000)
    assert res["acked"] == 1_000_000 and res["errors"] == 0, res
    assert res["rss_growth_mb"] < 16, res["rss_growth_mb"]
    assert res["rss_growth_second_half_mb"] < 4, res["rss_growth_second_half_mb"]


def test_http_tcp_both_clients_error_free():
    """Sinks over real TCP with the default keep-alive client and with aiohttp: every event
    acked, no handler errors (aiohttp under the native Driver needs its own task)."""
    from beholder_amd.bench import harness
    res = harness.run_config("http_tcp", events=20_000)
    for kind in ("h1", "aiohttp"):
        assert res[kind]["acked"] == 20_000 and res[kind]["errors"] == 0, (kind, res[kind]["error_samples"])


def test_shared_queue_competing_consumers_on_the_box():
    """The reference's scaling mode at full scale on the target machine: `run --workers 4` on one
    shared queue, 50k events per worker, every event acked exactly once at the broker, the work
    spread over all four workers."""
    from beholder_amd.bench.shared_queue import run_shared
    r = run_shared(4, 200_000)
    assert r["supervisor_rc"] == 0, r.get("supervisor_stderr")
    assert r["exactly_once"] and r["acked"] == r["published"] == 200_000
    assert len(r["per_connection_delivered"]) == 4 and min(r["per_connection_delivered"]) > 20_000
    assert r["events_per_sec"] > 100_000, r
