"""`run --workers N`: supervised competing-consumer processes on one AMQP queue."""
import os
import signal
import subprocess
import sys
import time

from beholder_amd.metrics import parse_exposition
from beholder_amd.parallel.workers import strip_workers_arg
from beholder_amd.topics import PROGRESS
from beholder_amd.transport.amqp.broker import BrokerThread

from helpers import progress_msg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_strip_workers_arg():
    assert strip_workers_arg(["run", "--workers", "3", "--x"]) == ["run", "--x"]
    assert strip_workers_arg(["run", "--workers=3"]) == ["run"]


def test_two_workers_share_the_queue(tmp_path):
    cfg = tmp_path / "events.yaml"
    cfg.write_text("keys: {trello: {key: k, token: t}}\ninstance: {flow_ids: {}}\n"
                   "service: {store: {backend: memory}, metrics: {enabled: false}, log: {level: warn}}\n")
    with BrokerThread() as bt:
        env = dict(os.environ, PYTHONPATH=ROOT)
        p = subprocess.Popen([sys.executable, "-m", "beholder_amd", "run", "--config", str(cfg), "--source", "amqp",
                              "--url", bt.url, "--workers", "2"], env=env, cwd=ROOT,
                             stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        try:
            deadline = time.time() + 60
            while time.time() < deadline:
                q = bt.call(lambda b: b.queues.get(PROGRESS))
                if q is not None and len(q.consumers) == 2:
                    break
                time.sleep(0.1)
            else:
                raise AssertionError("workers did not both subscribe")
            bodies = [progress_msg("missing", "QUEUED", i) for i in range(400)]
            bt.call(lambda b: [b.publish(PROGRESS, x) for x in bodies])
            while time.time() < deadline:
                st = bt.call(lambda b: b.stats(PROGRESS))
                if st["acked"] == 400:
                    break
                time.sleep(0.1)
            assert st["acked"] == 400 and st["consumers"] == 2
        finally:
            p.send_signal(signal.SIGTERM)
            rc = p.wait(60)
        assert rc == 0, p.stderr.read().decode()[-3000:]


def test_aggregate_merge_rules():
    from beholder_amd.metrics.aggregate import aggregate
    w0 = ("# HELP beholder_trello_comments Number of comments crreated\n# TYPE beholder_trello_comments counter\n"
          "beholder_trello_comments 3\n"
          "# HELP lat Latency\n# TYPE lat histogram\nlat_bucket{le=\"0.1\"} 1\nlat_bucket{le=\"+Inf\"} 2\n"
          "lat_sum 0.5\nlat_count 2\n"
          "# HELP process_start_time_seconds Start\n# TYPE process_start_time_seconds gauge\n"
          "process_start_time_seconds 200\n"
          "# HELP python_info Info\n# TYPE python_info gauge\npython_info{version=\"3.10\"} 1\n")
    w1 = w0.replace("beholder_trello_comments 3", "beholder_trello_comments 4").replace(
        "process_start_time_seconds 200", "process_start_time_seconds 100") + \
        "# HELP beholder_inflight In flight\n# TYPE beholder_inflight gauge\nbeholder_inflight 7\n"
    m = parse_exposition(aggregate([w0, w1]))
    assert m["beholder_trello_comments"] == 7
    assert m['lat_bucket{le="0.1"}'] == 2 and m['lat_bucket{le="+Inf"}'] == 4 and m["lat_count"] == 4
    assert m["lat_sum"] == 1.0
    assert m["process_start_time_seconds"] == 100  # min
    assert m['python_info{version="3.10"}'] == 1   # first
    assert m["beholder_inflight"] == 7            # present in one worker only
    text = aggregate([w0, w1])
    assert text.count("# TYPE beholder_trello_comments counter") == 1


def _free_port(span: int = 1) -> int:
    """A port P with P .. P+span-1 all free. The supervisor puts worker i on P+1+i, so the whole
    span must be free; it is taken below the kernel's ephemeral range, where the outgoing
    connections of tests running in parallel never land."""
    import random
    import socket
    rnd = random.Random(os.getpid() ^ time.monotonic_ns())
    for _ in range(200):
        base = rnd.randrange(20000, 32000 - span)
        socks = []
        try:
            for k in range(span):
                s = socket.socket()
                socks.append(s)
                s.bind(("127.0.0.1", base + k))
            return base
        except OSError:
            continue
        finally:
            for s in socks:
                s.close()
    raise RuntimeError("no free port span")


def test_workers_merged_metrics_endpoint(tmp_path):
    """One scrape target for N workers: the supervisor merges the workers' registries."""
    import urllib.error
    import urllib.request
    port = _free_port(3)  # the merged endpoint and the two workers' own
    cfg = tmp_path / "events.yaml"
    cfg.write_text("keys: {trello: {key: k, token: t}}\ninstance: {flow_ids: {}}\n"
                   f"service: {{store: {{backend: memory}}, metrics: {{enabled: true, host: 127.0.0.1, "
                   f"port: {port}}}, log: {{level: warn}}}}\n")
    with BrokerThread() as bt:
        env = dict(os.environ, PYTHONPATH=ROOT)
        p = subprocess.Popen([sys.executable, "-m", "beholder_amd", "run", "--config", str(cfg), "--source", "amqp",
                              "--url", bt.url, "--workers", "2"], env=env, cwd=ROOT,
                             stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        try:
            deadline = time.time() + 60
            while time.time() < deadline:
                q = bt.call(lambda b: b.queues.get(PROGRESS))
                if q is not None and len(q.consumers) == 2:
                    break
                time.sleep(0.1)
            bodies = [progress_msg("missing", "QUEUED", i) for i in range(300)]
            bt.call(lambda b: [b.publish(PROGRESS, x) for x in bodies])
            while time.time() < deadline and bt.call(lambda b: b.stats(PROGRESS))["acked"] < 300:
                time.sleep(0.1)
            # a worker whose scrape times out on a loaded host is left out of that one merge (and
            # reported by beholder_cluster_worker_up): scrape until both are in
            while True:
                text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
                m = parse_exposition(text)
                if m.get('beholder_progress_updates_total{status="queued"}') == 300 or time.time() > deadline:
                    break
                time.sleep(0.2)
            health = None
            while health != 200 and time.time() < deadline:  # a loaded host can answer late once
                try:
                    health = urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=5).status
                except urllib.error.HTTPError as e:
                    health = e.code
                    time.sleep(0.2)
        finally:
            p.send_signal(signal.SIGTERM)
            rc = p.wait(60)
        assert rc == 0, p.stderr.read().decode()[-3000:]
    m = parse_exposition(text)
    assert m['beholder_progress_updates_total{status="queued"}'] == 300  # summed over both workers
    assert m['beholder_messages_received{topic="v1.telemetry.progress"}'] == 300
    assert health == 200


# A stand-in worker program: worker 0 crashes (exit 3) after CRASH_AFTER_S, every other worker
# runs until SIGTERM. Each start of worker 0 appends a line to $STARTS.
FAKE_WORKER = r"""
import os, signal, sys, time
wid = os.environ["BEHOLDER_WORKER_ID"]
with open(os.environ["STARTS"], "a") as f:
    f.write(f"{wid} {os.getpid()}\n")
if wid == "0":
    time.sleep(float(os.environ["CRASH_AFTER_S"]))
    sys.exit(3)
signal.signal(signal.SIGTERM, lambda *a: sys.exit(0))
while True:
    time.sleep(0.05)
"""


def _supervise(tmp_path, crash_after_s, crashes_wanted, timeout_s, **policy):
    import threading
    from beholder_amd.parallel.workers import Supervisor
    starts = tmp_path / "starts"
    starts.write_text("")
    env = dict(os.environ, STARTS=str(starts), CRASH_AFTER_S=str(crash_after_s))
    logs = []
    sup = Supervisor([], 2, env=env, log=logs.append, command=[sys.executable, "-c", FAKE_WORKER],
                     backoff_base_s=0.01, backoff_max_s=0.05, poll_s=0.01, grace_s=5, **policy)
    t0 = time.monotonic()

    def watch():
        while time.monotonic() - t0 < timeout_s and not sup._stop:
            if sup.restarts[0] >= crashes_wanted:
                break
            time.sleep(0.01)
        sup.stop()
    th = threading.Thread(target=watch, daemon=True)
    th.start()
    rc = sup.run()
    th.join()
    lines = [x.split() for x in starts.read_text().splitlines()]
    return rc, sup, lines, logs


def test_spaced_crashes_never_stop_the_supervisor(tmp_path):
    """12 crashes, each after the worker ran longer than the window: no crash loop; the other
    worker keeps running the whole time (one process, never restarted); stop exits 0."""
    rc, sup, lines, logs = _supervise(tmp_path, crash_after_s=0.25, crashes_wanted=12, timeout_s=60,
                                      max_restarts=3, restart_window_s=0.2, healthy_s=10.0)
    assert sup.restarts[0] >= 12 and sup.restarts[1] == 0
    assert len({pid for wid, pid in lines if wid == "1"}) == 1
    assert rc == 0, logs
    assert not any("crash loop" in m for m in logs)


def test_backoff_starts_over_after_a_healthy_run():
    from beholder_amd.parallel.workers import RestartPolicy
    p = RestartPolicy(max_restarts=5, restart_window_s=100.0, healthy_s=10.0, backoff_base_s=1.0, backoff_max_s=30.0)
    assert [p.on_crash(0, started_at=t, now=t + 1) for t in (0, 2, 4)] == [1.0, 2.0, 4.0]
    assert p.on_crash(0, started_at=10, now=25) == 1.0  # ran 15 s > healthy_s: back to the base delay
    assert p.recent(0) == 1 and p.total[0] == 4


def test_crash_loop_stops_everything_with_exit_1(tmp_path):
    """A worker that dies at once, over and over: more than max_restarts crashes within the
    window stops the supervisor, SIGTERMs the healthy worker and exits 1."""
    rc, sup, lines, logs = _supervise(tmp_path, crash_after_s=0.0, crashes_wanted=100, timeout_s=30,
                                      max_restarts=3, restart_window_s=30.0, healthy_s=10.0)
    assert rc == 1
    assert sup.restarts[0] == 4 and any("crash loop" in m for m in logs)
    assert sup.procs == {} or all(p.poll() is not None for p in sup.procs.values())


def test_workers_config_is_validated():
    import pytest
    from beholder_amd.config import ConfigError
    from helpers import cfg
    assert cfg().data["service"]["workers"]["max_restarts"] == 10
    for k, bad in (("max_restarts", -1), ("restart_window_s", 0), ("healthy_s", "x")):
        with pytest.raises(ConfigError, match=f"service.workers.{k}"):
            cfg({"service": {"workers": {k: bad}}})


import pytest  # noqa: E402


@pytest.mark.parametrize("broker", ["native", "python"])
def test_shared_queue_two_workers_ack_every_event_exactly_once(broker):
    """The bench's shared-queue phase: `run --workers 2` on one broker queue;
    the broker counts every ack per event: all published events acked, none twice, none lost,
    no ack of an unknown tag, and both workers got deliveries."""
    from beholder_amd.bench.shared_queue import run_shared
    r = run_shared(2, 6000, broker=broker)
    assert r["supervisor_rc"] == 0 and r["broker"] == broker, r.get("supervisor_stderr")
    assert r["published"] == r["acked"] == 6000
    assert r["dup_acks"] == 0 and r["lost"] == 0 and r["unknown_acks"] == 0 and r["exactly_once"]
    assert r["connections"] == 2 and len(r["per_connection_delivered"]) == 2
    assert all(n > 0 for n in r["per_connection_delivered"]) and sum(r["per_connection_delivered"]) == 6000
    assert r["events_per_sec"] > 0 and r["broker_cpu_us_per_event"] > 0


def test_worker_command_is_the_service_unless_a_wrapper_opts_in(monkeypatch):
    """Workers run ``python -m beholder_amd`` whatever module hosts the supervisor (a
    launcher or test runner must not be restarted in its place); a wrapper entry that must be in
    force in every worker (the bench's shared_worker) names itself in BEHOLDER_WORKER_MODULE."""
    import types

    from beholder_amd import cli
    fake = types.ModuleType("__main__")
    fake.__spec__ = types.SimpleNamespace(name="some.launcher")
    monkeypatch.setitem(sys.modules, "__main__", fake)
    monkeypatch.delenv(cli.WORKER_MODULE_ENV, raising=False)
    assert cli.worker_command() == [sys.executable, "-m", "beholder_amd"]
    monkeypatch.setenv(cli.WORKER_MODULE_ENV, "beholder_amd.bench.shared_worker")
    assert cli.worker_command() == [sys.executable, "-m", "beholder_amd.bench.shared_worker"]
    monkeypatch.setenv(cli.WORKER_MODULE_ENV, " ")
    assert cli.worker_command() == [sys.executable, "-m", "beholder_amd"]


@pytest.mark.parametrize("broker", ["native", "python"])
def test_shared_queue_worker_crash_requeues_and_still_acks_every_event_once(broker):
    """A worker SIGKILLed mid-stream: the supervisor restarts it, the broker requeues the dead
    connection's un-acked deliveries (redelivered, as RabbitMQ does), and at the broker every
    published event ends up acked exactly once (the reference's at-least-once consumption with
    no loss: index.js acks after the handler, so nothing un-acked is lost)."""
    from beholder_amd.bench.shared_queue import run_shared
    r = run_shared(2, 60000, kill_one_after=4000, broker=broker)
    assert r.get("killed_worker_pid"), r
    assert r["supervisor_rc"] == 0, r.get("supervisor_stderr")
    assert r["published"] == r["acked"] == 60000 and r["lost"] == 0 and r["unknown_acks"] == 0
    assert r["dup_acks"] == 0 and r["exactly_once"]
    assert r["redelivered"] > 0  # the dead connection's un-acked deliveries went to the other worker


def test_native_shared_broker_ack_accounting_and_requeue():
    """SharedBroker (ops/csrc_bench/shared_broker.cpp) spoken to by the service's own AMQP client:
    the window is prefetch x consumers, single and multiple acks settle what they name, an ack of
    an unknown or already settled tag is counted, and deliveries a closed connection left un-acked
    go to the next consumer marked redelivered."""
    import array
    import asyncio
    import threading

    from beholder_amd.ops.bench_native import SharedBroker
    from beholder_amd.transport.amqp import wire
    from beholder_amd.transport.amqp.connection import Connection

    names = ("q.a", "q.b")
    events = [(names[i % 2], b"body-%d" % i) for i in range(40)]
    pieces = [wire.encode_content(1, 60, b, None, 131072) for _, b in events]
    offs = array.array("Q", [0])
    for p in pieces:
        offs.append(offs[-1] + len(p))
    b = SharedBroker(b"".join(pieces), offs.tobytes(), bytes(names.index(q) for q, _ in events), names, 1)
    port = b.listen()
    t = threading.Thread(target=b.run, args=(0.05,), daemon=True)
    t.start()

    async def consume(prefetch, take, ack):
        conn = await Connection(f"amqp://guest:guest@127.0.0.1:{port}/").open()
        ch = await conn.channel()
        await ch.basic_qos(prefetch)
        got = []
        for q in names:
            await ch.queue_declare(q)
            await ch.basic_consume(q, lambda c, m, props, body: got.append((m.delivery_tag, m.redelivered, body)))
        for _ in range(200):
            if len(got) >= take:
                break
            await asyncio.sleep(0.01)
        await asyncio.sleep(0.05)
        n = len(got)
        ack(ch, got)
        await asyncio.sleep(0.05)
        await conn.close()
        return n, got

    async def go():
        # first consumer: window 2 x 3 = 6; acks tag 1, tags <= 3 (multiple), tag 2 again, tag 99; the
        # rest stays un-acked until it closes
        def ack1(ch, got):
            ch.basic_ack(1)
            ch.basic_ack(3, multiple=True)
            ch.basic_ack(2)
            ch.basic_ack(99)
        n1, got1 = await consume(3, 6, ack1)
        # second consumer: gets the 3 requeued ones first (redelivered), then the rest; acks all
        n2, got2 = await consume(100, 37, lambda ch, got: ch.basic_ack(len(got), multiple=True))
        return n1, got1, n2, got2
    n1, got1, n2, got2 = asyncio.run(go())
    t.join(10)
    st = b.stats()
    assert n1 == 6  # prefetch 3 per consumer x 2 consumers on the channel
    k = len(got1) - 3  # un-acked at close (the acks freed room for more deliveries before it)
    assert k >= 3 and all(r for _, r, _ in got2[:k]) and not any(r for _, r, _ in got2[k:])
    assert {x for _, _, x in got2[:k]} == {x for _, _, x in got1[3:]}
    assert n2 == 37 and st["published"] == st["acked"] == 40 and st["finished"]
    assert st["unknown_acks"] == 2 and st["dup_acks"] == 0 and st["lost"] == 0 and st["redelivered"] == k
    assert st["per_conn"] == [len(got1), 37] and st["broker_s"] > 0
