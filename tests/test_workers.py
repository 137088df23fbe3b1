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


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_workers_merged_metrics_endpoint(tmp_path):
    """One scrape target for N workers: the supervisor merges the workers' registries."""
    import urllib.request
    port = _free_port()
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
            text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
            health = urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=5).status
        finally:
            p.send_signal(signal.SIGTERM)
            rc = p.wait(60)
        assert rc == 0, p.stderr.read().decode()[-3000:]
    m = parse_exposition(text)
    assert m['beholder_progress_updates_total{status="queued"}'] == 300  # summed over both workers
    assert m['beholder_messages_received{topic="v1.telemetry.progress"}'] == 300
    assert health == 200
