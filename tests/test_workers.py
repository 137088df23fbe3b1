"""`run --workers N`: supervised competing-consumer processes on one AMQP queue."""
import os
import signal
import subprocess
import sys
import time

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
