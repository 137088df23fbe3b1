"""CLI: `gen | run --source stdin` (the BASELINE plumbing config) and tools."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT)


def cli(*args, **kw):
    return subprocess.run([sys.executable, "-m", "beholder_amd", *args], capture_output=True, env=ENV, cwd=ROOT,
                          timeout=120, **kw)


def test_gen_decode_roundtrip(tmp_path):
    out = tmp_path / "ev.bin"
    r = cli("gen", "--events", "25", "--media", "5", "--out", str(out), "--media-out", str(tmp_path / "m.json"))
    assert r.returncode == 0
    d = cli("decode", str(out))
    recs = [json.loads(x) for x in d.stdout.decode().splitlines()]
    assert len(recs) == 25 and all("json" in x for x in recs)
    assert len(json.load(open(tmp_path / "m.json"))) == 5


def test_run_stdin_plumbing(tmp_path):
    cfg = tmp_path / "events.yaml"
    cfg.write_text("keys: {trello: {key: k, token: t}}\ninstance: {flow_ids: {queued: L}}\n"
                   "service: {store: {backend: memory}, metrics: {enabled: false}, endpoints: {trello: 'http://127.0.0.1:9',"
                   " telegram: 'http://127.0.0.1:9'}, http: {timeout_s: 0.2}}\n")
    ev = cli("gen", "--events", "30", "--media", "4", "--media-out", str(tmp_path / "m.json"),
             "--progress-fraction", "1.0")
    r = cli("run", "--config", str(cfg), "--source", "stdin", "--media-fixture", str(tmp_path / "m.json"),
            "--stats", input=ev.stdout)
    assert r.returncode == 0, r.stderr
    stats = json.loads(r.stderr.decode().strip().splitlines()[-1])
    assert stats["source"]["acked"] == 30  # progress handler always acks (Q7), even with Trello down
    lines = [json.loads(x) for x in r.stdout.decode().splitlines()]
    assert lines[0]["msg"] == "initialized" and lines[0]["name"] == "index.js"
    # the unpinned transport / store layout is stated once, after index.js:157's line
    assert lines[1]["msg"].startswith("consuming from fd stdin") and "store memory (4 rows)" in lines[1]["msg"]


def test_run_config_error_exit_code(tmp_path):
    cfg = tmp_path / "bad.yaml"
    cfg.write_text("instance: {flow_ids: {}}\n")
    r = cli("run", "--config", str(cfg), "--source", "stdin", input=b"")
    assert r.returncode == 2 and b"config error" in r.stderr


def test_run_amqp_unreachable_fails_fast(tmp_path):
    """Q10 fix: a startup failure exits non-zero instead of an unhandled rejection."""
    cfg = tmp_path / "events.yaml"
    cfg.write_text("keys: {trello: {key: k, token: t}}\ninstance: {flow_ids: {}}\n"
                   "service: {store: {backend: memory}, metrics: {enabled: false}, retries: 0}\n")
    r = cli("run", "--config", str(cfg), "--source", "amqp", "--url", "amqp://guest:guest@127.0.0.1:1/")
    assert r.returncode == 1 and b"fatal" in r.stderr


def test_run_stdin_ndjson(tmp_path):
    cfg = tmp_path / "events.yaml"
    cfg.write_text("keys: {trello: {key: k, token: t}}\ninstance: {flow_ids: {}}\n"
                   "service: {store: {backend: memory}, metrics: {enabled: false}}\n")
    (tmp_path / "m.json").write_text('[{"id": "m1", "creator": 0}]')
    lines = "\n".join([
        '{"topic": "v1.telemetry.progress", "json": {"mediaId": "m1", "status": "CONVERTING", "progress": 40}}',
        'not json',
        '{"topic": "v1.telemetry.status", "json": {"mediaId": "m1", "status": "DEPLOYED"}}',
    ]) + "\n"
    r = cli("run", "--config", str(cfg), "--source", "stdin", "--format", "ndjson", "--media-fixture",
            str(tmp_path / "m.json"), "--stats", input=lines.encode())
    assert r.returncode == 0, r.stderr
    stats = json.loads(r.stderr.decode().strip().splitlines()[-1])
    assert stats["source"]["acked"] == 2 and stats["source"]["bad_lines"] == 1
    assert stats["progress_updates"] == {"converting": 1.0}


def test_run_corrupt_stream_exits_nonzero(tmp_path):
    cfg = tmp_path / "events.yaml"
    cfg.write_text("keys: {trello: {key: k, token: t}}\ninstance: {flow_ids: {}}\n"
                   "service: {store: {backend: memory}, metrics: {enabled: false}}\n")
    r = cli("run", "--config", str(cfg), "--source", "stdin", input=b"\x09\x00\x00\x00\x01abc")  # truncated frame
    assert r.returncode == 1
    assert b"ingest source failed" in r.stdout and b"truncated" in r.stdout


def test_seed_sqlite_and_publish_to_broker(tmp_path):
    from beholder_amd.topics import PROGRESS, STATUS
    from beholder_amd.transport.amqp.broker import BrokerThread
    ev = cli("gen", "--events", "40", "--media", "3", "--media-out", str(tmp_path / "m.json"), "--out",
             str(tmp_path / "ev.bin"))
    assert ev.returncode == 0
    db = tmp_path / "media.db"
    r = cli("seed", str(tmp_path / "m.json"), "--store", "sqlite", "--dsn", str(db))
    assert r.returncode == 0 and r.stdout.strip() == b"3"
    with BrokerThread() as bt:
        r = cli("publish", "--url", bt.url, str(tmp_path / "ev.bin"))
        assert r.returncode == 0 and r.stdout.strip() == b"40"
        depth = bt.call(lambda b: b.depth(STATUS) + b.depth(PROGRESS))
    assert depth == 40


def test_config_command_masks_secrets(tmp_path):
    cfg = tmp_path / "events.yaml"
    cfg.write_text("keys: {trello: {key: SECRETK, token: SECRETT}, telegram: {token: 'SECRET:TG'}}\n"
                   "instance: {flow_ids: {queued: L1}}\n"
                   "service: {store: {backend: postgres, dsn: 'postgres://u:SECRETPW@db/media'}}\n")
    r = cli("config", "--config", str(cfg))
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert b"SECRET" not in r.stdout
    assert out["config"]["instance"]["flow_ids"] == {"queued": "L1"}
    assert out["config"]["service"]["store"]["dsn"] == "postgres://u:***@db/media"
    assert out["config"]["service"]["prefetch"] == 100
