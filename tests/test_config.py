"""Config loading (index.js:24-25,60,70,97-115)."""
import os

import pytest

from beholder_amd.config import Config, ConfigError, env_overrides, js_truthy_env
from beholder_amd.dynamics import dyn

MIN = "keys:\n  trello: {key: k, token: t}\ninstance:\n  flow_ids: {queued: L1}\n"


def test_load_by_name_from_config_path(tmp_path):
    (tmp_path / "events.yaml").write_text(MIN)
    c = Config.load("events", env={"CONFIG_PATH": str(tmp_path)})
    assert c.keys.trello.key == "k" and c.flow_ids == {"queued": "L1"}
    assert c.source.endswith("events.yaml")
    assert c.service.prefetch == 100  # index.js:43 default


def test_explicit_path_and_json(tmp_path):
    p = tmp_path / "x.json"
    p.write_text('{"keys": {"trello": {"key": "a", "token": "b"}}, "instance": {"flow_ids": {}}}')
    assert Config.load(path=str(p), env={}).keys.trello.token == "b"


def test_env_overrides_typed(tmp_path):
    (tmp_path / "events.yaml").write_text(MIN)
    env = {"CONFIG_PATH": str(tmp_path), "BEHOLDER_CFG__instance__telegram__enabled": "true",
           "BEHOLDER_CFG__service__prefetch": "7", "BEHOLDER_CFG__keys__trello__token": "override"}
    c = Config.load(env=env)
    assert c.instance.telegram.enabled is True and c.service.prefetch == 7 and c.keys.trello.token == "override"
    assert env_overrides({"BEHOLDER_CFG__a__b": "x"}) == {"a": {"b": "x"}}


def test_missing_config_and_bad_yaml(tmp_path):
    with pytest.raises(ConfigError):
        Config.load(env={"CONFIG_PATH": str(tmp_path)}, cwd=str(tmp_path))
    (tmp_path / "events.yaml").write_text("keys: [unclosed")
    with pytest.raises(ConfigError):
        Config.load(env={"CONFIG_PATH": str(tmp_path)})
    with pytest.raises(ConfigError):
        Config.load(path=str(tmp_path / "nope.yaml"), env={})


def test_required_keys_like_reference():
    with pytest.raises(ConfigError, match="trello"):
        Config.from_dict({"instance": {"flow_ids": {}}})
    # keys.trello present with missing leaf values is fine (JS reads undefined)
    Config.from_dict({"keys": {"trello": {}}, "instance": {"flow_ids": {}}})


def test_js_style_missing_values():
    c = Config.from_dict({"keys": {"trello": {"key": "k"}}, "instance": {"flow_ids": {}}})
    assert c.instance.telegram is None and c.keys.emby is None
    assert bool(c.instance) is True


def test_validation_of_service_knobs():
    base = {"keys": {"trello": {}}, "instance": {"flow_ids": {}}}
    for bad in ({"prefetch": 0}, {"ordering": "weird"}, {"on_status_error": "explode"}):
        with pytest.raises(ConfigError):
            Config.from_dict({**base, "service": bad})


def test_no_trello_flag():
    base = {"keys": {"trello": {}}, "instance": {"flow_ids": {}}}
    assert Config.from_dict(base, env={"NO_TRELLO": "1"}).no_trello
    assert not js_truthy_env({"NO_TRELLO": ""}, "NO_TRELLO")


def test_dynamics():
    assert dyn("rabbitmq", env={"RABBITMQ_ENDPOINT": "amqp://x"}) == "amqp://x"
    assert dyn("rabbitmq", env={}).startswith("amqp://")
    with pytest.raises(KeyError):
        dyn("unknown-service", env={})


def test_repo_example_config_loads():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    c = Config.load(path=os.path.join(root, "config", "events.example.yaml"), env={})
    assert "deployed" in c.flow_ids


def test_repo_has_no_unused_imports():
    """`make lint` (scripts/lint.py): pyflakes is not installed in the image."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "lint.py"), "beholder_amd", "tests",
                        "bench.py", "__graft_entry__.py", "scripts"], capture_output=True, text=True, cwd=root)
    assert r.returncode == 0, r.stdout


def test_kubernetes_example_config_loads(tmp_path):
    """deploy/kubernetes.yaml: the ConfigMap's events.yaml plus the Secret's env overrides make a
    valid config (keys reach the reference's key paths, index.js:25,100,110,115)."""
    import os
    import yaml
    from beholder_amd.config import Config
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    docs = list(yaml.safe_load_all(open(os.path.join(root, "deploy", "kubernetes.yaml"))))
    cm = next(d for d in docs if d["kind"] == "ConfigMap")
    secret = next(d for d in docs if d["kind"] == "Secret")
    (tmp_path / "events.yaml").write_text(cm["data"]["events.yaml"])
    cfg = Config.load("events", path=str(tmp_path / "events.yaml"), env=dict(secret["stringData"]))
    assert cfg.root.require("keys.trello").get("token") == "<trello token>"
    assert cfg.keys.emby.token == "<emby api key>" and cfg.flow_ids["deployed"] == "<list id>"
    assert cfg.data["service"]["prefetch"] == 100


def test_http_ca_file_reaches_the_native_tls_context(tmp_path):
    """service.http.ca_file: validated at load, handed to H1Client (ssl_cafile), mirrored by the
    native TLS context (sinks/h1.py _native_tls)."""
    from beholder_amd.bench.http_sink_server import TLS_CERT
    from beholder_amd.service import make_http_client
    base = {"keys": {"trello": {}}, "instance": {"flow_ids": {}}}
    with pytest.raises(ConfigError, match="ca_file"):
        Config.from_dict({**base, "service": {"http": {"ca_file": str(tmp_path / "missing.pem")}}})
    cfg = Config.from_dict({**base, "service": {"http": {"ca_file": TLS_CERT}}})
    c = make_http_client(cfg.data["service"]["http"])
    assert c.ssl_cafile == TLS_CERT and c._native_tls() is not None
    assert make_http_client({}).ssl_cafile is None
