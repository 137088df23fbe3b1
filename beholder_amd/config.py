"""Configuration loading — parity with ``triton-core/config`` as beholder uses it.

Reference behaviour (``/root/reference/index.js``):

* ``index.js:24`` — ``await Config('events')`` loads the config *named* ``events``.
* ``index.js:25`` — ``config.keys.trello.key`` / ``.token`` are dereferenced
  unconditionally at startup (a missing ``keys.trello`` object is a startup error).
* ``index.js:60`` — ``config.instance.flow_ids`` maps lower-case status → Trello list id.
* ``index.js:97-115`` — telegram / emby keys are read lazily inside the status handler.
* ``index.js:70`` — ``process.env.NO_TRELLO``: any *non-empty* value is truthy (JS
  string semantics, so ``"0"`` is true and ``""`` is false).

The file format is YAML (a JSON file is valid YAML too). Search order for a
config named ``<name>``:

1. an explicit ``path`` argument (``--config`` on the CLI);
2. ``$BEHOLDER_CONFIG`` (a file path);
3. ``$CONFIG_PATH/<name>.yaml`` / ``.yml`` / ``.json``;
4. ``./config/<name>.yaml`` and ``/stack/config/<name>.yaml`` (the reference
   image installs the service under ``/stack``, ``Dockerfile:3-6``).

Environment overrides are applied on top: ``BEHOLDER_CFG__a__b__c=value`` sets
``a.b.c`` (the value is parsed as a YAML scalar, so ``true``/``42`` are typed).

Our own service knobs (transport, store, metrics port, prefetch, ...) live
under a ``service:`` section and have defaults (``SERVICE_DEFAULTS``); the
reference hard-codes them (prefetch 100 at ``index.js:43``).
"""
from __future__ import annotations

import copy
import os
from typing import Any, Iterable, Mapping, MutableMapping, Optional

import yaml

ENV_PREFIX = "BEHOLDER_CFG__"

#: Defaults for knobs the reference hard-codes or inherits from triton-core.
SERVICE_DEFAULTS: dict = {
    "service": {
        # index.js:43 — new AMQP(dyn('rabbitmq'), 100, 2, prom): prefetch 100.
        "prefetch": 100,
        # index.js:43 — third AMQP arg; we use it as the reconnect/redelivery retry budget.
        "retries": 2,
        "transport": {"kind": "amqp", "url": None},
        # AMQP consume topology (transport/amqp/topology.py); triton-core/amqp is not vendored, the
        # default is our guess: a durable queue per topic on the default exchange
        "amqp": {"exchange": "", "exchange_type": "topic", "exchange_durable": True, "queue_names": {},
                 "routing_keys": {}, "durable": True, "passive_declare": False, "queue_arguments": {}},
        # index.js:42 `new Storage()` is always Postgres (triton-core/db); dsn default: dyn('postgres')
        # table/columns: triton-core/db's schema is not vendored; defaults are our guess (store/schema.py)
        # spread_at: queries in flight on every open connection before the pool opens another
        # stall_timeout_s: a connection with queries in flight and no reply for this long is dropped
        # min_connections: opened at startup (null = pool_size), so the first burst is spread at once
        "store": {"backend": "postgres", "dsn": None, "pool_size": 4, "spread_at": 8, "create_schema": False,
                  "table": "media", "columns": {}, "stall_timeout_s": 30.0, "min_connections": None},
        # index.js:28 — Prom.expose(); port/host are [inferred] (triton-core not vendored).
        "metrics": {"enabled": True, "host": "0.0.0.0", "port": 3000, "default_metrics": True},
        # index.js:11-13 — pino logger named after the file basename.
        # positional_args: append (Q11 fix, extra args kept) | drop (pino@5's exact msg text)
        "log": {"level": "info", "name": "index.js", "positional_args": "append"},
        # outbound sink HTTP: `h1` = native-parsed keep-alive client (sinks/h1.py), `aiohttp` = library client
        # preconnect: connections opened per sink origin at startup (0 = on demand, as the reference)
        # max_connecting: connects + TLS handshakes in progress per origin; requests beyond it queue for
        # the first keep-alive connection that frees up or the next connect slot (h1 client)
        "http": {"timeout_s": 30.0, "client": "h1", "max_per_host": 100, "keepalive_s": 4.0, "preconnect": 0,
                 "preconnect_wait_s": 5.0, "max_connecting": 8},
        # `run --workers N` supervisor (parallel/workers.py): more than max_restarts crashes of one worker
        # within restart_window_s is a crash loop (all workers stop, exit 1); a worker that ran healthy_s
        # starts its backoff over
        "workers": {"max_restarts": 10, "restart_window_s": 300.0, "healthy_s": 60.0},
        # SURVEY §5 race detection: opt-in per-mediaId serialisation (default off = parity, Q9).
        "ordering": "none",
        # Q1: what to do with a status message whose handler threw.
        #   leave_unacked (parity) | nack_requeue | nack_drop
        "on_status_error": "leave_unacked",
        "endpoints": {
            "trello": "https://api.trello.com",
            "telegram": "https://api.telegram.org",
        },
        "shutdown_grace_s": 10.0,
        # gc.freeze() after init: long-lived startup objects leave the collected generations
        "gc_freeze": True,
        # per-message trace span at debug level (needs log.level: debug)
        "trace": False,
        # handlers compiled to native state machines (ops/csrc/py_handlers.cpp); false = handlers.py
        "native_handlers": True,
        # how inbound bodies are decoded (index.js:63,129): protobufjs = the reference library's reader
        # (malformed input reads, fails and logs exactly as protobufjs 6.8.8 does, ops/csrc/pbjs.hpp);
        # upb = google.protobuf's stricter acceptance rules
        "proto": {"dialect": "protobufjs"},
        # Jaeger spans per delivery (utils/tracing.py); JAEGER_* env variables override
        "tracing": {"enabled": False, "service_name": "beholder",
                    # jaeger-client's fallback when no remote sampler answers: 1 trace in 1000
                    "sampler": {"type": "probabilistic", "param": 0.001},
                    "agent": {"host": "127.0.0.1", "port": 6831}},
    }
}


class ConfigError(Exception):
    """Raised for a missing / malformed config (startup fails fast — documented fix of Q10)."""


class Node:
    """Read-only attribute + item view over a nested mapping.

    ``Node`` mimics JS object access: a missing attribute yields ``None`` (JS
    ``undefined``) instead of raising, so code can reproduce the reference's
    ``config.instance.telegram && config.instance.telegram.enabled`` guards. Use
    :meth:`require` where the reference dereferences unconditionally.
    """

    __slots__ = ("_d", "_path")

    def __init__(self, data: Mapping, path: str = ""):
        object.__setattr__(self, "_d", data)
        object.__setattr__(self, "_path", path)

    def __getattr__(self, key: str) -> Any:
        if key.startswith("__"):
            raise AttributeError(key)
        return self[key]

    def __getitem__(self, key: str) -> Any:
        d = self._d
        v = d.get(key) if (type(d) is dict or isinstance(d, Mapping)) else None
        if type(v) is dict or (v is not None and not isinstance(v, (str, int, float, bool, list))
                               and isinstance(v, Mapping)):
            return Node(v, f"{self._path}.{key}" if self._path else key)
        return v

    def __setattr__(self, key, value):  # pragma: no cover - guard
        raise AttributeError("config is read-only")

    def __contains__(self, key: str) -> bool:
        return key in self._d

    def __iter__(self):
        return iter(self._d)

    def __len__(self) -> int:
        return len(self._d)

    def __bool__(self) -> bool:
        # A present (even empty) JS object is truthy.
        return True

    def __eq__(self, other) -> bool:
        if isinstance(other, Node):
            return self._d == other._d
        return self._d == other

    def __repr__(self) -> str:
        return f"Node({self._path or '<root>'}: {dict(self._d)!r})"

    def keys(self):
        return self._d.keys()

    def items(self):
        return self._d.items()

    def get(self, key: str, default: Any = None) -> Any:
        v = self[key]
        return default if v is None else v

    def require(self, dotted: str) -> Any:
        """Dereference ``a.b.c`` the way JS does *without* optional chaining.

        Reaching *through* a missing object raises (JS ``TypeError: Cannot read
        property 'x' of undefined``); a missing leaf returns ``None``.
        """
        cur: Any = self._d
        parts = dotted.split(".")
        for i, p in enumerate(parts):
            if not isinstance(cur, Mapping):
                where = ".".join(parts[:i]) or "<root>"
                raise ConfigError(f"Cannot read property '{p}' of undefined ({where})")
            cur = cur.get(p)
        return Node(cur, dotted) if isinstance(cur, Mapping) else cur


def deep_merge(base: MutableMapping, over: Mapping) -> MutableMapping:
    """Recursively merge ``over`` into ``base`` (in place) and return ``base``."""
    for k, v in over.items():
        if isinstance(v, Mapping) and isinstance(base.get(k), MutableMapping):
            deep_merge(base[k], v)
        else:
            base[k] = copy.deepcopy(v)
    return base


def _set_path(d: MutableMapping, parts: Iterable[str], value: Any) -> None:
    parts = list(parts)
    cur = d
    for p in parts[:-1]:
        nxt = cur.get(p)
        if not isinstance(nxt, MutableMapping):
            nxt = {}
            cur[p] = nxt
        cur = nxt
    cur[parts[-1]] = value


def env_overrides(env: Mapping[str, str]) -> dict:
    """Collect ``BEHOLDER_CFG__a__b=v`` overrides into a nested dict."""
    out: dict = {}
    for k, v in env.items():
        if not k.startswith(ENV_PREFIX):
            continue
        parts = [p for p in k[len(ENV_PREFIX):].split("__") if p]
        if not parts:
            continue
        try:
            val = yaml.safe_load(v) if v != "" else ""
        except yaml.YAMLError:
            val = v
        _set_path(out, parts, val)
    return out


def find_config_file(name: str, env: Mapping[str, str], cwd: Optional[str] = None) -> Optional[str]:
    cands = []
    if env.get("BEHOLDER_CONFIG"):
        cands.append(env["BEHOLDER_CONFIG"])
    roots = []
    if env.get("CONFIG_PATH"):
        roots.append(env["CONFIG_PATH"])
    roots.append(os.path.join(cwd or os.getcwd(), "config"))
    roots.append("/stack/config")
    for r in roots:
        for ext in (".yaml", ".yml", ".json"):
            cands.append(os.path.join(r, name + ext))
    for c in cands:
        if c and os.path.isfile(c):
            return c
    return None


def js_truthy_env(env: Mapping[str, str], key: str) -> bool:
    """``if (process.env.KEY)`` — any non-empty string is truthy (index.js:70)."""
    return bool(env.get(key, ""))


class Config:
    """Loaded configuration: the reference's keys plus our ``service`` section."""

    def __init__(self, data: Mapping, source: Optional[str] = None, env: Optional[Mapping[str, str]] = None):
        merged = deep_merge(copy.deepcopy(SERVICE_DEFAULTS), data or {})
        self._data = merged
        self.root = Node(merged)
        self.source = source
        self._env = dict(os.environ if env is None else env)
        self.validate()

    # -- construction -------------------------------------------------------
    @classmethod
    def load(cls, name: str = "events", path: Optional[str] = None,
             env: Optional[Mapping[str, str]] = None, cwd: Optional[str] = None) -> "Config":
        """``Config('events')`` (index.js:24)."""
        env = dict(os.environ if env is None else env)
        fpath = path or find_config_file(name, env, cwd)
        data: dict = {}
        if fpath:
            try:
                with open(fpath, "r", encoding="utf-8") as f:
                    loaded = yaml.safe_load(f)
            except OSError as e:
                raise ConfigError(f"cannot read config {fpath}: {e}") from e
            except yaml.YAMLError as e:
                raise ConfigError(f"invalid YAML in {fpath}: {e}") from e
            if loaded is None:
                loaded = {}
            if not isinstance(loaded, Mapping):
                raise ConfigError(f"config {fpath} must be a mapping, got {type(loaded).__name__}")
            data = dict(loaded)
        elif path:
            raise ConfigError(f"config file not found: {path}")
        deep_merge(data, env_overrides(env))
        if not fpath and not data:
            raise ConfigError(
                f"no config named '{name}' found (set --config, BEHOLDER_CONFIG or CONFIG_PATH)")
        return cls(data, source=fpath, env=env)

    @classmethod
    def from_dict(cls, data: Mapping, env: Optional[Mapping[str, str]] = None) -> "Config":
        return cls(copy.deepcopy(dict(data)), env=env if env is not None else {})

    # -- validation ---------------------------------------------------------
    def validate(self) -> None:
        # index.js:25 dereferences config.keys.trello.{key,token} unconditionally.
        self.root.require("keys.trello.key")
        self.root.require("keys.trello.token")
        # index.js:60 — `config.instance.flow_ids` is read at startup (needs `instance`).
        self.root.require("instance.flow_ids")
        svc = self._data["service"]
        if int(svc["prefetch"]) < 1:
            raise ConfigError("service.prefetch must be >= 1")
        if svc["ordering"] not in ("none", "per_media"):
            raise ConfigError("service.ordering must be 'none' or 'per_media'")
        if svc["on_status_error"] not in ("leave_unacked", "nack_requeue", "nack_drop"):
            raise ConfigError("service.on_status_error must be leave_unacked|nack_requeue|nack_drop")
        if svc["log"].get("positional_args", "append") not in ("append", "drop"):
            raise ConfigError("service.log.positional_args must be 'append' or 'drop'")
        if (svc.get("proto") or {}).get("dialect", "protobufjs") not in ("protobufjs", "upb"):
            raise ConfigError("service.proto.dialect must be 'protobufjs' or 'upb'")
        if svc["http"].get("client", "h1") not in ("h1", "aiohttp"):
            raise ConfigError("service.http.client must be 'h1' or 'aiohttp'")
        pc = svc["http"].get("preconnect", 0)
        if pc is None:
            pc = 0
        if isinstance(pc, bool) or not isinstance(pc, int) or pc < 0:
            raise ConfigError(f"service.http.preconnect must be an integer >= 0, got {pc!r}")
        wk = svc.get("workers") or {}
        for k, lo in (("max_restarts", 0), ("restart_window_s", 1e-9), ("healthy_s", 0)):
            v = wk.get(k, lo)
            if isinstance(v, bool) or not isinstance(v, (int, float)) or v < lo:
                raise ConfigError(f"service.workers.{k} must be a number >= {lo:g}, got {v!r}")
        mc = svc["http"].get("max_connecting", 8)
        if isinstance(mc, bool) or not isinstance(mc, int) or mc < 1:
            raise ConfigError(f"service.http.max_connecting must be an integer >= 1, got {mc!r}")
        pw = svc["http"].get("preconnect_wait_s", 5.0)
        if isinstance(pw, bool) or not isinstance(pw, (int, float)) or pw < 0:
            raise ConfigError(f"service.http.preconnect_wait_s must be a number >= 0, got {pw!r}")
        ca = svc["http"].get("ca_file")
        if ca is not None and (not isinstance(ca, str) or not os.path.isfile(ca)):
            raise ConfigError(f"service.http.ca_file: not a readable file: {ca!r}")
        from .store.schema import MediaSchema
        from .transport.amqp.topology import Topology
        try:
            Topology.from_config(svc.get("amqp"))
        except (TypeError, ValueError) as e:
            raise ConfigError(f"service.amqp: {e}") from None
        st = svc.get("store") or {}
        for k in ("pool_size", "spread_at"):
            v = st.get(k, 1)
            if isinstance(v, bool) or not isinstance(v, int) or v < 1:
                raise ConfigError(f"service.store.{k} must be an integer >= 1, got {v!r}")
        mc = st.get("min_connections")
        if mc is not None and (isinstance(mc, bool) or not isinstance(mc, int) or mc < 1):
            raise ConfigError(f"service.store.min_connections must be an integer >= 1 or null, got {mc!r}")
        stv = st.get("stall_timeout_s", 30.0)
        if stv is not None and (isinstance(stv, bool) or not isinstance(stv, (int, float)) or stv <= 0):
            raise ConfigError(f"service.store.stall_timeout_s must be a number > 0 or null, got {stv!r}")
        try:
            MediaSchema(st.get("table") or "media", st.get("columns") or {})
        except (TypeError, ValueError) as e:
            raise ConfigError(f"service.store: {e}") from None
        fl = self._data.get("instance", {}).get("flow_ids") if isinstance(self._data.get("instance"), Mapping) else None
        if fl is not None and not isinstance(fl, Mapping):
            raise ConfigError("instance.flow_ids must be a mapping of status -> list id")

    # -- accessors ------------------------------------------------------------
    def __getattr__(self, key: str) -> Any:
        if key.startswith("_"):
            raise AttributeError(key)
        return self.root[key]

    @property
    def data(self) -> dict:
        return self._data

    @property
    def service(self) -> Node:
        return self.root["service"]

    @property
    def env(self) -> Mapping[str, str]:
        return self._env

    @property
    def no_trello(self) -> bool:
        return js_truthy_env(self._env, "NO_TRELLO")

    @property
    def flow_ids(self) -> Optional[dict]:
        inst = self._data.get("instance")
        if not isinstance(inst, Mapping):
            return None
        fl = inst.get("flow_ids")
        return dict(fl) if isinstance(fl, Mapping) else fl
