"""Service discovery — parity with ``triton-core/dynamics`` (``dyn('rabbitmq')``, index.js:16,43).

triton-core is not vendored, so the resolution rules are ours [inferred]:

1. ``$<NAME>_ENDPOINT`` (e.g. ``RABBITMQ_ENDPOINT=amqp://user:pw@mq:5672/``);
2. ``$BEHOLDER_<NAME>_URL``;
3. ``service.dynamics.<name>`` from the loaded config;
4. a built-in default for the triton stack's in-cluster service names.
"""
from __future__ import annotations

import os
from typing import Mapping, Optional

DEFAULTS = {
    "rabbitmq": "amqp://guest:guest@127.0.0.1:5672/",
    "postgres": "postgres://postgres@127.0.0.1:5432/media",
    "minio": "http://127.0.0.1:9000",
}


def dyn(name: str, env: Optional[Mapping[str, str]] = None, config=None) -> str:
    """Resolve the endpoint for service ``name``."""
    env = os.environ if env is None else env
    key = name.upper().replace("-", "_")
    for var in (f"{key}_ENDPOINT", f"BEHOLDER_{key}_URL"):
        if env.get(var):
            return env[var]
    if config is not None:
        svc = config.data.get("service", {})
        dmap = svc.get("dynamics") or {}
        if dmap.get(name):
            return dmap[name]
    if name in DEFAULTS:
        return DEFAULTS[name]
    raise KeyError(f"no endpoint known for service '{name}' (set {key}_ENDPOINT)")
