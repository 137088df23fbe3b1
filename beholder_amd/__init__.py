"""beholder_amd — telemetry events / metrics service for the triton media stack.

A from-scratch rebuild of ``tritonmedia/beholder`` (reference: a 160-line
Node.js AMQP consumer, ``/root/reference/index.js``). Layers:

* :mod:`~beholder_amd.config`, :mod:`~beholder_amd.dynamics` — L1 config / discovery
* :mod:`~beholder_amd.models`   — protobuf schema + codec (``triton-core/proto``)
* :mod:`~beholder_amd.ops`      — native C++ runtime: codec, ingest ring, deliveries, metrics, text
* :mod:`~beholder_amd.transport` — AMQP 0-9-1 / stdin / file / in-memory sources
* :mod:`~beholder_amd.store`    — media store (``triton-core/db``): memory / sqlite / postgres
* :mod:`~beholder_amd.sinks`    — Trello / Telegram / Emby HTTP sinks
* :mod:`~beholder_amd.metrics`  — Prometheus registry + exposer (``triton-core/prom``)
* :mod:`~beholder_amd.handlers` — the status / progress handlers (index.js:50-155)
* :mod:`~beholder_amd.service`  — ``init()`` + dispatch loop (index.js:23-160)
* :mod:`~beholder_amd.parallel` — per-media ordering, multi-process consumers
"""
__version__ = "1.0.0"
