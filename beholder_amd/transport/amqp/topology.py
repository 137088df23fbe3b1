"""AMQP consume topology — what ``triton-core/amqp`` declares before ``listen`` (index.js:43-44,62,127).

triton-core is not vendored, so the broker-side layout the reference consumes from is unknown.
The default is our documented guess: one durable queue per topic, named after the topic, fed
through the default exchange (publishers use ``routing_key = topic``). Every part of it is a
knob (``service.amqp``), so a deployment can match whatever its publishers use::

    service:
      amqp:
        exchange: triton            # "" = the default exchange (no declare, no bind)
        exchange_type: topic        # direct | topic | fanout
        exchange_durable: true
        queue_names: {v1.telemetry.status: beholder.status}     # topic -> queue (default: topic)
        routing_keys: {v1.telemetry.status: ["v1.telemetry.status", "v1.telemetry.status.#"]}
        durable: true               # queue durability (must match an existing queue's)
        passive_declare: false      # true: only check that the exchange/queues exist
        queue_arguments: {}         # x-* arguments of queue.declare (e.g. x-dead-letter-exchange)

``passive_declare`` is the escape hatch for a topology owned by another service: the queues
are checked (``NOT_FOUND`` fails startup loudly) but never created or re-declared, so there
is no ``PRECONDITION_FAILED`` on an argument mismatch.
"""
from __future__ import annotations

from typing import Any, Dict, List, Mapping, Optional, Sequence

EXCHANGE_TYPES = ("direct", "topic", "fanout")


class Topology:
    def __init__(self, exchange: str = "", exchange_type: str = "topic", exchange_durable: bool = True,
                 queue_names: Optional[Mapping[str, str]] = None,
                 routing_keys: Optional[Mapping[str, Any]] = None, durable: bool = True,
                 passive_declare: bool = False, queue_arguments: Optional[Mapping[str, Any]] = None):
        if exchange_type not in EXCHANGE_TYPES:
            raise ValueError(f"amqp exchange_type must be one of {'|'.join(EXCHANGE_TYPES)}, not {exchange_type!r}")
        if routing_keys and not exchange:
            raise ValueError("amqp routing_keys need an exchange (the default exchange routes by queue name)")
        self.exchange = exchange or ""
        self.exchange_type = exchange_type
        self.exchange_durable = bool(exchange_durable)
        self.queue_names: Dict[str, str] = {str(k): str(v) for k, v in (queue_names or {}).items()}
        rk: Dict[str, List[str]] = {}
        for k, v in (routing_keys or {}).items():
            rk[str(k)] = [str(v)] if isinstance(v, str) else [str(x) for x in v]
        self.routing_keys = rk
        self.durable = bool(durable)
        self.passive = bool(passive_declare)
        self.queue_arguments = dict(queue_arguments or {})

    @classmethod
    def from_config(cls, d: Optional[Mapping[str, Any]]) -> "Topology":
        d = dict(d or {})
        known = {"exchange", "exchange_type", "exchange_durable", "queue_names", "routing_keys", "durable",
                 "passive_declare", "queue_arguments"}
        extra = set(d) - known
        if extra:
            raise ValueError(f"unknown service.amqp keys: {', '.join(sorted(extra))}")
        return cls(**d)

    def queue(self, topic: str) -> str:
        return self.queue_names.get(topic, topic)

    def keys(self, topic: str) -> List[str]:
        """Routing keys bound for ``topic`` (none on the default exchange)."""
        if not self.exchange:
            return []
        return self.routing_keys.get(topic, [topic])

    def publish_target(self, topic: str) -> tuple:
        """``(exchange, routing_key)`` a publisher uses so ``topic`` reaches this consumer: the
        first configured binding key that is a plain key (on a topic exchange, one without a
        ``*`` / ``#`` word), else the topic name (the default binding)."""
        if not self.exchange:
            return "", self.queue(topic)
        for k in self.routing_keys.get(topic, ()):
            if self.exchange_type != "topic" or not ({"*", "#"} & set(k.split("."))):
                return self.exchange, k
        return self.exchange, topic

    async def declare(self, ch, topics: Sequence[str]) -> None:
        """Declare (or, passively, check) the exchange, the queues and their bindings on ``ch``."""
        if self.exchange:
            await ch.exchange_declare(self.exchange, type=self.exchange_type, durable=self.exchange_durable,
                                      passive=self.passive)
        for t in topics:
            q = self.queue(t)
            await ch.queue_declare(q, durable=self.durable, passive=self.passive, arguments=self.queue_arguments)
            if self.exchange and not self.passive:
                for k in self.keys(t):
                    await ch.queue_bind(q, self.exchange, k)

    def describe(self, topics: Sequence[str]) -> str:
        """One line for the startup log: exchange, queue per topic, bindings, declare mode."""
        ex = (f"exchange={self.exchange}({self.exchange_type},{'durable' if self.exchange_durable else 'transient'})"
              if self.exchange else "exchange=(default)")
        qs = []
        for t in topics:
            keys = self.keys(t)
            qs.append(f"{t}->{self.queue(t)}" + (f"[{'|'.join(keys)}]" if keys else ""))
        mode = "passive" if self.passive else "declare"
        return (f"{ex} queues={','.join(qs)} queue_durable={str(self.durable).lower()} mode={mode}"
                + (f" queue_arguments={sorted(self.queue_arguments)}" if self.queue_arguments else ""))
