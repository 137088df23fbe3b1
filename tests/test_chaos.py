"""Fault injection across every dependency at once.

The service consumes from a real AMQP broker, reads/writes a Postgres-protocol
store and calls HTTP sinks, all over TCP, while a chaos task repeatedly drops
broker, database and HTTP connections. Reference semantics under failure
(SURVEY.md §5 "failure detection / recovery"):

* progress messages are always acked once handled (Q7), and handling fails soft on DB or
  HTTP errors;
* a status message whose handler throws stays un-acked (Q1). The broker redelivers it when
  the channel dies, and a later attempt can succeed;
* AMQP reconnects with backoff, the Postgres pool replaces broken connections, and
  the HTTP client discards dead keep-alive connections.

Nothing may be lost. Every published message ends up acked, or, for Q1 status messages still
outstanding when the run stops, un-acked and held by the broker for redelivery.
"""
import asyncio
import os
import random

import pytest

from beholder_amd.utils import netconn

from beholder_amd.bench.http_sink_server import TLS_CERT, server_ssl_context
from beholder_amd.service import Service
from beholder_amd.sinks import H1Client
from beholder_amd.store import Media
from beholder_amd.store.postgres import PostgresStore
from beholder_amd.topics import PROGRESS, STATUS
from beholder_amd.transport.amqp import AmqpSource
from beholder_amd.transport.amqp.broker import AmqpBroker
from beholder_amd.utils.log import Logger, MemoryStream

from helpers import cfg, progress_msg, status_msg
from pg_fake import FakePg


class _HttpSink:
    """Keep-alive HTTP endpoint answering 200 {} that can drop all its connections."""

    def __init__(self, tls: bool = False):
        self.requests = 0
        self.writers = set()
        self.tls = tls

    async def start(self):
        self.server = await asyncio.start_server(self._serve, "127.0.0.1", 0,
                                                 ssl=server_ssl_context() if self.tls else None)
        self.url = f"{'https' if self.tls else 'http'}://127.0.0.1:{self.server.sockets[0].getsockname()[1]}"
        return self

    async def _serve(self, r, w):
        self.writers.add(w)
        try:
            while True:
                await r.readuntil(b"\r\n\r\n")
                self.requests += 1
                w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\n{}")
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.LimitOverrunError, OSError):
            pass
        finally:
            self.writers.discard(w)
            w.close()

    def drop(self):
        for w in list(self.writers):
            if w.transport is not None:
                w.transport.abort()

    async def stop(self):
        self.server.close()
        await self.server.wait_closed()


@pytest.mark.parametrize("tls", [False, True], ids=["plain", "tls"])
def test_chaos_every_dependency_drops_connections(tls):
    """``tls``: HTTPS sinks and Postgres sslmode=verify-full, i.e. every sink and DB connection on
    the native TLS path (ops/csrc/py_tls.cpp) while the chaos task drops them."""
    rng = random.Random(int(os.environ.get("BEHOLDER_CHAOS_SEED", "7")))  # other seeds: a longer hunt by hand
    n_progress, n_status = 1500, 150
    medias = [Media(id=f"m{i}", name=f"Show {i}", creator=1, creatorId=f"card{i}", metadataId=str(i),
                    status=i % 5) for i in range(50)]

    async def go():
        broker = await AmqpBroker().start()
        pg = await FakePg(auth="trust", ssl_context=server_ssl_context() if tls else None).start()
        sink = await _HttpSink(tls).start()
        try:
            dsn = f"{pg.dsn}?sslmode=verify-full&sslrootcert={TLS_CERT}" if tls else pg.dsn
            store = PostgresStore(dsn, create_schema=True, pool_size=2)
            await store.connect()
            for m in medias:
                await store.upsert(m)
            log = MemoryStream()
            c = cfg({"service": {"endpoints": {"trello": sink.url, "telegram": sink.url},
                                 "on_status_error": "leave_unacked"},
                     "instance": {"emby": {"host": sink.url}}})
            src = AmqpSource(broker.url, prefetch=50, backoff_initial=0.02, backoff_max=0.2)
            http = H1Client(timeout_s=5, ssl_cafile=TLS_CERT if tls else None)
            svc = Service(c, source=src, store=store, http=http, logger=Logger(stream=log),
                          serve_metrics=False)
            await svc.init()
            run = asyncio.ensure_future(svc.run())

            hits = []

            async def fire(what):
                hits.append(what)
                if what == "amqp":
                    await broker.drop_connections()
                elif what == "pg":
                    pg.drop_connections()
                else:
                    sink.drop()

            async def chaos():  # drops at random times, in flight or not
                while True:
                    await asyncio.sleep(rng.uniform(0.03, 0.12))
                    await fire(rng.choice(("amqp", "pg", "http", "pg", "http")))

            # and one drop per 50 messages while they are being published, every kind in turn: a
            # seed whose random drops come late (a loop busy with TLS handshakes) still hits each
            # dependency with deliveries in flight
            turns = ["amqp", "pg", "http", "pg", "http"]
            rng.shuffle(turns)
            monkey = asyncio.ensure_future(chaos())
            for i in range(n_progress):
                broker.publish(PROGRESS, progress_msg(f"m{i % 50}", "CONVERTING", i % 101, f"w{i % 3}"))
                if i % 10 == 0:
                    broker.publish(STATUS, status_msg(f"m{(i // 10) % 50}", "DEPLOYED"))
                if i % 50 == 49:
                    await asyncio.sleep(rng.uniform(0.01, 0.05))  # ~1.5 s of traffic
                    await fire(turns[(i // 50) % len(turns)])
            # the random drops go on a little past the last publish, then stop: drops every ~75 ms
            # until the end would redeliver the window faster than a loaded machine (the pure
            # Python I/O path under pytest -n, test_native_io_matrix) works through it
            await asyncio.sleep(0.3)
            monkey.cancel()
            deadline = asyncio.get_running_loop().time() + 30
            while asyncio.get_running_loop().time() < deadline:
                if broker.stats(PROGRESS)["acked"] >= n_progress:
                    break
                await asyncio.sleep(0.05)
            # one clean redelivery round: Q1 status messages still un-acked come back once more
            await broker.drop_connections()
            deadline = asyncio.get_running_loop().time() + 10
            while asyncio.get_running_loop().time() < deadline:
                st = broker.stats(STATUS)
                if st["acked"] >= n_status:
                    break
                await asyncio.sleep(0.05)
            if tls and netconn.enabled():  # the sink and DB connections were native TLS ones
                assert http._native_tls().stats["handshakes"] >= 1
                assert all(c._net is not None and c._net.tls for c in store._pool._conns if not c.closed)
            svc.request_stop()
            try:
                stats = await asyncio.wait_for(asyncio.shield(run), 15)
            except asyncio.TimeoutError:  # diagnostics for a shutdown that does not finish
                stacks = []
                for t in asyncio.all_tasks():
                    fr = t.get_stack(limit=3)
                    stacks.append(f"{t.get_coro()!r}: " + " <- ".join(f"{f.f_code.co_name}:{f.f_lineno}" for f in fr))
                waiters = {k: (len(o.waiters), sum(1 for w in o.waiters if not w.done()), o.open, o.connecting,
                               len(o.idle)) for k, o in http._origins.items()}
                pool = store._pool
                pgc = [(c.closed, getattr(c._net, "pending", None), len(c._pending)) for c in pool._conns] if pool else None
                raise AssertionError(f"service did not stop: inflight={len(svc._inflight)} "
                                     f"http={http.stats()} waiters={waiters} dials={len(http._dials)} "
                                     f"busy={len(http._busy)} pg={pgc} source={src.stats()}\n"
                                     + "\n".join(stacks)) from None
            await svc.close()
            return broker.stats(PROGRESS), broker.stats(STATUS), stats, src.reconnects, pg.connections, \
                sink.requests, hits
        finally:
            await sink.stop()
            await pg.stop()
            await broker.stop()

    prog, stat, stats, reconnects, pg_conns, http_requests, hits = asyncio.run(asyncio.wait_for(go(), 90))
    assert len(hits) >= 8 and {"amqp", "pg", "http"} <= set(hits), hits
    assert reconnects >= 1 and pg_conns > 2  # the chaos actually hit the AMQP and Postgres links
    assert prog["published"] == n_progress and prog["acked"] == n_progress, prog
    # no status message lost: acked, or still held by the broker for redelivery (Q1)
    assert stat["published"] == n_status
    assert stat["acked"] + stat["depth"] + stat["unacked"] == n_status, stat
    assert stat["acked"] >= n_status * 0.9, stat
    assert http_requests >= n_progress  # every progress comment attempted at least once
