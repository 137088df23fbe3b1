"""Configurable AMQP consume topology (service.amqp) and media-table mapping (service.store).

Neither triton-core/amqp's queue layout (index.js:43-44,62,127) nor triton-core/db's media table
(index.js:42,68,76,140) is vendored, so both are knobs with our guess as the default. These
tests drive the knobs against the in-repo AMQP broker and the Postgres fake.
"""
import asyncio

import pytest

from beholder_amd import topics as T
from beholder_amd.config import ConfigError
from beholder_amd.service import Service, build_source
from beholder_amd.sinks import RecordingHttpClient
from beholder_amd.store import Media, MemoryStore, open_store
from beholder_amd.store.postgres import PostgresStore
from beholder_amd.store.schema import MediaSchema, pg_ph
from beholder_amd.transport.amqp import AmqpBroker
from beholder_amd.transport.amqp.source import AmqpPublisher
from beholder_amd.transport.amqp.topology import Topology
from beholder_amd.transport.amqp.wire import AmqpError
from beholder_amd.utils.log import Logger, MemoryStream

from helpers import cfg, progress_msg, status_msg, trello_media
from pg_fake import FakePg


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


TOPO = {"exchange": "triton", "exchange_type": "topic",
        "queue_names": {T.STATUS: "beholder.status", T.PROGRESS: "beholder.progress"},
        "routing_keys": {T.STATUS: [T.STATUS, "legacy.status.#"]}}


def _service(url, amqp, medias=(), retries=0, store=None):
    c = cfg({"service": {"amqp": amqp, "retries": retries, "transport": {"kind": "amqp", "url": url}}})
    stream = MemoryStream()
    log = Logger(stream=stream)
    src = build_source(c, log)
    svc = Service(c, source=src, store=store or MemoryStore(list(medias)), http=RecordingHttpClient(), logger=log,
                  serve_metrics=False)
    return svc, stream


async def _until(pred, timeout=5.0):
    t0 = asyncio.get_running_loop().time()
    while not pred():
        if asyncio.get_running_loop().time() - t0 > timeout:
            raise AssertionError("condition not reached")
        await asyncio.sleep(0.01)


def test_topic_exchange_bindings_route_to_the_consumer():
    async def go():
        broker = await AmqpBroker().start()
        try:
            svc, stream = _service(broker.url, TOPO, [trello_media("m1")])
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            assert broker.publish("legacy.status.v0", status_msg("m1", "CONVERTING"), exchange="triton") == 1
            assert broker.publish(T.STATUS, status_msg("m1", "UPLOADING"), exchange="triton") == 1
            assert broker.publish(T.PROGRESS, progress_msg("m1", "CONVERTING", 5), exchange="triton") == 1
            assert broker.publish("unbound.key", status_msg("m1", "QUEUED"), exchange="triton") == 0
            await _until(lambda: broker.stats("beholder.status")["acked"] == 2
                         and broker.stats("beholder.progress")["acked"] == 1)
            svc.request_stop()
            await task
            await svc.close()
            assert T.STATUS not in broker.queues and T.PROGRESS not in broker.queues  # nothing declared by topic
            return stream
        finally:
            await broker.stop()
    stream = run(go())
    msgs = [r["msg"] for r in stream.records()]
    line = next(m for m in msgs if m.startswith("consuming from amqp"))
    assert "exchange=triton(topic,durable)" in line
    assert f"{T.STATUS}->beholder.status[{T.STATUS}|legacy.status.#]" in line
    assert f"{T.PROGRESS}->beholder.progress[{T.PROGRESS}]" in line and "mode=declare" in line
    assert "store memory (1 rows)" in line


def test_publisher_with_the_same_topology_reaches_the_consumer():
    async def go():
        broker = await AmqpBroker().start()
        try:
            svc, _ = _service(broker.url, TOPO, [trello_media("m1")])
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            pub = await AmqpPublisher(broker.url, topology=Topology.from_config(TOPO)).connect()
            await pub.publish(T.PROGRESS, progress_msg("m1", "CONVERTING", 50), wait=True)
            await pub.close()
            await _until(lambda: broker.stats("beholder.progress")["acked"] == 1)
            svc.request_stop()
            await task
            await svc.close()
        finally:
            await broker.stop()
    run(go())


def test_publisher_uses_a_custom_binding_key():
    """with custom routing_keys only (the topic name is not bound), the publisher must
    route with a configured key, or its messages never reach the queue this consumer declared."""
    topo = {"exchange": "triton", "exchange_type": "topic",
            "routing_keys": {T.STATUS: ["beholder.status.*", "beholder.status"], T.PROGRESS: ["v1.#"]}}
    t = Topology.from_config(topo)
    assert t.publish_target(T.STATUS) == ("triton", "beholder.status")  # the wildcard key is skipped
    assert t.publish_target(T.PROGRESS) == ("triton", T.PROGRESS)        # only a pattern: the topic name
    assert Topology.from_config({"exchange": "x", "exchange_type": "direct",
                                 "routing_keys": {T.STATUS: ["k1", "k2"]}}).publish_target(T.STATUS) == ("x", "k1")

    async def go():
        broker = await AmqpBroker().start()
        try:
            svc, _ = _service(broker.url, topo, [trello_media("m1")])
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            pub = await AmqpPublisher(broker.url, topology=t).connect()
            await pub.publish(T.STATUS, status_msg("m1", "CONVERTING"), wait=True)
            await pub.publish(T.PROGRESS, progress_msg("m1", "CONVERTING", 5), wait=True)
            await pub.close()
            await _until(lambda: broker.stats(T.STATUS)["acked"] == 1 and broker.stats(T.PROGRESS)["acked"] == 1)
            svc.request_stop()
            await task
            await svc.close()
        finally:
            await broker.stop()
    run(go())


def test_passive_declare_fails_loudly_on_a_missing_queue():
    async def go():
        broker = await AmqpBroker().start()
        try:
            svc, _ = _service(broker.url, {"passive_declare": True})
            with pytest.raises(AmqpError, match="NOT_FOUND"):
                await svc.init()
            await svc.close()
        finally:
            await broker.stop()
    run(go())


def test_passive_declare_accepts_a_queue_owned_elsewhere():
    """A transient queue declared by another service: declaring it durable is PRECONDITION_FAILED,
    a passive declare just consumes from it."""
    async def go():
        broker = await AmqpBroker().start()
        try:
            for q in (T.STATUS, T.PROGRESS):
                pub = await AmqpPublisher(broker.url, durable=False).connect()
                await pub.publish(q, progress_msg("m1", "CONVERTING", 1) if q == T.PROGRESS else
                                  status_msg("m1", "QUEUED"), wait=True)
                await pub.close()
            bad, _ = _service(broker.url, {})
            with pytest.raises(AmqpError, match="PRECONDITION_FAILED"):
                await bad.init()
            await bad.close()
            svc, _ = _service(broker.url, {"passive_declare": True}, [trello_media("m1")])
            await svc.init()
            task = asyncio.ensure_future(svc.run())
            await _until(lambda: broker.stats(T.STATUS)["acked"] == 1 and broker.stats(T.PROGRESS)["acked"] == 1)
            svc.request_stop()
            await task
            await svc.close()
        finally:
            await broker.stop()
    run(go())


@pytest.mark.parametrize("amqp,match", [
    ({"exchnage": "x"}, "unknown service.amqp keys"),
    ({"routing_keys": {T.STATUS: "a"}}, "need an exchange"),
    ({"exchange": "x", "exchange_type": "headers"}, "exchange_type"),
])
def test_bad_amqp_topology_is_a_config_error(amqp, match):
    with pytest.raises(ConfigError, match=match):
        cfg({"service": {"amqp": amqp}})


@pytest.mark.parametrize("store,match", [
    ({"columns": {"creator_id": "x"}}, "unknown media field"),
    ({"columns": {"name": "bad name"}}, "invalid SQL identifier"),
    ({"columns": {"name": "status"}}, "distinct"),
    ({"table": "a.b.c"}, "invalid table name"),
])
def test_bad_store_mapping_is_a_config_error(store, match):
    with pytest.raises(ConfigError, match=match):
        cfg({"service": {"store": store}})


def test_default_schema_sql_is_the_documented_guess():
    s = MediaSchema()
    assert s.is_default
    assert s.select_by_id(pg_ph) == ('SELECT "id", "name", "creator", "creator_id", "type", "source", "source_uri", '
                                     '"metadata", "metadata_id", "status" FROM "media" WHERE "id" = $1')
    assert s.update_status(pg_ph) == 'UPDATE "media" SET "status" = $1 WHERE "id" = $2'


CAMEL = {"creatorId": "creatorId", "sourceURI": "sourceUri", "metadataId": "metadataId", "status": "state"}
M1 = Media(id="m1", name="Bebop", creator=1, creatorId="card", metadataId="7", status=2)


def test_sqlite_store_with_renamed_columns(tmp_path):
    async def go():
        st = open_store("sqlite", str(tmp_path / "m.db"), table="main.media_items", columns=CAMEL)
        await st.connect()
        await st.upsert(M1)
        await st.update_status("m1", 4)
        got = await st.get_by_id("m1")
        cols = [r[1] for r in st._conn.execute("PRAGMA table_info(media_items)").fetchall()]
        await st.close()
        return got, cols
    got, cols = run(go())
    assert got == M1._replace(status=4)
    assert cols == ["id", "name", "creator", "creatorId", "type", "source", "sourceUri", "metadata", "metadataId",
                    "state"]


@pytest.mark.parametrize("native", [True, False])
def test_postgres_renamed_columns_through_the_service(native):
    """Status handler over the wire with an ORM-style camelCase table: both handler
    implementations read and write the mapped columns (index.js:68,76)."""
    async def go():
        pg = await FakePg().start()
        try:
            st = PostgresStore(pg.dsn, table="public_media", create_schema=True, columns=CAMEL)
            await st.connect()
            await st.upsert(M1)
            c = cfg({"service": {"native_handlers": native}})
            from beholder_amd.transport.memory import MemoryBroker
            b = MemoryBroker()
            http = RecordingHttpClient()
            stream = MemoryStream()
            svc = Service(c, source=b.consumer(), store=st, http=http, logger=Logger(stream=stream),
                          serve_metrics=False)
            await svc.init()
            b.publish(T.STATUS, status_msg("m1", "DEPLOYED"))
            b.finish()
            await svc.run()
            row = await st.get_by_id("m1")
            raw = pg.db.execute('SELECT "state", "creatorId" FROM public_media').fetchall()
            await svc.close()
            return row, raw, http, pg.queries, stream
        finally:
            await pg.stop()
    row, raw, http, queries, stream = run(go())
    assert row.status == 4 and raw == [(4, "card")] and http.count == 3  # move + telegram + emby
    assert any('SET "state" = $1 WHERE "id" = $2' in q for q in queries)
    line = next(r["msg"] for r in stream.records() if r["msg"].startswith("consuming from"))
    assert "table=public_media" in line and "creatorId:creatorId" in line and "status:state" in line
