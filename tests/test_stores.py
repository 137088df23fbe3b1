"""Media stores (triton-core/db parity, index.js:42,68,76,140): memory, sqlite, postgres (wire protocol)."""
import asyncio

import pytest

from beholder_amd.store import Media, MediaNotFound, MemoryStore, open_store
from beholder_amd.store.pgwire import PgConnection, PgError, PgProtocolError
from beholder_amd.store.postgres import PostgresStore

from pg_fake import FakePg

M1 = Media(id="m1", name="Bebop", creator=1, creatorId="card", metadataId="1", status=2)


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


async def _contract(st):
    await st.connect()
    try:
        await st.upsert(M1)
        await st.upsert(Media(id="m2", name="Trigun"))
        assert await st.count() == 2
        assert await st.get_by_id("m1") == M1
        await st.update_status("m1", 4)
        assert (await st.getByID("m1")).status == 4
        await st.updateStatus("missing", 3)  # UPDATE of zero rows: no error
        with pytest.raises(MediaNotFound):
            await st.get_by_id("missing")
        await st.upsert(M1._replace(name="Cowboy Bebop"))
        got = await st.get_by_id("m1")
        assert got.name == "Cowboy Bebop" and got.status == 2 and await st.count() == 2
    finally:
        await st.close()


def test_memory_store_contract():
    run(_contract(MemoryStore()))


def test_sqlite_store_contract(tmp_path):
    run(_contract(open_store("sqlite", str(tmp_path / "media.db"))))


@pytest.mark.parametrize("auth", ["scram", "md5", "cleartext", "trust"])
def test_postgres_store_contract_over_wire(auth):
    async def go():
        pg = await FakePg(auth=auth).start()
        try:
            await _contract(PostgresStore(pg.dsn, create_schema=True, pool_size=2))
            # prepared statements are parsed once per connection and reused
            assert pg.statements_parsed <= 2 * 8
        finally:
            await pg.stop()
    run(go())


def test_postgres_bad_password():
    async def go():
        pg = await FakePg(auth="scram").start()
        try:
            bad = pg.dsn.replace("s3cret", "nope")
            with pytest.raises(PgError) as ei:
                await PgConnection(bad).connect()
            assert ei.value.sqlstate == "28P01"
        finally:
            await pg.stop()
    run(go())


def test_postgres_error_then_connection_still_usable():
    async def go():
        pg = await FakePg(auth="trust").start()
        try:
            c = await PgConnection(pg.dsn).connect()
            with pytest.raises(PgError) as ei:
                await c.execute("this is a syntax error")
            assert ei.value.sqlstate == "42601"
            rows, tag = await c.execute("SELECT 1 + $1", (41,))
            assert rows == [(42,)] and tag == "SELECT 1"
            await c.close()
            with pytest.raises(PgProtocolError):
                await c.execute("SELECT 1")
        finally:
            await pg.stop()
    run(go())


def test_postgres_store_in_service():
    """The status handler's UPDATE + SELECT go over the wire (index.js:68,76)."""
    from beholder_amd.service import Service
    from beholder_amd.sinks import RecordingHttpClient
    from beholder_amd.topics import STATUS
    from beholder_amd.transport.memory import MemoryBroker
    from beholder_amd.utils.log import Logger, MemoryStream

    from helpers import cfg, status_msg

    async def go():
        pg = await FakePg().start()
        try:
            st = PostgresStore(pg.dsn, create_schema=True)
            await st.connect()
            await st.upsert(M1)
            b = MemoryBroker()
            http = RecordingHttpClient()
            svc = Service(cfg(), source=b.consumer(), store=st, http=http, logger=Logger(stream=MemoryStream()),
                          serve_metrics=False)
            await svc.init()
            b.publish(STATUS, status_msg("m1", "DEPLOYED"))
            b.finish()
            await svc.run()
            row = await st.get_by_id("m1")
            await svc.close()
            return row, http
        finally:
            await pg.stop()
    row, http = run(go())
    assert row.status == 4 and http.count == 3  # move + telegram + emby
