"""The e2e bench's Postgres stand-in (bench/pg_sink_server.py): the native PgFake
(ops/csrc_bench/pg_fake.cpp, the default) and the asyncio server it replaced (``--python``) must
answer the media store identically: rows of the synthetic population, the status UPDATE applied,
unknown ids, an unsupported statement failing only its own Sync group, SSLRequest refused (the
client's sslmode=prefer goes on in plain text), pipelined queries, and DONE / STALLS lines on
SIGTERM."""
import asyncio
import json

import pytest

from beholder_amd.bench import harness
from beholder_amd.bench.generator import make_media
from beholder_amd.store import MediaNotFound
from beholder_amd.store.postgres import PostgresStore
from beholder_amd.store.pgwire import PgConnection, PgError


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


@pytest.fixture(params=["native", "python"])
def fake(request):
    args = ("--media", "200", "--seed", "3") + (("--python",) if request.param == "python" else ())
    port, procs = harness._spawn("beholder_amd.bench.pg_sink_server", 1, args)
    try:
        yield port, procs
    finally:
        harness._reap(procs)


def test_store_round_trip(fake):
    port, _ = fake
    media = make_media(200, 3)

    async def go():
        st = PostgresStore(f"postgres://beholder@127.0.0.1:{port}/media?sslmode=prefer", pool_size=2)
        await st.connect()
        try:
            first = await st.get_by_id(media[0].id)
            await st.update_status(media[0].id, 7)
            after = await st.get_by_id(media[0].id)
            many = await asyncio.gather(*(st.get_by_id(m.id) for m in media[:50]))  # pipelined
            try:
                await st.get_by_id("no-such-media")
                missing = False
            except MediaNotFound:
                missing = True
            return first, after, many, missing
        finally:
            await st.close()
    first, after, many, missing = run(go())
    assert tuple(first) == tuple(media[0])
    assert after.status == 7 and tuple(after)[:9] == tuple(media[0])[:9]
    assert [m.id for m in many] == [m.id for m in media[:50]] and many[1] == media[1]
    assert missing


def test_unsupported_statement_fails_only_its_sync_group(fake):
    port, _ = fake
    media = make_media(200, 3)

    async def go():
        c = await PgConnection(f"postgres://beholder@127.0.0.1:{port}/media").connect()
        try:
            try:
                await c.execute("DELETE FROM media")
                err = None
            except PgError as e:
                err = e
            rows, tag = await c.execute('SELECT id, name, creator, "creatorId", type, source, "sourceURI", '
                                        'metadata, "metadataId", status FROM media WHERE id = $1', (media[5].id,))
            return err, rows, tag
        finally:
            await c.close()
    err, rows, tag = run(go())
    assert err is not None and "unsupported statement" in str(err)
    assert tag == "SELECT 1" and rows[0][0] == media[5].id


def test_sigterm_reports_queries_and_stall_line():
    port, procs = harness._spawn("beholder_amd.bench.pg_sink_server", 1, ("--media", "50", "--seed", "1"))
    media = make_media(50, 1)

    async def go():
        st = PostgresStore(f"postgres://beholder@127.0.0.1:{port}/media", pool_size=1)
        await st.connect()
        try:
            for m in media[:10]:
                await st.get_by_id(m.id)
        finally:
            await st.close()
    try:
        run(go())
    finally:
        stalls: list = []
        counters = harness._reap(procs, stalls)
    assert counters["queries"] >= 10
    assert len(stalls) == 1 and stalls[0]["name"] == "pg" and stalls[0]["loop_stalls"] >= 0
    assert isinstance(stalls[0]["stall_intervals"], list)
    json.dumps(stalls[0])
