"""Property tests (SURVEY.md §4 layer 5): fuzzed inbound bytes never crash the service;
the progress path always acks (Q7); a status message ends acked or (Q1) un-acked, never
double-settled; every delivery is accounted for."""
import asyncio
import gc
import os

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from beholder_amd.ops import frames
from beholder_amd.service import Service
from beholder_amd.sinks import RecordingHttpClient
from beholder_amd.store import MemoryStore
from beholder_amd.topics import PROGRESS, PROGRESS_ID, STATUS, STATUS_ID
from beholder_amd.transport.ingest import BytesSource, FdSource
from beholder_amd.transport.memory import MemoryBroker
from beholder_amd.utils.log import Logger, NullStream

from helpers import cfg, progress_msg, status_msg, trello_media

MEDIA = [trello_media("m1"), trello_media("m2", card="C2")]

valid_progress = st.builds(lambda m, s, p, h: progress_msg(m, s, p, h), st.sampled_from(["m1", "m2", "nope"]),
                           st.integers(0, 7), st.integers(-5, 105), st.sampled_from(["", "w1"]))
valid_status = st.builds(lambda m, s: status_msg(m, s), st.sampled_from(["m1", "m2", "nope"]), st.integers(0, 7))
payload = st.one_of(st.binary(max_size=40), valid_progress, valid_status)


class _SlowStore(MemoryStore):
    """Every store call really suspends, so handlers run through the native Driver."""

    get_by_id_nowait = None
    update_status_nowait = None

    async def get_by_id(self, media_id):
        await asyncio.sleep(0)
        return await super().get_by_id(media_id)

    async def update_status(self, media_id, status):
        await asyncio.sleep(0)
        return await super().update_status(media_id, status)


def _run(msgs, suspend: bool = False):
    async def go():
        b = MemoryBroker()
        src = b.consumer(prefetch=1000)
        store = _SlowStore(MEDIA) if suspend else MemoryStore(MEDIA)
        http = RecordingHttpClient(keep=4, delay_s=0.0005 if suspend else 0.0)
        svc = Service(cfg(), source=src, store=store, http=http,
                      logger=Logger(stream=NullStream()), serve_metrics=False)
        await svc.init()
        for topic, body in msgs:
            b.publish(topic, body)
        b.finish()
        await svc.run()
        st_ = src.stats()
        await svc.close()
        return st_, b.stats()
    return asyncio.run(go())


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(st.tuples(st.sampled_from([STATUS, PROGRESS]), payload), max_size=30), st.booleans())
def test_fuzzed_messages_are_all_accounted_for(msgs, suspend):
    """Both dispatch paths: eager completion and suspension (native Driver resumes handlers)."""
    s, broker = _run(msgs, suspend)
    n_prog = sum(1 for t, _ in msgs if t == PROGRESS)
    n = len(msgs)
    # Q7: every progress message is acked; nothing is settled twice
    assert s["created"] == n
    assert s["acked"] >= n_prog
    assert s["acked"] + s["pending"] + s["abandoned"] + s["nacked"] + s["rejected"] == n
    assert s["nacked"] == 0 and s["rejected"] == 0  # default policy: leave_unacked (Q1)
    un = s["unacked_outstanding"]
    assert un == n - s["acked"]  # only status messages can be left un-acked


def test_stdin_dead_letter_replays_unacked_status(tmp_path):
    """Never-acked status frames (Q1) go to the dead-letter file and replay cleanly."""
    dl = str(tmp_path / "dead.bin")
    good = status_msg("m1", "QUEUED")
    bad = b"\x0a\x05ab"
    data = frames([(STATUS_ID, bad), (PROGRESS_ID, progress_msg("m1", "QUEUED", 1)), (STATUS_ID, good),
                   (STATUS_ID, bad)])

    async def go(src):
        svc = Service(cfg(), source=src, store=MemoryStore(MEDIA), http=RecordingHttpClient(),
                      logger=Logger(stream=NullStream()), serve_metrics=False)
        await svc.init()
        stats = await svc.run()
        await svc.close()
        return stats

    stats = asyncio.run(go(BytesSource(data, dead_letter=dl)))
    gc.collect()
    assert stats["handler_errors"][STATUS] == 2
    from beholder_amd.transport.framing import iter_frames
    with open(dl, "rb") as f:
        dead = list(iter_frames(f.read()))
    assert dead == [(STATUS_ID, bad), (STATUS_ID, bad)]
    # replay the dead letters (e.g. after a fix) through a file source
    stats2 = asyncio.run(go(FdSource(path=dl)))
    assert stats2["received"][STATUS] == 2
    assert os.path.getsize(dl) > 0
