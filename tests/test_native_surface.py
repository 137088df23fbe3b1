"""The small public surface of the native types that the service itself does not call: counters'
and parsers' getters, ``reset()`` methods, the IOFuture's asyncio-Future protocol methods, the
log sink's retarget and its counts. Operators, the bench and debugging sessions use them; each is
checked here against what it reports (``make coverage`` listed them as never executed,
VERDICT r5 item 2: every native function gets a test or is deleted)."""
import asyncio
import io

import pytest

from beholder_amd.ops import (AckBatcher, AmqpDemux, Counter, Delivery, H1Parser, Histogram, IOFuture, Ingest,
                              PgReader, Settler, native)
from beholder_amd.ops.bench_native import native_bench


def test_ack_batcher_reports_its_low_mark_and_pending_acks():
    b = AckBatcher(lambda: None)
    b.bind(object(), 1)
    assert (b.low, b.pending) == (1, 0)
    b.ack(2)
    assert (b.low, b.pending) == (1, 1)  # tag 1 still open: the run starts there
    b.ack(1)
    assert (b.low, b.pending) == (3, 2)
    b.flush()
    assert b.pending == 0


def test_amqp_demux_capture_headers_switch():
    dm = AmqpDemux(Settler(), 0)
    assert dm.capture_headers is False
    dm.capture_headers = True
    assert dm.capture_headers is True
    dm.capture_headers = 0
    assert dm.capture_headers is False


def test_settler_and_ingest_getters_and_delivery_repr():
    s = Settler()
    assert s.created == 0 and s.ack_batcher is None
    d = Delivery(b"\x0a\x01x", 2, 7, s)
    assert s.created == 1
    r = repr(d)
    assert "Delivery" in r and "7" in r and "pending" in r
    d.ack()
    assert "acked" in repr(d)
    ing = Ingest()
    assert isinstance(ing.settler, Settler) and ing.drained is False
    ing.close()
    assert ing.drained is True


def test_metric_resets():
    h = Histogram()
    for v in (1000, 2000, 3000):
        h.record(v)
    assert h.count == 3
    h.reset()
    assert h.count == 0
    c = Counter()
    c.inc(5)
    c.reset()
    assert c.value == 0
    b = native.Buckets((0.1, 1.0))
    b.observe(0.5)
    before = b.snapshot()
    b.reset()
    assert before != b.snapshot()
    b.observe(0.5)
    assert b.snapshot() == before


def test_sink_stats_names_its_sink():
    from beholder_amd.metrics import Registry
    from beholder_amd.sinks.http import SinkObserver
    st = SinkObserver(Registry()).child("telegram")
    assert st.sink == "telegram"


def test_parsers_count_what_they_read():
    p = H1Parser()
    assert p.responses == 0
    p.start(head=False)
    p.feed(b"HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n")
    assert p.responses == 1
    r = PgReader()
    assert r.messages == 0
    r.feed(b"Z\x00\x00\x00\x05I" + b"N\x00\x00\x00\x04")
    assert r.messages == 2


def test_io_future_follows_the_asyncio_future_protocol():
    """IOFuture is awaited by Tasks like an asyncio.Future: ``__await__`` / ``send`` / ``__next__``
    yield it until done, then return its result; ``_make_cancelled_error`` and
    ``_log_traceback`` are the hooks asyncio calls on futures."""
    async def go():
        loop = asyncio.get_running_loop()
        f = IOFuture(loop)
        it = f.__await__()
        assert next(it) is f  # not done: yields itself
        assert it.send(None) is f
        f.set_result(41)
        with pytest.raises(StopIteration) as e:
            next(it)
        assert e.value.value == 41
        g = IOFuture(loop)
        g.cancel("why")
        err = g._make_cancelled_error()
        assert isinstance(err, asyncio.CancelledError)
        h = IOFuture(loop)
        # an IOFuture never logs an unretrieved exception (its owner always reads it): asyncio's
        # flag reads False and writes are accepted and ignored
        assert h._log_traceback is False
        h._log_traceback = True
        assert h._log_traceback is False
    asyncio.run(go())


def test_log_sink_retarget_counts_and_bytes():
    from beholder_amd.utils.log import Logger, MemoryStream
    first, second = io.StringIO(), io.StringIO()
    log = Logger(stream=first, level="trace")
    sink = log._shared.sink
    log.trace("t")
    log.fatal("f")
    log.info("i")
    assert sink.pending_bytes > 0
    sink.flush()
    assert sink.pending_bytes == 0 and sink.bytes_written == len(first.getvalue().encode())
    counts = sink.counts
    assert counts["trace"] == 1 and counts["fatal"] == 1 and counts["info"] == 1
    sink.retarget(second.write, second.flush)
    log.warn("w")
    sink.flush()
    assert '"msg":"w"' in second.getvalue() and '"msg":"w"' not in first.getvalue()
    levels = [ln.split('"level":')[1].split(",")[0] for ln in first.getvalue().splitlines()]
    assert levels == ["10", "60", "30"]
    with pytest.raises(TypeError, match="callable"):
        sink.retarget(42)
    assert isinstance(MemoryStream(), MemoryStream)


def test_netpoll_switch_reports_on():
    assert native.netpoll_enabled() is True


def test_bench_natives_report_their_state():
    """The bench extension's small surface: the recorder's mode, its immediate awaitable driven by
    next(), and the Postgres fake's per-row status lookup."""
    from beholder_amd.sinks.http import HttpResponse
    from beholder_amd.sinks import RecordingHttpClient
    assert RecordingHttpClient()._rec.mode == "h1"
    c = RecordingHttpClient(stub="url")
    assert c._rec.mode == "url"
    aw = c._rec.request("GET", "https://api.telegram.org/bot1/sendMessage", {"chat_id": 1})
    with pytest.raises(StopIteration) as e:
        next(aw.__await__())
    assert isinstance(e.value.value, HttpResponse) and e.value.value.status == 200
    from beholder_amd.bench.generator import Workload
    media = Workload(n_media=3, seed=1).media
    pf = native_bench.PgFake([list(m) for m in media])
    assert pf.status_of(media[0].id) == str(media[0].status) and pf.status_of("nope") is None


def test_tls_context_reports_openssls_reason_for_a_bad_ca_file(tmp_path):
    """TlsContext(cafile=...) that OpenSSL cannot load: FileNotFoundError with OpenSSL's own error
    text (py_tls.cpp last_error_text), not a generic message."""
    bad = tmp_path / "not-a-cert.pem"
    bad.write_text("this is not PEM\n")
    for path in (str(tmp_path / "missing.pem"), str(bad)):
        with pytest.raises(FileNotFoundError, match="cannot load verify locations") as e:
            native.TlsContext(cafile=path)
        assert len(str(e.value).split(": ", 1)[1]) > 0
