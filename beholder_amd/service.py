"""Service bootstrap and dispatch loop — ``init()`` of the reference (index.js:23-160).

Startup order mirrors index.js:23-158:

1. config (``Config('events')``)                        index.js:24
2. Trello client                                         index.js:25
3. Prometheus registry + HTTP exposure                   index.js:27-28
4. the two counters                                      index.js:29-40
5. media store                                           index.js:42
6. transport connect (prefetch 100)                      index.js:43-44
7. proto types                                           index.js:46-48
8. ``listen`` on status + progress                       index.js:62,127
9. log ``initialized``                                   index.js:157

Differences, all documented fixes:

* **Q10** — ``init()`` in the reference is fire-and-forget; a startup failure
  is an unhandled rejection that leaves a half-started process. Here startup
  errors propagate and the CLI exits non-zero.
* graceful shutdown (SIGTERM/SIGINT): stop consuming, drain in-flight
  handlers for ``service.shutdown_grace_s``, close transport/store/sinks.

Dispatch: deliveries arrive in batches. Each handler coroutine is driven eagerly by
the native ``dispatch_batch`` (``PyIter_Send``; no Task for a handler that never
blocks). A handler that suspends on real I/O is resumed by a native ``Driver``
when the awaited future completes. At most ``service.prefetch`` (default 100,
index.js:43) are in flight, matching the broker's prefetch window.
"""
from __future__ import annotations

import array
import asyncio
import gc
import time
from typing import Any, Callable, Dict, List, Optional

from . import topics as T
from .config import Config
from .handlers import TelemetryHandlers, err_message, native_handlers
from .metrics import MetricsServer, NativeHistogramView, Registry, default_metrics
from .metrics.registry import Gauge
from .parallel.ordering import KeyedSerializer
from .utils.waits import Signal
from .sinks import AiohttpClient, EmbyClient, H1Client, HttpClient, SinkObserver, TelegramClient, TrelloClient
from .sinks.ratelimit import from_config as sink_policy
from .store import MediaStore, open_store
from .transport.base import Source
from .ops import Driver, Histogram, Window, dispatch_batch
from .utils.fdtable import reserve_fd_table
from .utils.log import Logger
from .utils.tracing import extract as extract_trace_context, tracer_from_config

Handler = Callable[[Any], Any]


def build_source(config: Config, logger: Optional[Logger] = None, capture_headers: bool = False) -> Source:
    """Construct the ingest transport from ``service.transport``."""
    tcfg = config.data["service"]["transport"]
    kind = (tcfg.get("kind") or "amqp").lower()
    prefetch = int(config.data["service"]["prefetch"])
    if kind in ("stdin", "file") and tcfg.get("format", "binary") == "ndjson":
        from .transport.ingest import NdjsonSource
        return NdjsonSource(path=tcfg.get("path") if kind == "file" else None,
                            policy=tcfg.get("policy", "block"), dead_letter=tcfg.get("dead_letter"))
    if kind == "stdin":
        from .transport.ingest import FdSource
        return FdSource(policy=tcfg.get("policy", "block"),
                        capacity_bytes=int(tcfg.get("capacity_bytes", 64 << 20)),
                        capacity_events=int(tcfg.get("capacity_events", 0)),
                        dead_letter=tcfg.get("dead_letter"))
    if kind == "file":
        from .transport.ingest import FdSource
        if not tcfg.get("path"):
            raise ValueError("service.transport.path is required for kind=file")
        return FdSource(path=tcfg["path"], policy=tcfg.get("policy", "block"),
                        capacity_bytes=int(tcfg.get("capacity_bytes", 64 << 20)),
                        capacity_events=int(tcfg.get("capacity_events", 0)),
                        dead_letter=tcfg.get("dead_letter"))
    if kind == "amqp":
        from .dynamics import dyn
        from .transport.amqp import AmqpSource
        url = tcfg.get("url") or dyn("rabbitmq", env=config.env, config=config)
        hb = tcfg.get("heartbeat")
        from .transport.amqp.topology import Topology
        return AmqpSource(url, prefetch=prefetch, retries=int(config.data["service"]["retries"]),
                          logger=logger, heartbeat=None if hb is None else int(hb), capture_headers=capture_headers,
                          topology=Topology.from_config(config.data["service"].get("amqp")))
    raise ValueError(f"unknown transport kind {kind!r} (amqp|stdin|file)")


def make_http_client(http_cfg) -> HttpClient:
    """``service.http``: ``client: h1`` (default, sinks/h1.py) or ``aiohttp``."""
    timeout = float(http_cfg.get("timeout_s", 30.0))
    if http_cfg.get("client", "h1") == "aiohttp":
        return AiohttpClient(timeout_s=timeout)
    return H1Client(timeout_s=timeout, max_per_host=int(http_cfg.get("max_per_host", 100)),
                    keepalive_s=float(http_cfg.get("keepalive_s", 4.0)), ssl_cafile=http_cfg.get("ca_file") or None,
                    max_connecting=int(http_cfg.get("max_connecting", 8)))


def _gc_pause_recorder(hist):
    """A ``gc.callbacks`` entry recording each collection's duration (ns) into ``hist``. It holds
    only the histogram, so a service that is never closed does not stay alive through it."""
    t0 = [0]
    mono = time.monotonic_ns

    def cb(phase, _info):
        if phase == "start":
            t0[0] = mono()
        elif t0[0]:
            hist.record(mono() - t0[0])
            t0[0] = 0
    return cb


class Service:
    """The beholder service. Inject ``source``/``store``/``http`` for tests and benches."""

    def __init__(self, config: Config, *, source: Optional[Source] = None, store: Optional[MediaStore] = None,
                 http: Optional[HttpClient] = None, registry: Optional[Registry] = None,
                 logger: Optional[Logger] = None, serve_metrics: Optional[bool] = None):
        self.config = config
        svc = config.data["service"]
        self.log = logger or Logger(name=svc["log"]["name"], level=svc["log"]["level"],
                                    positional_args=svc["log"].get("positional_args", "append"))
        self._source = source
        self._store = store
        self._http = http
        self.registry = registry
        self._serve_metrics = svc["metrics"]["enabled"] if serve_metrics is None else serve_metrics
        self.metrics_server: Optional[MetricsServer] = None
        self.prefetch = int(svc["prefetch"])
        self.on_status_error = svc["on_status_error"]
        self.ordering = svc["ordering"]
        self.grace_s = float(svc["shutdown_grace_s"])
        # per-message trace spans (SURVEY.md §5 tracing): one debug line per handled delivery
        self.trace = bool(svc.get("trace", False))
        # Jaeger spans per delivery (utils/tracing.py): service.tracing or JAEGER_* env
        self.tracer = tracer_from_config(svc.get("tracing"), env=config.env)
        self._routes: List[Optional[Handler]] = [None] * len(T.TOPIC_NAMES_BY_ID)
        # handlers suspended on I/O, at most `prefetch` (index.js:43); drivers report back in C
        self._inflight = Window(self.prefetch, self._on_handler_error, self._on_wake)
        self._slot_free: Optional[Signal] = None
        self._slot_waits = 0  # times the dispatch loop waited for a prefetch slot
        self._idle: Optional[asyncio.Event] = None  # set when the last suspended handler finishes
        self._stop = False
        self._running = False
        self._initialized = False
        self.handlers: Optional[TelemetryHandlers] = None
        self.handler_impl: Any = None  # handlers or their compiled form (ops.NativeHandlers)
        self.serializer: Optional[KeyedSerializer] = None
        self.started_at = 0.0
        self.received = array.array("Q", [0] * len(T.TOPIC_NAMES_BY_ID))
        self.source_error: Optional[str] = None
        self._preconnecting: set = set()  # preconnect tasks still running after startup
        # event-loop lag (how late the 100 ms log flusher wakes) and GC pauses, in ns: the two
        # process-side causes of a slow delivery (bench/stallmon.py attributes them in the bench)
        self.loop_lag = Histogram()
        self.gc_pause = Histogram()
        self._gc_cb = None

    # ------------------------------------------------------------ properties --
    @property
    def source(self) -> Source:
        assert self._source is not None, "service not initialised"
        return self._source

    @property
    def store(self) -> MediaStore:
        assert self._store is not None, "service not initialised"
        return self._store

    # ------------------------------------------------------------------ init --
    async def init(self) -> "Service":
        cfg = self.config
        svc = cfg.data["service"]
        keys = cfg.root.require("keys.trello")
        # descriptor table sized now: a grow later blocks the loop thread for an RCU grace period
        # (140-160 ms on the box) in the socket() of a sink connect (utils/fdtable.py)
        reserve_fd_table(max(1024, 4 * int(svc["http"].get("max_per_host", 100)) + 256))
        # 2. Trello client (index.js:25)
        if self._http is None:
            self._http = make_http_client(svc["http"])
        endpoints = svc["endpoints"]
        # 3-4. registry + counters (index.js:27-40)
        if self.registry is None:
            self.registry = Registry("beholder")
        reg = self.registry
        observer = SinkObserver(reg) if svc["metrics"].get("sink_metrics", True) else None
        sinks = svc.get("sinks") or {}
        tl, tr = sink_policy(sinks.get("trello"))  # opt-in rate limits / 429 retries (sinks/ratelimit.py)
        gl, gr = sink_policy(sinks.get("telegram"))
        el, er = sink_policy(sinks.get("emby"))
        self.trello = TrelloClient(keys.get("key"), keys.get("token"), self._http, base_url=endpoints["trello"],
                                   observer=observer, limiter=tl, retry=tr)
        self.telegram = TelegramClient(None, self._http, base_url=endpoints["telegram"], observer=observer,
                                       limiter=gl, retry=gr)
        self.emby = EmbyClient(None, None, self._http, observer=observer, limiter=el, retry=er)

        self.progress_updates_total = reg.counter(
            "beholder_progress_updates_total", "Total number of messages processed in this processes lifetime",
            ["status"])
        # name without `_total` and the "crreated" typo are the reference's (index.js:35-38)
        self.trello_comments_total = reg.counter(
            "beholder_trello_comments", "Total trello comments crreated in this processes lifetime")
        self._register_service_metrics(reg)
        if svc["metrics"].get("default_metrics", True):
            reg.add_collector(default_metrics)
        if self._serve_metrics:
            m = svc["metrics"]
            self.metrics_server = await MetricsServer(reg, m["host"], int(m["port"]), health=self.healthy,
                                                      stats=self.stats, logger=self.log).start()

        # 5. store (index.js:42)
        if self._store is None:
            st = svc["store"]
            backend = st.get("backend", "postgres")
            kw = {"table": st.get("table") or "media", "columns": dict(st.get("columns") or {})}
            if backend in ("postgres", "postgresql", "pg"):
                kw.update(pool_size=int(st.get("pool_size", 4)), create_schema=bool(st.get("create_schema", False)),
                          spread_at=int(st.get("spread_at", 8)), stall_timeout_s=st.get("stall_timeout_s", 30.0),
                          min_connections=st.get("min_connections"))
            self._store = open_store(backend, st.get("dsn"), **kw)
        await self._store.connect()

        # 6. transport (index.js:43-44)
        if self._source is None:
            self._source = build_source(cfg, self.log, capture_headers=self.tracer is not None)

        # 7. proto types + handlers (index.js:46-60)
        self.handlers = TelemetryHandlers(
            config=cfg, store=self._store, trello=self.trello, telegram=self.telegram, emby=self.emby,
            progress_counter=self.progress_updates_total, comments_counter=self.trello_comments_total,
            logger=self.log)

        # 8. listeners (index.js:62,127): the compiled handlers unless disabled (same semantics)
        impl = self.handlers
        if svc.get("native_handlers", True):
            impl = native_handlers(self.handlers) or self.handlers
        self.handler_impl = impl
        if any(u.lower().startswith("https:") for u in self._sink_urls(endpoints)):
            # HTTPS sinks: the native TLS context (one-time OpenSSL warm-up, handshake threads)
            # is made now, not by the first connect of the first burst
            prep = getattr(self._http, "prepare_tls", None)
            if prep is not None:
                prep()
        pc = int(svc["http"].get("preconnect") or 0)
        if pc > 0:  # opt-in: sink connections made before the first delivery, not inside it
            await self._preconnect(pc, endpoints)
        self.listen(T.STATUS, impl.on_status)
        self.listen(T.PROGRESS, impl.on_progress)
        await self._source.start([t for t in T.TOPIC_IDS if self._routes[T.TOPIC_IDS[t]] is not None])
        if pc > 0:  # the preconnected connections' keep-alive window starts with consumption
            touch = getattr(self._http, "touch_idle", None)
            if touch is not None:
                touch()
        if self.ordering == "per_media":
            self.serializer = KeyedSerializer(self._dispatch_now, self._media_key)

        # 9.
        self._initialized = True
        self.started_at = time.time()
        if svc.get("gc_freeze", True):
            # Config, descriptors, store rows and handlers live for the whole process:
            # move them out of the collected generations so young-gen passes stay cheap.
            gc.collect()
            gc.freeze()
        self._gc_cb = _gc_pause_recorder(self.gc_pause)
        gc.callbacks.append(self._gc_cb)
        self.log.info("initialized")
        # the unpinned parts (triton-core's queue layout and media table are not vendored), stated
        # once so a mismatch with the real deployment is visible in the log
        self.log.info(f"consuming from {self._source.describe()}; store {self._store.describe()}")
        return self

    def _sink_urls(self, endpoints) -> List[str]:
        """The sink URLs the handlers will call: Trello; Telegram and Emby when their DEPLOYED
        hooks are on."""
        from .sinks.emby import _PATH as emby_path
        urls = [endpoints["trello"]]
        try:
            tg_on, _, _, emby_on, emby_host, _ = self.handlers._hooks_plan()
            if tg_on:
                urls.append(endpoints["telegram"])
            if emby_on and emby_host:
                urls.append(emby_path(emby_host))
        except Exception:  # noqa: BLE001 -- a hook config the handler would reject at its own point
            pass
        return [str(u) for u in urls]

    async def _preconnect(self, n: int, endpoints) -> None:
        """``service.http.preconnect``: ``n`` connections to each sink origin the handlers will
        call (Trello; Telegram and Emby when their DEPLOYED hooks are on), all at once, with
        startup held for at most ``preconnect_wait_s``. A sink that cannot be reached is warned
        about, never fatal: the reference only meets it on the first event, and the handlers
        connect on demand as they always do."""
        from .sinks.http import redact
        urls = self._sink_urls(endpoints)
        seen, origins = set(), []
        for u in urls:
            o = str(u).split("/", 3)[:3]
            key = "/".join(o).lower()
            if key not in seen:
                seen.add(key)
                origins.append(str(u))
        pre = getattr(self._http, "preconnect", None)
        if pre is None:  # a duck-typed client without the HttpClient base: nothing to open
            return

        def report(u, t):
            if t.cancelled():
                return
            e = t.exception()
            opened, err = (0, e) if e is not None else t.result()
            origin = redact("/".join(u.split("/", 3)[:3]))
            if err is not None:
                self.log.warn(f"preconnect to {origin}: {opened}/{n} connections ({type(err).__name__}: {err})")
            else:
                self.log.info(f"preconnect to {origin}: {opened} connections")

        tasks = []
        for u in origins:
            t = asyncio.ensure_future(pre(u, n))
            t.add_done_callback(lambda t, u=u: report(u, t))
            tasks.append(t)
        # startup waits for the connections at most `preconnect_wait_s` (a sink that drops
        # packets would otherwise hold it for the whole request timeout); the rest finish in
        # the background and are parked in the pool as they come
        wait_s = float(self.config.data["service"]["http"].get("preconnect_wait_s", 5.0))
        _, pending = await asyncio.wait(tasks, timeout=wait_s)
        if pending:
            self.log.warn(f"preconnect: {len(pending)} origin(s) still connecting after {wait_s:g} s; "
                          "continuing startup")
            self._preconnecting = pending
        await asyncio.sleep(0)  # the done callbacks of the finished ones log before `initialized`

    def _media_key(self, d) -> Any:
        h = self.handlers
        if d.topic_id == T.STATUS_ID:
            return h.decode_status(d.content).mediaId
        if d.topic_id == T.PROGRESS_ID:
            return h.decode_progress(d.content).mediaId
        return None

    def listen(self, topic: str, handler: Handler) -> None:
        """``amqp.listen(topic, fn)`` — register the handler for a topic."""
        self._routes[T.topic_id(topic)] = handler

    # --------------------------------------------------------------- metrics --
    def _register_service_metrics(self, reg: Registry) -> None:
        """Our additions for the §6 measurement plan (ingest rate, latency, drops)."""

        def settler():
            return self._source.settler if self._source is not None else None

        def ack_collect(g: Gauge):
            s = settler()
            if s is not None:
                st = s.stats()
                for k in ("acked", "nacked", "rejected", "abandoned", "pending"):
                    g.set({"state": k}, st[k])

        reg.register(Gauge("beholder_deliveries", "Deliveries by settlement state since start "
                           "(abandoned = never acked, reference quirk Q1)", ["state"], collect=ack_collect))

        def recv_collect(g: Gauge):
            for tid, n in enumerate(self.received):
                if T.TOPIC_NAMES_BY_ID[tid]:
                    g.set({"topic": T.TOPIC_NAMES_BY_ID[tid]}, n)

        reg.register(Gauge("beholder_messages_received", "Messages received per topic since start", ["topic"],
                           collect=recv_collect))
        self.handler_errors = reg.counter("beholder_handler_errors_total",
                                          "Handler invocations that raised (status handler: quirk Q1)", ["topic"])

        def drop_collect(g: Gauge):
            st = self._source.stats() if self._source is not None else {}
            for tid, n in (st.get("dropped_by_topic") or {}).items():
                g.set({"topic": T.topic_name(int(tid)) or str(tid)}, n)

        reg.register(Gauge("beholder_ingest_dropped", "Messages dropped by ingest backpressure", ["topic"],
                           collect=drop_collect))
        reg.register(Gauge("beholder_inflight", "Handlers currently suspended on I/O",
                           collect=lambda g: g.set(len(self._inflight))))

        # transport metrics (the reference hands `prom` to triton-core/amqp, index.js:43)
        def transport_collect(g: Gauge):
            if self._source is None:
                return
            st = self._source.stats()
            g.set({"kind": self._source.kind, "field": "connected"}, 1.0 if self._source.ready() else 0.0)
            for k in ("reconnects", "stale_settles", "bytes_in", "bytes_out", "ack_frames", "bytes_read",
                      "frames_read", "depth", "high_water_events"):
                v = st.get(k)
                if isinstance(v, (int, float)):
                    g.set({"kind": self._source.kind, "field": k}, v)

        reg.register(Gauge("beholder_transport", "Ingest transport state (connected flag, reconnects, bytes, "
                           "ring depth)", ["kind", "field"], collect=transport_collect))

        # outbound dependency pools: HTTP keep-alive connections (sinks/h1.py), Postgres connections
        def pools_collect(g: Gauge):
            http_stats = getattr(self._http, "stats", None)
            if callable(http_stats):
                for k, v in http_stats().items():
                    g.set({"pool": "http", "field": k}, v)
            pool = getattr(self._store, "_pool", None)
            if pool is not None and hasattr(pool, "connections"):
                g.set({"pool": "postgres", "field": "open"}, pool.connections)
                for k in ("grows", "grow_errors"):  # background grow (store/pgwire.py Pool)
                    v = getattr(pool, k, None)
                    if isinstance(v, int):
                        g.set({"pool": "postgres", "field": k}, v)

        reg.register(Gauge("beholder_pool", "Outbound connection pools (HTTP sinks, Postgres): open/idle "
                           "connections and request/connect/error counts", ["pool", "field"],
                           collect=pools_collect))

        reg.register(NativeHistogramView("beholder_handle_latency_seconds",
                                         "Handler start to ack latency",
                                         lambda: settler().handle_latency if settler() is not None else None))
        reg.register(NativeHistogramView("beholder_ingest_latency_seconds",
                                         "Receive to ack latency (includes queueing)",
                                         lambda: settler().ingest_latency if settler() is not None else None))
        reg.register(NativeHistogramView("beholder_event_loop_lag_seconds",
                                         "How late the event loop ran a 100 ms timer (a long callback, "
                                         "a GC pause, the process descheduled)", lambda: self.loop_lag))
        reg.register(NativeHistogramView("beholder_gc_pause_seconds",
                                         "Cyclic garbage collector pauses", lambda: self.gc_pause))
        reg.register(NativeHistogramView("beholder_queue_latency_seconds",
                                         "Receive to handler start: time a delivery waited for the consumer "
                                         "(backlog, prefetch window, event-loop wake-up)",
                                         lambda: settler().queue_latency if settler() is not None else None))

    # ------------------------------------------------------------------ run ---
    def healthy(self) -> bool:
        return self._initialized and not self._stop and (self._source is None or self._source.ready())

    def request_stop(self) -> None:
        """Graceful stop: stop consuming, let in-flight handlers finish and ack, then return
        from :meth:`run` (the caller closes the source/store afterwards)."""
        self._stop = True
        if self._source is not None:
            asyncio.ensure_future(self._source.stop_consuming())

    async def run(self) -> Dict[str, Any]:
        """Consume until the source ends or :meth:`request_stop`; then drain and return stats."""
        if not self._initialized:
            await self.init()
        self._running = True
        self._slot_free = Signal()
        flusher = asyncio.ensure_future(self._flush_logs_periodically())
        log = self.log
        routes = self._routes
        nroutes = len(routes)
        received = self.received
        dispatch = self.serializer.submit if self.serializer is not None else self._dispatch_now
        inflight = self._inflight
        prefetch = self.prefetch
        sleep = asyncio.sleep
        # native fast path: the per-delivery loop runs in C (ops.dispatch_batch); per-media
        # ordering and debug-line spans keep the Python loop; with Jaeger tracing only the
        # sampled deliveries leave it
        native = self.serializer is None and not self.trace
        tracer = self.tracer
        routes = tuple(routes)
        on_error, on_suspend, on_unroutable = self._on_handler_error, self._inflight, self._unroutable
        # a source that counts its waits (`idle_wakeups`): a batch that came after a wait was
        # preceded by a trip through the loop already, so it needs no extra yield (below)
        src = self.source
        counts_waits = isinstance(getattr(src, "idle_wakeups", None), int)
        last_wakeups = -1
        # a source that can hand deliveries over from its read callback (AmqpSource.direct) gets
        # the native dispatch itself while this task waits: a delivery at a low rate then starts
        # its handler with no wake-up of this task, one trip through the loop fewer
        direct = native and tracer is None and hasattr(src, "direct")
        if direct:
            src.direct = self._direct_dispatcher(routes, on_error, on_suspend, on_unroutable)
        try:
            async for batch in src.batches():
                waited = self._slot_waits
                if native and tracer is not None:
                    await self._dispatch_sampled(batch, routes, on_error, on_suspend, on_unroutable)
                elif native:
                    await self._dispatch_native(batch, routes, on_error, on_suspend, on_unroutable)
                else:
                    for d in batch:
                        tid = d.topic_id
                        if tid >= nroutes or routes[tid] is None:
                            self._unroutable(d)
                            continue
                        received[tid] += 1
                        dispatch(d)
                        if inflight and len(inflight) >= prefetch:
                            await self._wait_slots()
                log.flush()
                if self._stop:
                    break
                if counts_waits:
                    w = src.idle_wakeups
                    if w != last_wakeups:  # this batch followed a wait: the loop ran just before it
                        last_wakeups = w
                        continue
                if self._slot_waits != waited:  # it waited for a prefetch slot: the loop ran meanwhile
                    continue
                await sleep(0)  # keep timers / the metrics endpoint responsive under sustained load
        finally:
            if direct:
                src.direct = None
            self._running = False
            flusher.cancel()
            await self._drain()
            err = (self._source.stats() or {}).get("error") if self._source is not None else None
            if err:
                self.source_error = err
                log.error(f"ingest source failed: {err}")
            log.flush()
        return self.stats()

    def _direct_dispatcher(self, routes, on_error, on_suspend, on_unroutable):
        """The source's direct hand-over (AmqpSource.direct): dispatch what the prefetch window
        allows (ops.dispatch_batch, as _dispatch_native) and return the rest, which the source
        queues for this task; None once all of it started. Nothing after a stop request."""
        received, inflight, prefetch, log = self.received, self._inflight, self.prefetch, self.log

        def hand_over(batch):
            if self._stop:
                return batch
            n = len(batch)
            i = dispatch_batch(batch, 0, routes, received, on_error, on_suspend, on_unroutable) \
                if len(inflight) < prefetch else 0
            log.flush()
            return batch[i:] if i < n else None
        return hand_over

    async def _dispatch_native(self, batch, routes, on_error, on_suspend, on_unroutable) -> None:
        """The per-delivery loop in C (ops.dispatch_batch), pausing while `prefetch` handlers
        are suspended (index.js:43)."""
        i, n = 0, len(batch)
        inflight, prefetch = self._inflight, self.prefetch
        while i < n:
            i = dispatch_batch(batch, i, routes, self.received, on_error, on_suspend, on_unroutable)
            if i < n or len(inflight) >= prefetch:
                await self._wait_slots()

    async def _dispatch_sampled(self, batch, routes, on_error, on_suspend, on_unroutable) -> None:
        """Tracing on: each run of unsampled deliveries goes through the native loop, and each
        sampled delivery through the Python path that opens and closes its span."""
        i, n = 0, len(batch)
        while i < n:
            j, decision = self._next_sampled(batch, i)
            if i < j:
                await self._dispatch_native(batch[i:j] if i or j < n else batch, routes, on_error, on_suspend,
                                            on_unroutable)
            if j < n:
                d = batch[j]
                tid = d.topic_id
                if tid >= len(routes) or routes[tid] is None:
                    self._unroutable(d)
                else:
                    self.received[tid] += 1
                    self._dispatch_now(d, decision=decision)
                    if self._inflight and len(self._inflight) >= self.prefetch:
                        await self._wait_slots()
            i = j + 1

    async def _flush_logs_periodically(self, every_s: float = 0.1) -> None:
        """Lines logged outside the batch loop (reconnects, idle periods) reach the stream within
        100 ms. How late each of these wake-ups comes is the event loop's lag
        (``beholder_event_loop_lag_seconds``): no extra timer for it."""
        mono = time.monotonic_ns
        period_ns = int(every_s * 1e9)
        lag = self.loop_lag
        try:
            while True:
                due = mono() + period_ns
                await asyncio.sleep(every_s)
                late = mono() - due
                lag.record(late if late > 0 else 0)
                self.log.flush()
                if self.tracer is not None:
                    self.tracer.flush()
        except asyncio.CancelledError:
            pass

    def _span(self, d, outcome: str) -> None:
        now = time.monotonic_ns()
        self.log.debug({"span": d.topic, "tag": d.tag, "queue_us": (d.start_ns - d.recv_ns) // 1000,
                        "handle_us": (now - d.start_ns) // 1000, "outcome": outcome, "state": d.state},
                       "handled")

    def _next_sampled(self, batch, i: int):
        """``(j, decision)``: the first delivery at or after ``i`` whose trace is sampled, with
        its sampling decision (``j == len(batch)``, None when there is none)."""
        sample = self.tracer.sample
        n = len(batch)
        while i < n:
            h = batch[i].headers
            decision = sample(extract_trace_context(h) if h is not None else None)
            if decision is not None:
                return i, decision
            i += 1
        return n, None

    def _trace_start(self, d, decision=None):
        """A Jaeger span for this delivery (None when not sampled). Called after ``d.start()``."""
        topic = d.topic or str(d.topic_id)
        tags = {"span.kind": "consumer", "component": "beholder", "message_bus.destination": topic,
                "amqp.delivery_tag": d.tag, "amqp.redelivered": d.redelivered,
                "beholder.queue_us": max(0, d.start_ns - d.recv_ns) // 1000}
        if decision is not None:
            return self.tracer.start_sampled(decision, topic, tags=tags)
        return self.tracer.start_span(topic, child_of=extract_trace_context(d.headers), tags=tags)

    def _trace_finish(self, span, d, exc: Optional[BaseException]) -> None:
        h = self.handlers
        try:
            dec = h.decode_status if d.topic_id == T.STATUS_ID else h.decode_progress
            span.set_tag("mediaId", dec(d.content).mediaId)
        except Exception:  # noqa: BLE001 — undecodable message: the error tag says why
            pass
        span.set_tag("beholder.outcome", d.state)  # pending = left un-acked (quirk Q1)
        if exc is not None:
            span.set_tag("error", True)
            span.log_kv({"event": "error", "error.kind": type(exc).__name__, "message": err_message(exc)})
        span.finish()

    def _dispatch_now(self, d, on_finish: Optional[Callable[[], None]] = None, decision=None) -> bool:
        """Python dispatch path (per-media ordering, trace spans). Returns True when the handler
        finished synchronously; otherwise a Driver finishes it and calls ``on_finish()`` then.
        ``decision``: a sampling decision already taken (``Tracer.sample``) for this delivery."""
        handler = self._routes[d.topic_id]
        d.start()
        span = self._trace_start(d, decision) if self.tracer is not None else None
        coro = handler(d)
        try:
            first = coro.send(None)
        except StopIteration:
            if self.trace:
                self._span(d, "ok" if d.settled else "unsettled")
            if span is not None:
                self._trace_finish(span, d, None)
            return True
        except BaseException as exc:  # noqa: BLE001 — handler errors are data here
            self._on_handler_error(d, exc)
            if span is not None:
                self._trace_finish(span, d, exc)
            exc = None  # the traceback reaches this frame via f_back: don't keep a cycle alive
            if self.trace:
                self._span(d, "ok" if d.settled else "unsettled")
            return True
        if on_finish is None and not self.trace and span is None:
            self._inflight.suspend(d, coro, first)
            return False

        def done(drv, exc, on_finish=on_finish, d=d, span=span):
            self._inflight.release(drv, exc)
            if self.trace:
                self._span(d, "ok" if d.settled else "unsettled")
            if span is not None:
                self._trace_finish(span, d, exc)
            if on_finish is not None:
                on_finish()
        drv = Driver(coro, done, d)
        self._inflight.track(drv)
        drv.start(first)
        return False

    def _on_wake(self) -> None:
        """From the native Window: a slot freed after the window was full, or it emptied."""
        if self._slot_free is not None:
            self._slot_free.set()
        if not len(self._inflight) and self._idle is not None:
            self._idle.set()

    async def _wait_slots(self) -> None:
        while len(self._inflight) >= self.prefetch:
            self._slot_free.clear()
            self._slot_waits += 1
            await self._slot_free.wait()

    def _on_handler_error(self, d, exc: BaseException) -> None:
        topic = d.topic or str(d.topic_id)
        self.handler_errors.labels(topic).inc()
        # Node would print an UnhandledPromiseRejectionWarning here (index.js:62 has no catch).
        self.log.error(f"unhandled error in {topic} handler: {err_message(exc)}")
        # Drop the traceback: it references the handler frame (and so the delivery). Freeing it
        # promptly lets an un-acked delivery be reported as abandoned right away (Q1 accounting).
        exc.__traceback__ = None
        if d.settled or d.topic_id != T.STATUS_ID:
            # `service.on_status_error` is the Q1 knob (a throwing status handler); any other
            # handler's error leaves its delivery as the reference would (un-acked)
            return
        policy = self.on_status_error
        try:
            if policy == "nack_requeue":
                d.nack(True)
            elif policy == "nack_drop":
                d.nack(False)
            # leave_unacked: reference behaviour (Q1) — the delivery stays pending
        except Exception as e:  # noqa: BLE001
            self.log.warn("failed to settle errored delivery:", err_message(e))

    def _unroutable(self, d) -> None:
        self.log.warn(f"dropping message for unknown topic id {d.topic_id}")
        if not d.settled:
            d.reject(False)

    async def _drain(self) -> None:
        if self.serializer is not None:
            await self.serializer.drain(self.grace_s)
        if self._inflight:
            self._idle = asyncio.Event()
            try:
                await asyncio.wait_for(self._idle.wait(), self.grace_s)
            except asyncio.TimeoutError:
                for drv in list(self._inflight):
                    drv.cancel()
                await asyncio.sleep(0)  # deliver the cancellations
            finally:
                self._idle = None

    async def close(self) -> None:
        """Release transport, store, HTTP client and the metrics server."""
        if self._gc_cb is not None:
            try:
                gc.callbacks.remove(self._gc_cb)
            except ValueError:
                pass
            self._gc_cb = None
        for t in self._preconnecting:
            t.cancel()
        if self._preconnecting:
            await asyncio.gather(*self._preconnecting, return_exceptions=True)
            self._preconnecting = set()
        if self._source is not None:
            await self._source.close()
        if self._store is not None:
            await self._store.close()
        if self._http is not None:
            await self._http.close()
        if self.metrics_server is not None:
            await self.metrics_server.stop()
        if self.tracer is not None:
            self.tracer.close()
        self.log.flush()

    # ---------------------------------------------------------------- stats ---
    def stats(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {"received": {T.TOPIC_NAMES_BY_ID[i]: n for i, n in enumerate(self.received) if i},
                               "inflight": len(self._inflight)}
        if self._source is not None:
            out["source"] = self._source.stats()
            s = self._source.settler
            if s is not None:
                out["handle_latency_ns"] = s.handle_latency.summary()
                out["ingest_latency_ns"] = s.ingest_latency.summary()
                out["queue_latency_ns"] = s.queue_latency.summary()  # receive -> handler start
        if self.registry is not None and hasattr(self, "handler_errors"):
            out["handler_errors"] = {k[0]: v for k, v in self.handler_errors.values().items()}
            out["trello_comments"] = self.trello_comments_total.get()
            out["progress_updates"] = {k[0]: v for k, v in self.progress_updates_total.values().items()}
        if self.serializer is not None:  # per-media ordering (opt-in)
            out["ordering"] = {"active_keys": self.serializer.active_keys,
                               "serialized": self.serializer.serialized, "max_chain": self.serializer.max_chain}
        if self.tracer is not None:
            out["tracing"] = self.tracer.reporter.stats()
        limits = {name: c.limiter.stats() for name, c in (("trello", getattr(self, "trello", None)),
                                                          ("telegram", getattr(self, "telegram", None)),
                                                          ("emby", getattr(self, "emby", None)))
                  if c is not None and c.limiter is not None}
        if limits:
            out["rate_limits"] = limits
        http_stats = getattr(self._http, "stats", None)
        if callable(http_stats):  # keep-alive pool accounting (sinks/h1.py)
            out["http"] = http_stats()
        store_pool = getattr(self._store, "_pool", None)
        if store_pool is not None and hasattr(store_pool, "connections"):
            out["store"] = {"connections": store_pool.connections}
        return out


async def run_service(config: Config, **kw) -> Dict[str, Any]:
    """Build, initialise, run to completion and close a service."""
    svc = Service(config, **kw)
    try:
        await svc.init()
        return await svc.run()
    finally:
        await svc.close()
