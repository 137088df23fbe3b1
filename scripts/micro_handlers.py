"""Per-event CPU cost of the compiled handlers, split by branch (main-thread CPU time).

Deliveries are pre-built and driven through dispatch_batch directly (no ingest thread), so
the numbers are the handler path alone: decode, log lines, counters, store read, the Trello
request through the in-process recorder, ack. Run on the target host; prints ns/event.
"""
import array
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from beholder_amd.bench.generator import Workload  # noqa: E402
from beholder_amd.handlers import native_handlers  # noqa: E402
from beholder_amd.ops import Delivery, Settler, dispatch_batch  # noqa: E402
from beholder_amd.sinks import RecordingHttpClient, SinkObserver, TrelloClient  # noqa: E402
from beholder_amd.utils.log import Logger  # noqa: E402
from helpers import Rig  # noqa: E402


def run(label, level="info", trello_fraction=0.5, progress_fraction=0.9, native=True, n=200_000):
    w = Workload(n_media=2000, seed=1, trello_fraction=trello_fraction, progress_fraction=progress_fraction)
    evs = w.events(n)
    r = Rig(medias=w.media, http=RecordingHttpClient(keep=16))
    r.h.log = r.log = Logger(stream=open(os.devnull, "w"), level=level)
    r.h.trello = TrelloClient("k", "t", r.http, observer=SinkObserver(r.registry))
    impl = native_handlers(r.h) if native else r.h
    s = Settler()
    ds = [Delivery(b, t, i, s) for i, (t, b) in enumerate(evs)]
    routes = (None, impl.on_status, impl.on_progress)
    cnt = array.array("Q", [0, 0, 0])
    t0 = time.thread_time()
    dispatch_batch(ds, 0, routes, cnt, None, None, None)
    dt = time.thread_time() - t0
    print(f"{label:48s} {dt / n * 1e9:7.0f} ns/event", flush=True)


if __name__ == "__main__":
    run("bench mix (90% progress, 50% Trello media)")
    run("bench mix, Python handlers", native=False)
    run("progress only, no Trello media", trello_fraction=0.0, progress_fraction=1.0)
    run("progress only, all Trello media", trello_fraction=1.0, progress_fraction=1.0)
    run("progress only, no Trello, log level warn", level="warn", trello_fraction=0.0, progress_fraction=1.0)
    run("progress only, all Trello, log level warn", level="warn", trello_fraction=1.0, progress_fraction=1.0)
    run("status only", progress_fraction=0.0)
