"""Multi-process competing consumers: ``beholder run --workers N``.

The reference scales horizontally only by running more replicas that consume
the same RabbitMQ queues (SURVEY.md §2.3 "horizontal scaling"). One Python
process is bound by one core, so on a many-core host the idiomatic scale-out
is N worker processes on the same queues (the broker round-robins between
them, each with its own prefetch window). This module is the supervisor:

* spawns N children running the same ``run`` command with
  ``BEHOLDER_WORKER_ID=i``;
* metrics: the supervisor serves the *merged* exposition of all workers on
  the configured port (:mod:`beholder_amd.metrics.aggregate`). Worker ``i``
  listens on ``127.0.0.1:port+1+i``, so one scrape target covers the host;
* restarts a crashed worker with exponential backoff. The policy tells a crash
  loop from occasional crashes:

  - crashes are counted per worker in a sliding window: more than
    ``max_restarts`` crashes within ``restart_window_s`` is a crash loop;
  - the backoff (``backoff_base_s`` doubling up to ``backoff_max_s``) grows with
    the crashes still inside the window, and starts over once a worker has run
    for ``healthy_s`` (its earlier crashes no longer count);
  - a crash loop stops the supervisor: every worker gets SIGTERM and the exit
    code is 1. A worker that keeps crashing at once almost always means every
    worker will (bad config, unreachable dependency), and the non-zero exit lets
    the container orchestrator's restart policy and alerting see it. Crashes
    spread out over time (one a day for weeks) never add up to that;
* forwards SIGTERM/SIGINT and waits for graceful shutdown, then SIGKILLs
  stragglers after ``grace_s``.

Only broker transports can be shared (AMQP); a stdin/file stream has a single
reader.
"""
from __future__ import annotations

import collections
import os
import signal
import subprocess
import sys
import time
from typing import Deque, Dict, List, Optional


class RestartPolicy:
    """Per-worker crash accounting: sliding-window crash-loop detection and a backoff that
    resets after a healthy run (see the module docstring)."""

    def __init__(self, max_restarts: int = 10, restart_window_s: float = 300.0, healthy_s: float = 60.0,
                 backoff_base_s: float = 0.5, backoff_max_s: float = 30.0):
        if max_restarts < 0 or restart_window_s <= 0:
            raise ValueError("max_restarts must be >= 0 and restart_window_s > 0")
        self.max_restarts = max_restarts
        self.window_s = restart_window_s
        self.healthy_s = healthy_s
        self.base_s = backoff_base_s
        self.max_s = backoff_max_s
        self.crashes: Dict[int, Deque[float]] = collections.defaultdict(collections.deque)
        self.total: Dict[int, int] = collections.defaultdict(int)

    def on_crash(self, worker: int, started_at: float, now: float) -> Optional[float]:
        """Record a crash; the delay before the restart, or None for a crash loop (give up)."""
        q = self.crashes[worker]
        if now - started_at >= self.healthy_s:
            q.clear()  # ran healthy: earlier crashes no longer count towards the loop or the backoff
        while q and now - q[0] > self.window_s:
            q.popleft()
        q.append(now)
        self.total[worker] += 1
        if len(q) > self.max_restarts:
            return None
        return min(self.max_s, self.base_s * 2 ** (len(q) - 1))

    def recent(self, worker: int) -> int:
        return len(self.crashes[worker])


class Supervisor:
    def __init__(self, argv: List[str], workers: int, *, metrics_port: Optional[int] = None,
                 metrics_host: str = "0.0.0.0", max_restarts: int = 10, restart_window_s: float = 300.0,
                 healthy_s: float = 60.0, backoff_base_s: float = 0.5, backoff_max_s: float = 30.0,
                 grace_s: float = 15.0, env: Optional[Dict[str, str]] = None, log=print,
                 command: Optional[List[str]] = None, poll_s: float = 0.1):
        if workers < 1:
            raise ValueError("workers must be >= 1")
        self.argv = list(argv)
        self.n = workers
        self.metrics_port = metrics_port  # None / < 0: workers run without metrics endpoints
        self.metrics_host = metrics_host
        self.cluster_metrics = None
        self.policy = RestartPolicy(max_restarts, restart_window_s, healthy_s, backoff_base_s, backoff_max_s)
        self.grace_s = grace_s
        self.env = dict(os.environ if env is None else env)
        self.log = log
        # the worker program (tests substitute one); argv and --metrics-port are appended
        self.command = list(command) if command else [sys.executable, "-m", "beholder_amd"]
        self.poll_s = poll_s
        self.procs: Dict[int, subprocess.Popen] = {}
        self.started_at = [0.0] * workers
        self.next_start = [0.0] * workers
        self._stop = False

    @property
    def restarts(self) -> List[int]:
        """Crashes (restarts) per worker over the supervisor's lifetime."""
        return [self.policy.total[i] for i in range(self.n)]

    @property
    def _metrics_on(self) -> bool:
        return self.metrics_port is not None and self.metrics_port >= 0

    def worker_port(self, i: int) -> int:
        return self.metrics_port + 1 + i

    def _cmd(self, i: int) -> List[str]:
        cmd = [*self.command, *self.argv]
        cmd += ["--metrics-port", str(self.worker_port(i)) if self._metrics_on else "-1"]
        return cmd

    def _spawn(self, i: int) -> None:
        env = dict(self.env, BEHOLDER_WORKER_ID=str(i), BEHOLDER_WORKERS=str(self.n))
        if self._metrics_on:
            env["BEHOLDER_CFG__service__metrics__host"] = "127.0.0.1"  # internal; merged on the main port
        self.procs[i] = subprocess.Popen(self._cmd(i), env=env)
        self.started_at[i] = time.monotonic()
        self.log(f"worker {i} started pid={self.procs[i].pid}")

    def stop(self, *_a) -> None:
        self._stop = True

    def run(self) -> int:
        signal.signal(signal.SIGTERM, self.stop)
        signal.signal(signal.SIGINT, self.stop)
        if self._metrics_on:
            from ..metrics.aggregate import ClusterMetricsServer
            self.cluster_metrics = ClusterMetricsServer(
                self.metrics_host, self.metrics_port,
                worker_ports=lambda: [(i, self.worker_port(i)) for i in sorted(self.procs)],
                alive=lambda: not self._stop and len(self.procs) == self.n).start()
            self.log(f"merged metrics on {self.metrics_host}:{self.cluster_metrics.port}")
        for i in range(self.n):
            self._spawn(i)
        failed = False
        done = set()  # workers that exited cleanly (finite source)
        while not self._stop and len(done) < self.n:
            time.sleep(self.poll_s)
            for i in range(self.n):
                if i in done:
                    continue
                p = self.procs.get(i)
                if p is None:
                    if time.monotonic() >= self.next_start[i]:
                        self._spawn(i)
                    continue
                rc = p.poll()
                if rc is None:
                    continue
                del self.procs[i]
                if rc == 0:
                    self.log(f"worker {i} exited cleanly")
                    done.add(i)
                    continue
                now = time.monotonic()
                delay = self.policy.on_crash(i, self.started_at[i], now)
                if delay is None:
                    self.log(f"worker {i} crashed {self.policy.recent(i)} times within "
                             f"{self.policy.window_s:g}s (rc={rc}): crash loop, stopping all workers")
                    failed = True
                    self._stop = True
                    break
                self.log(f"worker {i} exited rc={rc}; restart in {delay:.1f}s "
                         f"({self.policy.recent(i)} crash(es) within {self.policy.window_s:g}s, "
                         f"{self.policy.total[i]} in total)")
                self.next_start[i] = now + delay
        return self._shutdown(failed)

    def _shutdown(self, failed: bool) -> int:
        if self.cluster_metrics is not None:
            self.cluster_metrics.stop()
        for p in self.procs.values():
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        deadline = time.monotonic() + self.grace_s
        rc = 1 if failed else 0
        for i, p in list(self.procs.items()):
            try:
                r = p.wait(max(0.0, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                r = p.wait()
                self.log(f"worker {i} killed after grace period")
            if r not in (0, -signal.SIGTERM):
                rc = rc or 1
        return rc


def strip_workers_arg(argv: List[str]) -> List[str]:
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a == "--workers":
            skip = True
            continue
        if a.startswith("--workers="):
            continue
        out.append(a)
    return out
