"""CPU (user, sys) per operation of the two production clients in isolation: H1Client requests and pgwire
queries against the bench fakes (separate processes), `prefetch` operations in flight like the
service. Prints one JSON line: rusage CPU µs per operation (this process only) and ops/s."""
import asyncio
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from beholder_amd.bench import harness  # noqa: E402
from beholder_amd.sinks import H1Client  # noqa: E402
from beholder_amd.store.postgres import PostgresStore  # noqa: E402


def cpu() -> "tuple":
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime, r.ru_stime


def per_op(c0, c1, n: int, key: str) -> dict:
    return {f"{key}_user_us": (c1[0] - c0[0]) / n * 1e6, f"{key}_sys_us": (c1[1] - c0[1]) / n * 1e6}


async def bench_http(port: int, n: int, inflight: int = 100) -> dict:
    h = H1Client(timeout_s=30)
    url = f"http://127.0.0.1:{port}"

    async def worker(k):
        for i in range(k):
            await h.request("POST", f"{url}/1/cards/c{i % 5000}/actions/comments",
                            params={"key": "K", "token": "T", "text": "CONVERTING: Progress **5%**"})
    await asyncio.gather(*(worker(200) for _ in range(inflight)))  # warm: pool filled
    c0, t0 = cpu(), time.perf_counter()
    await asyncio.gather(*(worker(n // inflight) for _ in range(inflight)))
    c1, t1 = cpu(), time.perf_counter()
    await h.close()
    return {**per_op(c0, c1, n, "http_per_req"), "http_req_per_s": n / (t1 - t0)}


async def bench_pg(port: int, n: int, inflight: int = 100) -> dict:
    st = PostgresStore(f"postgres://beholder@127.0.0.1:{port}/media", pool_size=4)
    await st.connect()

    async def worker(k, j):
        for i in range(k):
            try:
                await st.get_by_id(f"m{(i * 7 + j) % 10000}")
            except LookupError:
                pass
    await asyncio.gather(*(worker(200, j) for j in range(inflight)))
    c0, t0 = cpu(), time.perf_counter()
    await asyncio.gather(*(worker(n // inflight, j) for j in range(inflight)))
    c1, t1 = cpu(), time.perf_counter()
    await st.close()
    return {**per_op(c0, c1, n, "pg_per_query"), "pg_query_per_s": n / (t1 - t0)}


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    out = {}
    hport, hp = harness._spawn("beholder_amd.bench.http_sink_server", 2)
    pport, pp = harness._spawn("beholder_amd.bench.pg_sink_server", 2, ("--media", "10000", "--seed", "0"))
    try:
        out.update(asyncio.run(bench_http(hport, n)))
        out.update(asyncio.run(bench_pg(pport, n)))
    finally:
        harness._reap(hp + pp)
    print(json.dumps({k: round(v, 3) for k, v in out.items()}))


if __name__ == "__main__":
    main()
