"""malloc bytes in use (mallinfo2) over plain-HTTP connection churn of the H1 client: one request
per connection (the server closes each), against tests/test_h1.py's scripted server in this process
(its request log cleared as it goes, so only the client's allocations remain).

    python scripts/churn_probe.py 24000
"""
import asyncio
import ctypes
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from beholder_amd.sinks import H1Client  # noqa: E402
import test_h1  # noqa: E402


class MI2(ctypes.Structure):
    _fields_ = [(n, ctypes.c_size_t) for n in ("arena","ordblks","smblks","hblks","hblkhd","usmblks","fsmblks","uordblks","fordblks","keepcost")]
libc = ctypes.CDLL("libc.so.6"); libc.mallinfo2.restype = MI2
def inuse(): gc.collect(); return libc.mallinfo2().uordblks / 1e6
CLOSE = b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\nConnection: close\r\n\r\n{}"
async def go(n):
    s = await test_h1.Scripted(lambda k, m, t, h: (s.requests.clear(), (CLOSE, "close"))[1]).start()
    c = H1Client(timeout_s=5)
    marks = []
    for i in range(n):
        await c.request("POST", f"http://127.0.0.1:{s.port}/1/cards/c{i%7}/actions/comments", params={"text": "x", "key": "k"})
        if i in (2000, n // 2, n - 1):
            marks.append((i, round(inuse(), 3), c.counts.get("connections") if hasattr(c, "counts") else None))
    await c.close(); await s.stop()
    return marks
print(asyncio.run(go(int(sys.argv[1]))))
