"""Price GPU offload of the per-event decode against the service's CPU decode (MI355X box).

The service decodes each event on arrival with the native codec (ops/csrc/py_codec.cpp). The
alternative is to gather a batch of events in pinned memory, copy it to HBM, decode with
ops/hip/telemetry_decode.hip and copy the field table back. This script times both for a range
of batch sizes:

* cpu_decode_ns: the native codec, per message (what the service does today);
* gpu: pack (host), H2D + kernel + D2H + synchronize (wall), kernel alone (HIP events), and
  materialise (turning table rows into the Python values the handlers use, in C);
* added_latency_us: how long the first event of a batch waits for its fields.

Output: one JSON object (stdout). docs/DESIGN.md "Why there are no HIP kernels in the event path" cites it.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from beholder_amd import ops  # noqa: E402
from beholder_amd.bench.generator import Workload  # noqa: E402
from beholder_amd.models import proto  # noqa: E402
from beholder_amd.ops import gpu_decode as gd  # noqa: E402


def best(fn, reps: int):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), statistics.median(ts)


def main() -> int:
    if not torch.cuda.is_available():
        print(json.dumps({"error": "no GPU"}))
        return 1
    dev = torch.device("cuda", 0)
    # the service's own decoders: the protobufjs dialect (handlers._dialect), as the kernel's default
    codecs = {1: ops.codec_for(proto.load("api.TelemetryStatus"), "protobufjs"),
              2: ops.codec_for(proto.load("api.TelemetryProgress"), "protobufjs")}
    evs = list(Workload(n_media=1024, seed=1).events(262_144))
    out = {"device": torch.cuda.get_device_name(0), "messages": len(evs),
           "mean_bytes": round(sum(len(b) for _, b in evs) / len(evs), 1), "batches": []}

    # the service today: one native decode per event, as it arrives
    sample = evs[:65536]
    decs = [(codecs[t].decode, b) for t, b in sample]

    def cpu_all():
        for dec, b in decs:
            dec(b)
    mn, med = best(cpu_all, 5)
    out["cpu_decode_ns"] = round(mn / len(sample) * 1e9, 1)

    for n in (1, 64, 1024, 16384, 262144):
        bodies = [b for _, b in evs[:n]]
        buf, offs = gd.pack(bodies)
        gd.check_layout(len(buf), offs)
        h_buf = torch.empty(len(buf), dtype=torch.uint8, pin_memory=True)
        h_buf.numpy()[:] = np.frombuffer(buf, dtype=np.uint8)
        h_offs = torch.from_numpy(offs).pin_memory()
        h_out = torch.empty((n, 8), dtype=torch.int32, pin_memory=True)
        d_buf = torch.empty(len(buf), dtype=torch.uint8, device=dev)
        d_offs = torch.empty(n + 1, dtype=torch.int32, device=dev)
        d_out = torch.empty((n, 8), dtype=torch.int32, device=dev)

        def pack():
            b2, o2 = gd.pack(bodies)
            h_buf.numpy()[:len(b2)] = np.frombuffer(b2, dtype=np.uint8)
            h_offs.numpy()[:] = o2

        def roundtrip():
            d_buf.copy_(h_buf, non_blocking=True)
            d_offs.copy_(h_offs, non_blocking=True)
            gd.decode_batch(d_buf, d_offs, n, d_out)
            h_out.copy_(d_out, non_blocking=True)
            torch.cuda.synchronize()

        tab = h_out.numpy()

        def materialise():  # native (C) rows -> Python values, the handlers' input
            gd.materialise(buf, tab)

        reps = 50 if n <= 16384 else 10
        for _ in range(3):
            roundtrip()
        assert np.array_equal(tab[:min(n, 512)], gd.reference_table(bodies[:min(n, 512)], "protobufjs"))
        p_mn, _ = best(pack, reps)
        r_mn, r_med = best(roundtrip, reps)
        m_mn, _ = best(materialise, max(3, reps // 5))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ks = []
        for _ in range(reps):
            e0.record()
            gd.decode_batch(d_buf, d_offs, n, d_out)
            e1.record()
            e1.synchronize()
            ks.append(e0.elapsed_time(e1) * 1e3)
        ku = []  # the same launch in the upb dialect (the other template instantiation)
        for _ in range(reps):
            e0.record()
            gd.decode_batch(d_buf, d_offs, n, d_out, dialect="upb")
            e1.record()
            e1.synchronize()
            ku.append(e0.elapsed_time(e1) * 1e3)
        gpu_ns = (p_mn + r_mn + m_mn) / n * 1e9
        out["batches"].append({
            "n": n, "bytes": len(buf),
            "pack_ns_per_msg": round(p_mn / n * 1e9, 1),
            "roundtrip_us": round(r_mn * 1e6, 1), "roundtrip_median_us": round(r_med * 1e6, 1),
            "kernel_us": round(min(ks), 2), "kernel_upb_us": round(min(ku), 2),
            "materialise_ns_per_msg": round(m_mn / n * 1e9, 1),
            "gpu_total_ns_per_msg": round(gpu_ns, 1),
            "vs_cpu_decode": round(gpu_ns / out["cpu_decode_ns"], 2),
            "added_latency_us": round((p_mn + r_mn) * 1e6, 1),
        })
        print(f"n={n}: {out['batches'][-1]}", file=sys.stderr, flush=True)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
