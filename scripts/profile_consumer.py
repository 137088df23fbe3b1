"""cProfile of one bench consumer (single process), top functions by self time.

The service has no GPU kernels, so the per-event CPU profile is the relevant
profile (rocprofv3 would show zero kernel dispatches).
"""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = ["bench.py", "--steps", "6", "--warmup", "1", "--procs-per-rank", "1"]
import runpy  # noqa: E402

prof = cProfile.Profile()
prof.enable()
try:
    runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
except SystemExit:
    pass
prof.disable()
s = io.StringIO()
pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(40)
print(s.getvalue())
