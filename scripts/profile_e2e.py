"""cProfile of the production-shaped `tcp_e2e` config: AMQP + Postgres + HTTP sinks, all over
TCP, in one consumer process. The broker and endpoint fakes run in other processes, so they are
not in the profile. Prints the top functions by self time, then by cumulative time."""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from beholder_amd.bench import harness  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
prof = cProfile.Profile()
prof.enable()
res = harness.run_config("tcp_e2e", events=n)
prof.disable()
print({k: res[k] for k in ("events", "acked", "ingest_rate_eps", "cpu_us_per_event", "sys_cpu_us_per_event")})
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats(key).print_stats(35)
    print(s.getvalue())
