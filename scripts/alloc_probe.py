"""Python allocations that survive a paced production-path run (tcp_e2e at RATE events/s, N events):
tracemalloc snapshots around the measured phase, the largest differences with their tracebacks.

    python scripts/alloc_probe.py N RATE
"""
import sys, tracemalloc, gc
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from beholder_amd.bench import harness
snaps = {}
def start():
    gc.collect(); snaps['a'] = tracemalloc.take_snapshot()
def stop():
    gc.collect(); snaps['b'] = tracemalloc.take_snapshot()
tracemalloc.start(12)
r = harness._tcp_e2e(int(sys.argv[1]), rate=float(sys.argv[2]), hooks=(start, stop), stall_period_s=0.001)
print('measured', r['measured_events'], 'cpu', r['cpu_us_per_event'], 'rss growth', r['rss_growth_mb'])
diff = snaps['b'].compare_to(snaps['a'], 'traceback')
tot = sum(s.size_diff for s in diff)
print('total python alloc diff bytes', tot)
for s in diff[:8]:
    print(s.size_diff, s.count_diff)
    for line in s.traceback.format()[-8:]:
        print('   ', line)
