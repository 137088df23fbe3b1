"""Host facts for sizing consumer processes, read without importing torch or touching HIP.

The bench launcher (``bench.py``) and the multi-process runner (``parallel/workers.py``) size the
number of competing consumers from the CPUs and GPU slots of the node. Counting
GPUs through ``torch.cuda.device_count()`` is only HIP-free while torch finds ``amdsmi``; if it
falls back to ``hipGetDeviceCount`` the counting process has initialised HIP, and such a process
must not fork+exec consumers afterwards. So GPUs are counted here from the KFD topology in sysfs
and the DRM render nodes under ``/dev``, which is what the ROCm runtime enumerates itself.
"""
from __future__ import annotations

import glob
import os
from typing import Dict, Mapping, Optional

_VISIBLE_VARS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def _kfd_properties(path: str) -> Dict[str, int]:
    out: Dict[str, int] = {}
    try:
        with open(path) as f:
            for ln in f:
                k, _, v = ln.strip().partition(" ")
                try:
                    out[k] = int(v)
                except ValueError:
                    pass
    except OSError:
        pass
    return out


def _openable(dev: str) -> bool:
    """A render node this process may use: present and openable (a device cgroup denies the open)."""
    try:
        fd = os.open(dev, os.O_RDWR | os.O_CLOEXEC)
    except OSError:
        return False
    os.close(fd)
    return True


def gpus_on_node(sys_root: str = "/sys", dev_root: str = "/dev", env: Optional[Mapping[str, str]] = None,
                 check_open: bool = True) -> int:
    """GPUs this process can use, from sysfs: KFD topology nodes with SIMDs (CPU nodes have none)
    whose DRM render node exists under ``dev_root`` (and opens, with ``check_open``), capped by the
    ``*_VISIBLE_DEVICES`` variables. 0 on a host without a GPU driver. Never imports torch."""
    env = os.environ if env is None else env
    n = 0
    for props in sorted(glob.glob(os.path.join(sys_root, "class/kfd/kfd/topology/nodes/*/properties"))):
        p = _kfd_properties(props)
        if p.get("simd_count", 0) <= 0:
            continue
        minor = p.get("drm_render_minor", -1)
        if minor < 0:
            continue
        dev = os.path.join(dev_root, "dri", f"renderD{minor}")
        if not os.path.exists(dev) or (check_open and not _openable(dev)):
            continue
        n += 1
    for var in _VISIBLE_VARS:
        v = env.get(var)
        if v is None:
            continue
        ids = [x for x in v.split(",") if x.strip()]
        n = min(n, len(ids))
    return n


def available_cpus() -> int:
    """CPUs this process may use: affinity mask, capped by a cgroup v2/v1 CPU quota."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return max(1, n)


def cgroup_cpu_quota() -> Optional[float]:
    """The CFS quota in CPUs (cgroup v2 ``cpu.max`` or v1 ``cfs_quota_us``), None without one."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return q / p if q > 0 else None
    except (OSError, ValueError):
        return None


def cpu_share() -> dict:
    """What the CPU budget is made of: affinity CPUs, the cgroup quota (CPUs, None = no quota)
    and the distinct physical cores behind the affinity CPUs. On the MI355X pool the share is a
    16-CPU quota over all 256 hardware threads, so consumers run next to other tenants' work and
    a many-process number moves with host load (profiles/box_r1_share/)."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = list(range(os.cpu_count() or 1))
    cores = set()
    for c in aff:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            with open(base + "physical_package_id") as f1, open(base + "core_id") as f2:
                cores.add((f1.read().strip(), f2.read().strip()))
        except OSError:
            cores.add(("?", str(c)))
    q = cgroup_cpu_quota()
    return {"affinity_cpus": len(aff), "quota_cpus": None if q is None else round(q, 2),
            "physical_cores": len(cores)}


def default_procs(local_world: int, gpus: Optional[int] = None) -> int:
    """Consumer processes per rank: the CPU share of one GPU slot minus one, at most 16.

    The share is the node's CPUs divided by the number of GPU slots on the node (at least the
    local world size). It does not depend on how many ranks run, so per-rank work stays fixed
    as N grows (weak scaling): on an 8-GPU node with 16 CPUs per GPU, N=1 and N=8 both run 15
    consumers per rank.
    """
    slots = max(1, local_world, gpus_on_node() if gpus is None else gpus)
    return max(1, min(16, available_cpus() // slots - 1))


def cgroup_cpu_stat() -> Dict[str, int]:
    """CFS throttling counters of this process's cgroup: ``nr_periods``, ``nr_throttled`` and
    ``throttled_usec`` (cgroup v2 ``cpu.stat``; v1 ``cpu/cpu.stat``, whose ``throttled_time`` is
    in ns). Empty when no CPU controller is visible. A phase whose delta shows throttling ran
    against the share's quota, not against its own code."""
    for path, ns in (("/sys/fs/cgroup/cpu.stat", False), ("/sys/fs/cgroup/cpu/cpu.stat", True),
                     ("/sys/fs/cgroup/cpu,cpuacct/cpu.stat", True)):
        try:
            with open(path) as f:
                raw = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
        except (OSError, ValueError):
            continue
        out: Dict[str, int] = {}
        for k in ("nr_periods", "nr_throttled"):
            if k in raw:
                out[k] = int(raw[k])
        if "throttled_usec" in raw:
            out["throttled_usec"] = int(raw["throttled_usec"])
        elif "throttled_time" in raw:
            out["throttled_usec"] = int(raw["throttled_time"]) // 1000 if ns else int(raw["throttled_time"])
        if out:
            return out
    return {}


def cgroup_delta(before: Mapping[str, int], after: Mapping[str, int]) -> Dict[str, int]:
    return {k: after[k] - before.get(k, 0) for k in after}


def host_cpu_times() -> Optional[tuple]:
    """(busy, total) jiffies of the whole host from /proc/stat's ``cpu`` line (all CPUs, all
    tenants: /proc/stat is not namespaced), or None."""
    try:
        with open("/proc/stat") as f:
            parts = f.readline().split()
    except OSError:
        return None
    if not parts or parts[0] != "cpu":
        return None
    v = [int(x) for x in parts[1:]]
    idle = v[3] + (v[4] if len(v) > 4 else 0)  # idle + iowait
    total = sum(v[:8])  # user nice system idle iowait irq softirq steal (guest is inside user)
    return total - idle, total


def host_busy_pct(before: Optional[tuple], after: Optional[tuple]) -> Optional[float]:
    """Share of the host's CPU time that was busy between two :func:`host_cpu_times` readings:
    how loaded the machine was around a phase, whoever loaded it."""
    if not before or not after or after[1] <= before[1]:
        return None
    return round(100.0 * (after[0] - before[0]) / (after[1] - before[1]), 1)


def thread_run_delay_ns() -> Optional[int]:
    """Nanoseconds the calling thread has spent runnable but waiting for a CPU
    (``/proc/thread-self/schedstat`` field 2), or None where the kernel has no schedstat. A loop
    stall with this moving is the host's (no CPU to wake on), not the loop's own work."""
    try:
        with open("/proc/thread-self/schedstat") as f:
            return int(f.read().split()[1])
    except (OSError, IndexError, ValueError):
        return None


def proc_run_delay_ns(pid="self") -> Optional[int]:
    """Run-queue wait of every thread of a process so far (the sum of ``schedstat`` field 2 over
    ``/proc/<pid>/task/*``), or None. Threads that exited meanwhile drop out of the sum, so take
    differences over a window in which the process keeps its threads."""
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return None
    total = 0
    for t in tids:
        try:
            with open(f"/proc/{pid}/task/{t}/schedstat") as f:
                total += int(f.read().split()[1])
        except (OSError, IndexError, ValueError):
            continue
    return total


def proc_cpu_s(pid: int) -> Optional[float]:
    """User + system CPU seconds a process has used so far (``/proc/<pid>/stat`` fields 14-15),
    or None when it is gone. The e2e bench phases read it for each fake around the measured window,
    so a slow phase can be put on the consumer or on the processes it talks to."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            raw = f.read()
    except OSError:
        return None
    # the command name (field 2) may hold spaces and parentheses: split after its last ')'
    fields = raw[raw.rfind(")") + 2:].split()
    try:
        ticks = int(fields[11]) + int(fields[12])  # utime, stime (fields 14 and 15 of the line)
    except (IndexError, ValueError):
        return None
    return ticks / os.sysconf("SC_CLK_TCK")
