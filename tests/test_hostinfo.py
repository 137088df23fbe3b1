"""GPU and CPU counting for consumer sizing (utils/hostinfo.py) without torch or HIP."""
import os
import subprocess
import sys

from beholder_amd.utils import hostinfo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fake_node(root, idx, simd, minor):
    d = root / "sys" / "class" / "kfd" / "kfd" / "topology" / "nodes" / str(idx)
    d.mkdir(parents=True)
    (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\ndrm_render_minor {minor}\n")


def _tree(tmp_path, gpus=3, with_dev=None):
    _fake_node(tmp_path, 0, 0, 0)  # CPU node: no SIMDs
    for i in range(gpus):
        _fake_node(tmp_path, i + 1, 1024, 128 + i)
    dri = tmp_path / "dev" / "dri"
    dri.mkdir(parents=True)
    for i in (range(gpus) if with_dev is None else with_dev):
        (dri / f"renderD{128 + i}").write_text("")
    return str(tmp_path / "sys"), str(tmp_path / "dev")


def test_counts_gpu_nodes_with_render_nodes(tmp_path):
    s, d = _tree(tmp_path, gpus=3)
    assert hostinfo.gpus_on_node(s, d, env={}) == 3


def test_render_node_missing_means_not_visible(tmp_path):
    s, d = _tree(tmp_path, gpus=8, with_dev=[2])  # a container that was given one card
    assert hostinfo.gpus_on_node(s, d, env={}) == 1


def test_visible_devices_cap(tmp_path):
    s, d = _tree(tmp_path, gpus=8)
    assert hostinfo.gpus_on_node(s, d, env={"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert hostinfo.gpus_on_node(s, d, env={"ROCR_VISIBLE_DEVICES": "3", "CUDA_VISIBLE_DEVICES": "0,1,2"}) == 1
    assert hostinfo.gpus_on_node(s, d, env={"CUDA_VISIBLE_DEVICES": ""}) == 0


def test_no_driver_no_gpus(tmp_path):
    assert hostinfo.gpus_on_node(str(tmp_path / "nope"), str(tmp_path / "nodev"), env={}) == 0


def test_default_procs_shares_cpus_per_gpu_slot(monkeypatch):
    monkeypatch.setattr(hostinfo, "available_cpus", lambda: 128)
    assert hostinfo.default_procs(1, gpus=8) == 15
    assert hostinfo.default_procs(8, gpus=8) == 15
    assert hostinfo.default_procs(1, gpus=0) == 16  # capped
    monkeypatch.setattr(hostinfo, "available_cpus", lambda: 2)
    assert hostinfo.default_procs(1, gpus=1) == 1


def test_default_procs_without_torch():
    """bench.py's sizing works with torch blocked from import (never imported, HIP never touched)."""
    code = ("import sys\n"
            "class Block:\n"
            "    def find_spec(self, name, path=None, target=None):\n"
            "        if name.split('.')[0] == 'torch':\n"
            "            raise ModuleNotFoundError(name, name=name)\n"
            "sys.meta_path.insert(0, Block())\n"
            "sys.path.insert(0, %r)\n"
            "from beholder_amd.utils.hostinfo import default_procs, gpus_on_node, available_cpus\n"
            "import bench\n"
            "n = default_procs(1)\n"
            "assert n == max(1, min(16, available_cpus() // max(1, gpus_on_node()) - 1)), n\n"
            "assert 'torch' not in sys.modules\n"
            "print(n)\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert int(r.stdout.strip()) >= 1


def test_host_busy_share_and_cgroup_stat_readers():
    from beholder_amd.utils import hostinfo as hi
    assert hi.host_busy_pct((10, 100), (60, 200)) == 50.0
    assert hi.host_busy_pct(None, (1, 2)) is None and hi.host_busy_pct((5, 10), (5, 10)) is None
    t = hi.host_cpu_times()
    assert t is None or (0 <= t[0] <= t[1])
    st = hi.cgroup_cpu_stat()  # whatever this host exposes: known keys, integer values
    assert set(st) <= {"nr_periods", "nr_throttled", "throttled_usec"}
    assert all(isinstance(v, int) for v in st.values())
    assert hi.cgroup_delta({"nr_throttled": 2}, {"nr_throttled": 5, "throttled_usec": 7}) == \
        {"nr_throttled": 3, "throttled_usec": 7}


def test_run_queue_delay_readers():
    """schedstat readers: this thread's and this process's time runnable but without a CPU
    (None where the kernel has no schedstat); the process total covers the thread's."""
    from beholder_amd.utils import hostinfo as hi
    t = hi.thread_run_delay_ns()
    p = hi.proc_run_delay_ns()
    if t is None:
        return
    assert isinstance(t, int) and t >= 0 and p is not None and p >= 0
    assert hi.proc_run_delay_ns(os.getpid()) >= t
    assert hi.proc_run_delay_ns(2 ** 22 + 12345) is None  # no such process
