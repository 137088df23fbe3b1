"""Build the native runtime in-tree (``beholder_amd/ops/_native*.so``), the bench/test natives
(``beholder_amd/ops/_native_bench*.so``, not part of the service) and the HIP offload probe
(``beholder_amd/ops/hip/libbeholder_hip.so``, gfx950).

Beholder's runtime around the Python handlers (ingest reader thread, ring,
codec, deliveries, histograms) is C++ — see ``csrc/``. The service has no
device kernels in its event path (the reference has none), so the runtime is a
host build with the system C++ compiler. ``build_hip`` compiles the batched-decode kernel that
``scripts/gpu_offload_probe.py`` measures against it (``ops/gpu_decode.py``).
``__graft_entry__.build()`` calls both.

The HIP library is optional for the service: ``main`` builds it only when ``hipcc`` is present
(``--hip`` makes it required, ``--no-hip`` skips it), so the deployment image and CI, which have
no ROCm, build the runtime alone.

Usage: ``python -m beholder_amd.ops.build [--debug] [--sanitize=address,undefined] [--coverage] [--hip|--no-hip]
[--no-bench]`` (``--coverage``: gcov-instrumented, objects and their ``.gcno`` / ``.gcda`` kept under
``build/coverage/``; ``scripts/native_coverage.py`` and ``make coverage`` use it)
(thin CLI over this module)
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ops")
CSRC = os.path.join(HERE, "csrc")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
TARGET = os.path.join(HERE, "_native" + EXT_SUFFIX)
STAMP = TARGET + ".srchash"


# OpenSSL for the native TLS connections (ops/csrc/py_tls.cpp): the same libssl the interpreter's
# `ssl` module loads (headers from libssl-dev)
LIBS = ["-lssl", "-lcrypto"]


# bench / test / diagnostic natives (the sink stub, the paced producer, calibration loops, the
# sampling profiler): a module of their own, `_native_bench`, never linked into the service's
# extension; the runtime image does not build it (`--no-bench`, Dockerfile)
CSRC_BENCH = os.path.join(HERE, "csrc_bench")
BENCH_TARGET = os.path.join(HERE, "_native_bench" + EXT_SUFFIX)


def sources(src_dir: str = CSRC) -> list:
    return sorted(glob.glob(os.path.join(src_dir, "*.cpp")))


def source_hash(flags: list, dirs=(CSRC,)) -> str:
    h = hashlib.sha256()
    for d in dirs:
        for p in sorted(glob.glob(os.path.join(d, "*"))):
            with open(p, "rb") as f:
                h.update(os.path.basename(p).encode())
                h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


# objects of a --coverage build (gcov reads the .gcno written at compile time and the .gcda the
# instrumented extension writes next to them at exit)
COVERAGE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "coverage")


def compile_flags(debug: bool = False, sanitize: str = "", coverage: bool = False) -> list:
    inc = sysconfig.get_paths()["include"]
    flags = ["-std=c++17", "-fPIC", "-shared", "-pthread", "-fvisibility=hidden",
             "-Wall", "-Wextra", "-Wno-missing-field-initializers", "-Wno-cast-function-type",
             f"-I{inc}", f"-I{CSRC}", f"-I{CSRC_BENCH}"]
    if coverage:  # line / branch counts per source line: unoptimised, counters updated atomically
        flags += ["-O0", "-g", "--coverage", "-fprofile-update=atomic"]
    elif debug:
        flags += ["-O0", "-g"]
    else:
        # x86-64-v2 keeps the .so portable across the build container and the
        # GPU box hosts (both are x86-64 with SSE4.2/POPCNT); other machines get the compiler's default
        import platform
        flags += ["-O3", "-DNDEBUG"] + (["-march=x86-64-v2", "-mtune=generic"]
                                         if platform.machine() in ("x86_64", "AMD64") else [])
    if sanitize:
        flags += [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer", "-g"]
    return flags


def _stamp_matches(target: str, stamp: str, digest: str) -> bool:
    if not (os.path.exists(target) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read().strip() == digest


def _write_atomic(path: str, text: str) -> None:
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)


class _BuildLock:
    """``flock`` on ``<target>.lock``: one compile per tree, however many processes import at
    once (workers of ``run --workers N`` starting together, parallel test runners). The others
    wait, then find the stamp current and load what the first one built."""

    def __init__(self, target: str):
        self.path = target + ".lock"
        self.fd = -1

    def __enter__(self):
        import fcntl
        self.fd = os.open(self.path, os.O_RDWR | os.O_CREAT, 0o644)
        fcntl.flock(self.fd, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl
        fcntl.flock(self.fd, fcntl.LOCK_UN)
        os.close(self.fd)
        self.fd = -1


def build(force: bool = False, debug: bool = False, sanitize: str = "", cxx: str = "", verbose: bool = False,
          coverage: bool = False) -> str:
    """The service's extension ``_native`` from ``csrc/``."""
    return _build_module(TARGET, sources(CSRC), (CSRC,), LIBS, force, debug, sanitize, cxx, verbose, coverage)


def build_bench(force: bool = False, debug: bool = False, sanitize: str = "", cxx: str = "",
                verbose: bool = False, coverage: bool = False) -> str:
    """The bench/test extension ``_native_bench`` from ``csrc_bench/`` (headers from ``csrc/``:
    it calls the service's code through ``_native._C_API``, never links it)."""
    return _build_module(BENCH_TARGET, sources(CSRC_BENCH), (CSRC_BENCH, CSRC), [], force, debug, sanitize, cxx,
                         verbose, coverage)


def coverage_objdir(target: str) -> str:
    """Where a --coverage build of ``target`` keeps its objects (and gcov its counts)."""
    return os.path.join(COVERAGE_DIR, os.path.basename(target).split(".")[0])


def _build_module(target: str, srcs: list, dirs: tuple, libs: list, force: bool, debug: bool, sanitize: str,
                  cxx: str, verbose: bool, coverage: bool = False) -> str:
    cxx = cxx or os.environ.get("CXX") or "g++"
    flags = compile_flags(debug, sanitize, coverage)
    stamp = target + ".srchash"
    # hash path-independent flags so a snapshot copied elsewhere (GPU box) reuses the .so
    digest = source_hash([f for f in flags if not f.startswith("-I")] + libs + [cxx, sysconfig.get_config_var("SOABI") or ""],
                         dirs)
    if not force and _stamp_matches(target, stamp, digest):
        return target
    with _BuildLock(target):
        if not force and _stamp_matches(target, stamp, digest):  # built while this process waited
            return target
        print(f"beholder: building the native runtime ({os.path.basename(target)}, pid {os.getpid()})",
              file=sys.stderr)
        tmp = f"{target}.{os.getpid()}.tmp"  # per process: nothing else ever writes this file
        # compile translation units in parallel (one compiler process each), then link
        import concurrent.futures
        import tempfile
        cflags = [f for f in flags if f != "-shared"]
        jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 1), 16))
        try:
            if coverage:
                import shutil
                shutil.rmtree(coverage_objdir(target), ignore_errors=True)  # stale counts with the objects
                os.makedirs(coverage_objdir(target))
            with tempfile.TemporaryDirectory(prefix="beholder-build-") as tmpd:
                td = coverage_objdir(target) if coverage else tmpd

                def compile_one(src: str) -> str:
                    obj = os.path.join(td, os.path.basename(src) + ".o")
                    cmd = [cxx, *cflags, "-c", src, "-o", obj]
                    if verbose:
                        print(" ".join(cmd), file=sys.stderr)
                    subprocess.run(cmd, check=True)
                    return obj
                with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
                    objs = list(ex.map(compile_one, srcs))
                link = [cxx, *[f for f in flags if not f.startswith("-I") and not f.startswith("-W")], *objs, *libs,
                        "-o", tmp]
                if verbose:
                    print(" ".join(link), file=sys.stderr)
                subprocess.run(link, check=True)
            os.replace(tmp, target)
        finally:
            if os.path.exists(tmp):
                os.unlink(tmp)
        _write_atomic(stamp, digest)
    return target


HIP_DIR = os.path.join(HERE, "hip")
HIP_TARGET = os.path.join(HIP_DIR, "libbeholder_hip.so")
HIP_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
             "-Wall", "-Wextra"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC", ""), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    import shutil
    return shutil.which("hipcc") or ""


def build_hip(force: bool = False, verbose: bool = False) -> str:
    """Compile ``ops/hip/*.hip`` for gfx950 into one shared library (cached by source hash)."""
    cc = hipcc()
    if not cc:
        raise RuntimeError("hipcc not found (ROCm is required to build the HIP extension)")
    srcs = sorted(glob.glob(os.path.join(HIP_DIR, "*.hip")))
    h = hashlib.sha256(" ".join(HIP_FLAGS).encode())
    for p in srcs:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode())
            h.update(f.read())
    digest = h.hexdigest()
    stamp = HIP_TARGET + ".srchash"
    if not force and _stamp_matches(HIP_TARGET, stamp, digest):
        return HIP_TARGET
    with _BuildLock(HIP_TARGET):
        if not force and _stamp_matches(HIP_TARGET, stamp, digest):
            return HIP_TARGET
        tmp = f"{HIP_TARGET}.{os.getpid()}.tmp"
        cmd = [cc, *HIP_FLAGS, *srcs, "-o", tmp]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        try:
            subprocess.run(cmd, check=True)
            os.replace(tmp, HIP_TARGET)
        finally:
            if os.path.exists(tmp):
                os.unlink(tmp)
        _write_atomic(stamp, digest)
    return HIP_TARGET


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--sanitize", default="")
    ap.add_argument("--coverage", action="store_true", help="gcov-instrumented build (objects kept in build/coverage)")
    ap.add_argument("--cxx", default="")
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--hip", action="store_true", help="require the gfx950 HIP extension (fail without hipcc)")
    g.add_argument("--no-hip", action="store_true", help="skip the gfx950 HIP extension")
    ap.add_argument("--no-bench", action="store_true",
                    help="skip the bench/test extension _native_bench (the runtime image ships only the service)")
    a = ap.parse_args(argv)
    print(build(force=a.force, debug=a.debug, sanitize=a.sanitize, cxx=a.cxx, verbose=True, coverage=a.coverage))
    if not a.no_bench:
        print(build_bench(force=a.force, debug=a.debug, sanitize=a.sanitize, cxx=a.cxx, verbose=True,
                          coverage=a.coverage))
    if a.no_hip or a.sanitize or a.coverage:
        return 0
    if not a.hip and not hipcc():
        print("hipcc not found: skipping the optional gfx950 HIP extension (ops/hip); the service does not use it",
              file=sys.stderr)
        return 0
    print(build_hip(force=a.force, verbose=True))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
