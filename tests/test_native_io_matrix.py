"""``BEHOLDER_NATIVE_IO``, the one native-I/O switch (utils/netconn.py): the handler, service,
chaos and H1 suites pass with all native I/O on and with all of it off (sockets on asyncio
transports, TLS included; Python request paths for the H1 client and the Postgres pool; replies
on plain asyncio futures). The switch is read at import, so each side runs in its own process."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITES = ["tests/test_handlers.py", "tests/test_service.py", "tests/test_chaos.py", "tests/test_h1_fast.py",
          "tests/test_direct_dispatch.py"]


@pytest.mark.parametrize("native_io", ["1", "0"])
def test_suites_pass_with_native_io(native_io):
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-x", "--timeout", "120", *SUITES, "-rs"],
                       cwd=ROOT, capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, BEHOLDER_NATIVE_IO=native_io))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    if native_io == "0":  # the native-only H1 tests say why they did not run
        assert "native I/O switched off" in r.stdout
    else:
        assert "skipped" not in r.stdout.splitlines()[-1]


def test_no_per_component_switches_left():
    """The A/B switches of rounds 1-2 are gone from the code; the compiled handlers read no
    private module globals of other layers (they use the clients' capabilities)."""
    gone = ("BEHOLDER_NATIVE_NET", "BEHOLDER_NATIVE_H1", "BEHOLDER_NATIVE_TLS", "BEHOLDER_NATIVE_POLLER",
            "BEHOLDER_NATIVE_POOL", "BEHOLDER_NATIVE_HANDLERS", "BEHOLDER_NATIVE_DISPATCH", "BEHOLDER_IOFUTURE",
            "BEHOLDER_PG_BACKGROUND_GROW")
    hits = []
    for d, _, files in os.walk(os.path.join(ROOT, "beholder_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hpp")):
                text = open(os.path.join(d, f), encoding="utf-8").read()
                hits += [(f, g) for g in gone if g in text]
    assert hits == []
    src = open(os.path.join(ROOT, "beholder_amd", "ops", "csrc", "py_handlers.cpp"), encoding="utf-8").read()
    assert "_h1_fast" not in src and "_pg_pool_execute" not in src
