"""The drop-in boundary of the reference's main.c, on CPU.

* Every library symbol src/main.c needs at link time -- the data in
  tests/golden/mainc_symbols.json, generated from the reference's main.c by
  tests/golden/make_mainc_symbols.py -- is exported by libpinc.so and
  declared in include/pinc.h.
* The launcher bootstrap's TCP host transport (pinc_boot.c, PINC_TRANSPORT=
  host), which lets several ranks of the C driver share one GPU, passes its
  self-test in 2 and 3 processes: rendezvous, mesh, paired neighbour
  exchange, allgather, allreduce.  No GPU is touched.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "pinc_amd" / "lib" / "libpinc.so"
SYMS = json.loads((ROOT / "tests" / "golden" / "mainc_symbols.json").read_text())


def _needed():
    return sorted(set(SYMS["functions"]) | set(SYMS["selectors"]) | set(SYMS["slice_ops"]))


def test_mainc_symbol_list_is_complete():
    """The list covers main.c's operators, objects, asserts, output and timer
    calls (a regression guard on the generator)."""
    need = set(_needed())
    for name in ("pVelAssertMax", "pPosAssertInLocalFrame", "oOpenH5", "oReadH5", "oCloseH5", "puMove",
                 "puMigrate", "gHaloOp", "selectInner", "tAlloc", "puAccND0KE_set", "puDistrND0_set",
                 "mgMode_set", "sSolver_set", "addSlice", "setSlice"):
        assert name in need, name
    assert not any(n.startswith(("MPI_", "gsl_")) for n in need)


def test_mainc_symbols_resolve_in_libpinc(built):
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in _needed() if n not in exported]
    assert not missing, f"main.c needs symbols libpinc.so does not export: {missing}"


def test_mainc_symbols_declared_in_header():
    sys.path.insert(0, str(ROOT))
    text = (ROOT / "include" / "pinc.h").read_text()
    import re
    missing = [n for n in _needed() if not re.search(rf"\b{n}\s*\(", text)]
    assert not missing, f"include/pinc.h does not declare: {missing}"


_WORKER = r"""
import ctypes, sys
lib = ctypes.CDLL(sys.argv[1])
rank, size = int(sys.argv[2]), int(sys.argv[3])
rc = lib.pinc_host_mesh_selftest(rank, size)
print("rank", rank, "rc", rc, flush=True)
sys.exit(0 if rc == 0 else 10 + rc)
"""


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("size", [2, 3])
def test_host_mesh_transport_selftest(built, size):
    env = dict(os.environ, PINC_MASTER_ADDR="127.0.0.1", PINC_MASTER_PORT=str(_free_port()), PINC_BOOT_TIMEOUT="60")
    procs = [subprocess.Popen([sys.executable, "-c", _WORKER, str(LIB), str(r), str(size)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(size)]
    outs = [p.communicate(timeout=120) for p in procs]
    for r, (p, (o, e)) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, (r, p.returncode, o[-500:], e[-1500:])
