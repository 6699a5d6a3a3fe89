"""The RCCL watchdog (runtime.hip): every RCCL call
records an event behind it and a host thread ends the process with status 3
when the calls enqueued since the stream was last drained have not completed
within PINC_COMM_TIMEOUT seconds.

A single-rank RCCL communicator works on one GPU, so each case runs in a
child process: a communicator of one rank, an allreduce held behind a kernel
that occupies the stream for a bounded time (pinc_hip_test_spin, which ends
by itself), then a stream synchronisation.
  * timeout 1 s, spin 4 s: the watchdog fires -- exit status 3 and the
    "[pinc rank 0] RCCL watchdog" message naming the allreduce;
  * timeout 5 s (and the default 300 s), spin 2 s: it must not fire -- the
    allreduce completes and its result is the input (one rank).
"""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent

pytestmark = pytest.mark.gpu

_CHILD = r"""
import ctypes as C, sys
import numpy as np
sys.path.insert(0, {root!r})
from pinc_amd import _lib
H = _lib.HIP
spin = float(sys.argv[1])
assert H.pinc_hip_set_device(0) == 0
st = C.c_void_p()
assert H.pinc_hip_stream_create(C.byref(st)) == 0
cid = _lib.comm_unique_id()
comm = C.c_void_p()
buf = (C.c_ubyte * len(cid)).from_buffer_copy(cid)
assert H.pinc_hip_comm_init(C.byref(comm), buf, 1, 0) == 0, H.pinc_hip_error_string()
n = 1024
d = C.c_void_p()
assert H.pinc_hip_malloc(C.byref(d), C.c_ulong(8 * n)) == 0
x = np.arange(n, dtype=np.float64)
assert H.pinc_hip_h2d(d, x.ctypes.data_as(C.c_void_p), C.c_ulong(8 * n), st) == 0
H.pinc_hip_test_spin.argtypes = [C.c_double, C.c_void_p]
assert H.pinc_hip_test_spin(spin, st) == 0, H.pinc_hip_error_string()
H.pinc_hip_comm_note(b"watchdog test allreduce")
assert H.pinc_hip_comm_allreduce_sum(comm, d, d, C.c_long(n), st) == 0, H.pinc_hip_error_string()
assert H.pinc_hip_stream_sync(st) == 0
y = np.zeros(n)
assert H.pinc_hip_d2h(y.ctypes.data_as(C.c_void_p), d, C.c_ulong(8 * n), st) == 0
assert H.pinc_hip_stream_sync(st) == 0
assert np.array_equal(x, y)
assert H.pinc_hip_comm_destroy(comm) == 0
print("completed", flush=True)
"""


def _run(spin: float, timeout_env):
    env = dict(os.environ)
    env.pop("PINC_COMM_TIMEOUT", None)
    if timeout_env is not None:
        env["PINC_COMM_TIMEOUT"] = str(timeout_env)
    return subprocess.run([sys.executable, "-c", _CHILD.format(root=str(ROOT)), str(spin)], env=env,
                          capture_output=True, text=True, timeout=120)


def test_watchdog_fires_on_a_stalled_call(built):
    r = _run(4.0, 1)
    assert r.returncode == 3, (r.returncode, r.stdout[-800:], r.stderr[-2000:])
    assert "[pinc rank 0] RCCL watchdog" in r.stderr and "PINC_COMM_TIMEOUT" in r.stderr, r.stderr[-2000:]
    assert "allreduce" in r.stderr
    assert "completed" not in r.stdout


@pytest.mark.parametrize("timeout_env", [5, None])
def test_watchdog_quiet_when_calls_complete(built, timeout_env):
    r = _run(2.0, timeout_env)
    assert r.returncode == 0, (r.returncode, r.stdout[-800:], r.stderr[-2000:])
    assert "completed" in r.stdout
    assert "watchdog" not in r.stderr
