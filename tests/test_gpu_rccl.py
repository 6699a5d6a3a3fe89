"""The RCCL leg of the C ABI on hardware ("the RCCL collectives
have never executed").

RCCL refuses two ranks on one device, so multi-rank runs on the one-GPU test
box use the host transport.  What can run here is a one-rank communicator:
every call the multi-rank path makes (pinc_hip_comm_init, the grouped
send/recv of pinc_hip_comm_exchange as used by the halo and migrant
exchanges, pinc_hip_comm_allgather, pinc_hip_comm_allreduce_sum,
pinc_hip_comm_destroy) is executed through the library on device buffers
and its result checked.  Self send/recv is how the reference exchanges with
itself under periodic boundaries (grid.c:379-403).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip(built):
    from pinc_amd import _lib
    h = _lib.HIP
    vp = C.c_void_p
    sigs = {
        "pinc_hip_set_device": [C.c_int],
        "pinc_hip_stream_create": [C.POINTER(vp)],
        "pinc_hip_stream_destroy": [vp],
        "pinc_hip_stream_sync": [vp],
        "pinc_hip_malloc": [C.POINTER(vp), C.c_ulong],
        "pinc_hip_free": [vp],
        "pinc_hip_h2d": [vp, vp, C.c_ulong, vp],
        "pinc_hip_d2h": [vp, vp, C.c_ulong, vp],
        "pinc_hip_comm_init": [C.POINTER(vp), C.c_void_p, C.c_int, C.c_int],
        "pinc_hip_comm_destroy": [vp],
        "pinc_hip_comm_exchange": [vp, C.c_int, C.POINTER(C.c_int), C.POINTER(vp), C.POINTER(C.c_long),
                                   C.POINTER(C.c_int), C.POINTER(vp), C.POINTER(C.c_long), vp],
        "pinc_hip_comm_allgather": [vp, vp, vp, C.c_long, vp],
        "pinc_hip_comm_allreduce_sum": [vp, vp, vp, C.c_long, vp],
    }
    for n, a in sigs.items():
        getattr(h, n).argtypes = a
        getattr(h, n).restype = C.c_int
    assert h.pinc_hip_set_device(0) == 0
    return h, _lib


def _dev(h, nbytes):
    p = C.c_void_p()
    assert h.pinc_hip_malloc(C.byref(p), nbytes) == 0
    return p


def test_one_rank_rccl_collectives(hip):
    h, lib = hip
    st = C.c_void_p()
    assert h.pinc_hip_stream_create(C.byref(st)) == 0
    uid = lib.comm_unique_id()
    idbuf = (C.c_ubyte * len(uid)).from_buffer_copy(uid)
    comm = C.c_void_p()
    rc = h.pinc_hip_comm_init(C.byref(comm), C.cast(idbuf, C.c_void_p), 1, 0)
    assert rc == 0, h.pinc_hip_error_string()
    n = 66564  # one ghost plane of a C4 z-slab (258 x 258 doubles)
    rng = np.random.default_rng(5)
    a = rng.standard_normal(n)
    b = rng.standard_normal(n)
    bufs = [_dev(h, 8 * n) for _ in range(4)]
    try:
        assert h.pinc_hip_h2d(bufs[0], a.ctypes.data, 8 * n, st) == 0
        assert h.pinc_hip_h2d(bufs[1], b.ctypes.data, 8 * n, st) == 0
        # two paired ops to self (the z+1 and z-1 exchanges of one rank)
        peers = (C.c_int * 2)(0, 0)
        sends = (C.c_void_p * 2)(bufs[0], bufs[1])
        recvs = (C.c_void_p * 2)(bufs[2], bufs[3])
        nb = (C.c_long * 2)(8 * n, 8 * n)
        rc = h.pinc_hip_comm_exchange(comm, 2, peers, sends, nb, peers, recvs, nb, st)
        assert rc == 0, h.pinc_hip_error_string()
        assert h.pinc_hip_stream_sync(st) == 0
        got = np.zeros(n)
        assert h.pinc_hip_d2h(got.ctypes.data, bufs[2], 8 * n, st) == 0
        assert np.array_equal(got, a)
        assert h.pinc_hip_d2h(got.ctypes.data, bufs[3], 8 * n, st) == 0
        assert np.array_equal(got, b)
        # allgather of one rank is a copy; allreduce of one rank is identity
        assert h.pinc_hip_comm_allgather(comm, bufs[0], bufs[2], n, st) == 0
        assert h.pinc_hip_comm_allreduce_sum(comm, bufs[1], bufs[3], n, st) == 0
        assert h.pinc_hip_stream_sync(st) == 0
        assert h.pinc_hip_d2h(got.ctypes.data, bufs[2], 8 * n, st) == 0
        assert np.array_equal(got, a)
        assert h.pinc_hip_d2h(got.ctypes.data, bufs[3], 8 * n, st) == 0
        assert np.array_equal(got, b)
    finally:
        for p in bufs:
            h.pinc_hip_free(p)
        assert h.pinc_hip_comm_destroy(comm) == 0
        h.pinc_hip_stream_destroy(st)
