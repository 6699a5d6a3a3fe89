"""Kernel-level GPU tests through the C ABI (libpinc_hip.so), device memory
from torch.  Reference values come from the library's own reference-order
kernels or from plain numpy restatements of the same arithmetic.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class Lvl(C.Structure):
    _fields_ = [("nd", C.c_int), ("T", C.c_int * 3)]


@pytest.fixture(scope="module")
def hip(built):
    import torch
    assert torch.cuda.is_available()
    from pinc_amd import _lib
    h = _lib.HIP
    vp = C.c_void_p
    h.pinc_hip_gs_sweep.argtypes = [vp, vp, vp, Lvl, vp]
    h.pinc_hip_gs_pass.argtypes = [vp, vp, Lvl, C.c_int, C.c_int, vp, vp, C.POINTER(C.c_int), vp]
    return h


@pytest.mark.parametrize("shape", [(16, 16, 16), (32, 48, 64), (64, 32, 16)])
def test_fused_sweep_equals_two_passes(hip, shape):
    """k_gs_sweep (native mode) is one red-black iteration of mgGS3D, bit for
    bit equal to the red pass followed by the black pass."""
    import torch
    tx, ty, tz = shape
    n = tx * ty * tz
    g = torch.Generator(device="cpu").manual_seed(1)
    phi = torch.randn(n, dtype=torch.float64, generator=g).cuda()
    rho = torch.randn(n, dtype=torch.float64, generator=g).cuda()
    out = torch.empty_like(phi)
    L = Lvl(3, (C.c_int * 3)(tx, ty, tz))
    assert hip.pinc_hip_gs_sweep(phi.data_ptr(), out.data_ptr(), rho.data_ptr(), L, None) == 0
    ref = phi.clone()
    part = torch.empty(8192, dtype=torch.float64, device="cuda")
    nb = C.c_int()
    for p in (0, 1):
        assert hip.pinc_hip_gs_pass(ref.data_ptr(), rho.data_ptr(), L, p, 1, None, part.data_ptr(),
                                    C.byref(nb), None) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # and against a numpy restatement of the red-black iteration
    a = phi.cpu().numpy().reshape(tz, ty, tx).copy()
    r = rho.cpu().numpy().reshape(tz, ty, tx)
    z, y, x = np.meshgrid(np.arange(tz), np.arange(ty), np.arange(tx), indexing="ij")
    for colour in (0, 1):
        m = ((x + y + z) & 1) == colour
        s = (np.roll(a, -1, 2) + np.roll(a, 1, 2)) + np.roll(a, -1, 1)
        s = ((s + np.roll(a, 1, 1)) + np.roll(a, -1, 0)) + np.roll(a, 1, 0)
        a = np.where(m, (1.0 / 6.0) * (s + r), a)
    np.testing.assert_array_equal(out.cpu().numpy().reshape(tz, ty, tx), a)


def test_fused_sweep_rejects_untiled_level(hip):
    L = Lvl(3, (C.c_int * 3)(24, 16, 16))
    assert hip.pinc_hip_gs_sweep(None, None, None, L, None) != 0
