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
    h.pinc_hip_gs_sweep2x.argtypes = [vp, vp, vp, Lvl, vp]
    h.pinc_hip_gs_pass.argtypes = [vp, vp, Lvl, C.c_int, C.c_int, vp, vp, C.POINTER(C.c_int), vp]
    return h


@pytest.mark.parametrize("shape", [(16, 16, 16), (32, 48, 64), (64, 32, 16), (64, 32, 96)])
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


@pytest.mark.parametrize("shape", [(32, 8, 16), (64, 32, 96), (32, 16, 64), (96, 24, 32)])
def test_double_sweep_equals_two_sweeps(hip, shape):
    """k_gs_sweep4 (two red-black iterations per launch, four-stage z-march)
    is bit for bit equal to two single-iteration sweeps, and to the numpy
    restatement of two red-black iterations."""
    import torch
    tx, ty, tz = shape
    n = tx * ty * tz
    g = torch.Generator(device="cpu").manual_seed(2)
    phi = torch.randn(n, dtype=torch.float64, generator=g).cuda()
    rho = torch.randn(n, dtype=torch.float64, generator=g).cuda()
    out = torch.full_like(phi, float("nan"))
    mid = torch.empty_like(phi)
    ref = torch.empty_like(phi)
    L = Lvl(3, (C.c_int * 3)(tx, ty, tz))
    assert hip.pinc_hip_gs_sweep2x(phi.data_ptr(), out.data_ptr(), rho.data_ptr(), L, None) == 0
    assert hip.pinc_hip_gs_sweep(phi.data_ptr(), mid.data_ptr(), rho.data_ptr(), L, None) == 0
    assert hip.pinc_hip_gs_sweep(mid.data_ptr(), ref.data_ptr(), rho.data_ptr(), L, None) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    a = phi.cpu().numpy().reshape(tz, ty, tx).copy()
    r = rho.cpu().numpy().reshape(tz, ty, tx)
    z, y, x = np.meshgrid(np.arange(tz), np.arange(ty), np.arange(tx), indexing="ij")
    for colour in (0, 1, 0, 1):
        m = ((x + y + z) & 1) == colour
        s = (np.roll(a, -1, 2) + np.roll(a, 1, 2)) + np.roll(a, -1, 1)
        s = ((s + np.roll(a, 1, 1)) + np.roll(a, -1, 0)) + np.roll(a, 1, 0)
        a = np.where(m, (1.0 / 6.0) * (s + r), a)
    np.testing.assert_array_equal(out.cpu().numpy().reshape(tz, ty, tx), a)


def test_fused_sweep_rejects_untiled_level(hip):
    L = Lvl(3, (C.c_int * 3)(24, 16, 16))
    assert hip.pinc_hip_gs_sweep(None, None, None, L, None) != 0


class Geom(C.Structure):
    _fields_ = [("nd", C.c_int), ("T", C.c_int * 3), ("nloc", C.c_int), ("off", C.c_int), ("nranks", C.c_int),
                ("literal", C.c_int)]


class Pop(C.Structure):
    _fields_ = [("x", C.c_void_p * 3), ("v", C.c_void_p * 3), ("nSpecies", C.c_int), ("nd", C.c_int),
                ("iStart", C.c_long * 9), ("iStop", C.c_long * 8)]


@pytest.mark.parametrize("n,T,start", [(100_000, (16, 16, 16), 0), (77_777, (32, 16, 8), 13), (5, (8, 8, 8), 1)])
def test_cell_sort(hip, n, T, start):
    """pinc_hip_sort_tiles: a permutation of the particles, ordered by the
    tile-major cell key, with pos and vel moved together."""
    import torch
    rng = np.random.default_rng(n)
    cap = start + n + 3
    pos = [torch.zeros(cap, dtype=torch.float64) for _ in range(3)]
    vel = [torch.zeros(cap, dtype=torch.float64) for _ in range(3)]
    for d in range(3):
        pos[d][start:start + n] = torch.from_numpy(0.1 + rng.random(n) * (T[d] + 0.8))
        vel[d][start:start + n] = torch.from_numpy(rng.standard_normal(n))
    pos = [p.cuda() for p in pos]
    vel = [v.cuda() for v in vel]
    out_p = [torch.zeros_like(p) for p in pos]
    out_v = [torch.zeros_like(v) for v in vel]
    pop = Pop((C.c_void_p * 3)(*[p.data_ptr() for p in pos]), (C.c_void_p * 3)(*[v.data_ptr() for v in vel]),
              1, 3, (C.c_long * 9)(start, start + n + 3), (C.c_long * 8)(start + n))
    out = Pop((C.c_void_p * 3)(*[p.data_ptr() for p in out_p]), (C.c_void_p * 3)(*[v.data_ptr() for v in out_v]),
              1, 3, (C.c_long * 9)(start, start + n + 3), (C.c_long * 8)(start + n))
    g = Geom(3, (C.c_int * 3)(*T), T[2], 0, 1)
    hip.pinc_hip_sort_tiles.argtypes = [Pop, Pop, C.c_int, Geom, C.c_int, C.c_void_p, C.c_long,
                                        C.POINTER(C.c_long), C.c_void_p]
    nk = C.c_long()
    assert hip.pinc_hip_sort_tiles(pop, out, 0, g, 4, None, 0, C.byref(nk), None) != 0
    need = 2 * (nk.value + 1) + 2 * (nk.value // 4096 + 1) + 1
    work = torch.zeros(need, dtype=torch.int32, device="cuda")
    assert hip.pinc_hip_sort_tiles(pop, out, 0, g, 4, work.data_ptr(), need, C.byref(nk), None) == 0
    torch.cuda.synchronize()
    P = np.stack([p.cpu().numpy()[start:start + n] for p in out_p], 1)
    V = np.stack([v.cpu().numpy()[start:start + n] for v in out_v], 1)
    P0 = np.stack([p.cpu().numpy()[start:start + n] for p in pos], 1)
    V0 = np.stack([v.cpu().numpy()[start:start + n] for v in vel], 1)
    c = P.astype(int)
    nt = [(t + 1) // 4 + 1 for t in T]
    # tile_key_of (k_particles.hip): tiles along a serpentine (x rows
    # alternate direction, y columns alternate per z plane), the z layers of
    # odd tiles reversed, cells x fastest inside a layer
    t = c // 4
    ty = np.where(t[:, 2] % 2 == 1, nt[1] - 1 - t[:, 1], t[:, 1])
    r = t[:, 2] * nt[1] + ty
    tx = np.where(r % 2 == 1, nt[0] - 1 - t[:, 0], t[:, 0])
    tile = r * nt[0] + tx
    inz = np.where(tile % 2 == 1, 3 - c[:, 2] % 4, c[:, 2] % 4)
    key = tile * 64 + (c[:, 0] % 4) + 4 * ((c[:, 1] % 4) + 4 * inz)
    assert np.all(np.diff(key) >= 0)
    a = np.concatenate([P, V], 1)
    b = np.concatenate([P0, V0], 1)
    np.testing.assert_array_equal(a[np.lexsort(a.T[::-1])], b[np.lexsort(b.T[::-1])])


@pytest.mark.parametrize("hw3d", [1, 0])
@pytest.mark.parametrize("shape", [(4, 4, 4), (32, 8, 16), (64, 32, 96), (96, 24, 32)])
def test_resid_restrict_equals_residual_then_restrict(hip, shape, hw3d):
    """pinc_hip_resid_restrict (k_resid_restrict3p: x pairs, the residual
    never stored) is bit for bit the residual (mgResidual), then the
    restriction (mgHalfRestrict3D or the ND form), then the native x4; and
    the residual norm (k_residual_sumsq3p) matches numpy's to rounding."""
    import torch
    vp = C.c_void_p
    hip.pinc_hip_resid_restrict.argtypes = [vp, vp, vp, Lvl, C.c_int, C.c_double, vp]
    hip.pinc_hip_residual.argtypes = [vp, vp, vp, Lvl, vp]
    hip.pinc_hip_restrict.argtypes = [vp, vp, Lvl, C.c_int, vp]
    hip.pinc_hip_scale.argtypes = [vp, C.c_long, C.c_double, vp]
    hip.pinc_hip_residual_sumsq.argtypes = [vp, vp, Lvl, vp, C.POINTER(C.c_int), vp]
    hip.pinc_hip_reduce.argtypes = [vp, C.c_int, C.c_double, vp, vp]
    tx, ty, tz = shape
    n = tx * ty * tz
    g = torch.Generator(device="cpu").manual_seed(5)
    phi = torch.randn(n, dtype=torch.float64, generator=g).cuda()
    rho = torch.randn(n, dtype=torch.float64, generator=g).cuda()
    Lf = Lvl(3, (C.c_int * 3)(tx, ty, tz))
    Lc = Lvl(3, (C.c_int * 3)(tx // 2, ty // 2, tz // 2))
    nc = n // 8
    out = torch.full((nc,), float("nan"), dtype=torch.float64, device="cuda")
    res = torch.empty_like(phi)
    ref = torch.empty_like(out)
    assert hip.pinc_hip_resid_restrict(phi.data_ptr(), rho.data_ptr(), out.data_ptr(), Lc, hw3d, 4.0, None) == 0
    assert hip.pinc_hip_residual(res.data_ptr(), phi.data_ptr(), rho.data_ptr(), Lf, None) == 0
    assert hip.pinc_hip_restrict(res.data_ptr(), ref.data_ptr(), Lc, hw3d, None) == 0
    assert hip.pinc_hip_scale(ref.data_ptr(), nc, 4.0, None) == 0
    part = torch.empty(65536, dtype=torch.float64, device="cuda")
    tot = torch.empty(1, dtype=torch.float64, device="cuda")
    nb = C.c_int()
    assert hip.pinc_hip_residual_sumsq(phi.data_ptr(), rho.data_ptr(), Lf, part.data_ptr(), C.byref(nb), None) == 0
    assert hip.pinc_hip_reduce(part.data_ptr(), nb.value, 1.0, tot.data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    a = phi.cpu().numpy().reshape(tz, ty, tx)
    r = rho.cpu().numpy().reshape(tz, ty, tx)
    s = (np.roll(a, -1, 2) + np.roll(a, 1, 2)) + np.roll(a, -1, 1)
    s = ((s + np.roll(a, 1, 1)) + np.roll(a, -1, 0)) + np.roll(a, 1, 0)
    resn = (-6.0 * a + s) + r
    np.testing.assert_array_equal(res.cpu().numpy().reshape(tz, ty, tx), resn)
    np.testing.assert_allclose(tot.item(), float((resn * resn).sum()), rtol=1e-12)
