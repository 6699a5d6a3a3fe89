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


def _small_levels(tx, ty):
    lv = []
    while True:
        lv.append((tx, ty))
        if tx % 2 or ty % 2 or tx // 2 < 2 or ty // 2 < 2:
            break
        tx, ty = tx // 2, ty // 2
    return lv


def _small_solve(hip, phi, rho, lv, npre, npost, ncoarse, cycles, basis=None):
    import torch
    n = len(lv)
    arr = (Lvl * n)(*[Lvl(2, (C.c_int * 3)(a, b, 1)) for a, b in lv])
    res = torch.empty_like(phi)
    out = torch.zeros(64, dtype=torch.float64, device="cuda")
    rc = hip.pinc_hip_mg_solve_small(phi.data_ptr(), rho.data_ptr(), res.data_ptr(), n, arr, npre, npost, ncoarse,
                                     cycles, 1e-10, None if basis is None else basis.data_ptr(), out.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _fourier_basis(n):
    """The real orthonormal Fourier basis and its eigenvalues, as
    pinc_mg.c's small_basis builds them (the launcher's coarseBasis)."""
    hn = n // 2
    j = np.arange(n)[:, None]
    k = np.arange(n)[None, :]
    Q = np.where(k == 0, 1 / np.sqrt(n),
                 np.where(k < hn, np.sqrt(2 / n) * np.cos(2 * np.pi * (j * k % n) / n),
                          np.where(k == hn, np.where(j % 2, -1.0, 1.0) / np.sqrt(n),
                                   np.sqrt(2 / n) * np.sin(2 * np.pi * (j * (k - hn) % n) / n))))
    f = np.where(np.arange(n) <= hn, np.arange(n), np.arange(n) - hn)
    lam = 2.0 - 2.0 * np.cos(2 * np.pi * f / n)
    return np.concatenate([Q.ravel(), lam])


@pytest.mark.parametrize("shape", [(128, 128), (64, 32), (16, 128), (128, 64)])
def test_small_solve_vcycle_equals_per_level_launches(hip, shape):
    """pinc_hip_mg_solve_small without a basis: each cycle bit for bit the
    per-level launches of the native V-cycle (k_gs_pass x 2 nPre, k_residual,
    k_restrict, x 4, k_mg_coarse for levels 1.., k_prolong_add, k_gs_pass x
    2 nPost), over three cycles; the history is the RMS residual after each
    cycle (to 1e-12: another summation order)."""
    import torch
    vp = C.c_void_p
    hip.pinc_hip_mg_solve_small.argtypes = [vp, vp, vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.c_double, vp, vp, vp]
    hip.pinc_hip_residual.argtypes = [vp, vp, vp, Lvl, vp]
    hip.pinc_hip_restrict.argtypes = [vp, vp, Lvl, C.c_int, vp]
    hip.pinc_hip_scale.argtypes = [vp, C.c_long, C.c_double, vp]
    hip.pinc_hip_mg_coarse.argtypes = [vp, vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp]
    hip.pinc_hip_prolong_add.argtypes = [vp, vp, Lvl, vp]
    tx, ty = shape
    lv = _small_levels(tx, ty)
    g = torch.Generator(device="cpu").manual_seed(3)
    rho = torch.randn(tx * ty, dtype=torch.float64, generator=g)
    rho -= rho.mean()
    rho = rho.cuda()
    phi0 = torch.randn(tx * ty, dtype=torch.float64, generator=g).cuda()
    npre, npost, ncoarse = 4, 4, 10
    phi = phi0.clone()
    out = _small_solve(hip, phi, rho, lv, npre, npost, ncoarse, 3)
    assert out[0] == 3
    # the per-level launches
    ref = phi0.clone()
    L = [Lvl(2, (C.c_int * 3)(a, b, 1)) for a, b in lv]
    arr = (Lvl * (len(lv) - 1))(*L[1:])
    res = torch.empty_like(ref)
    n1 = lv[1][0] * lv[1][1]
    rho1 = torch.empty(n1, dtype=torch.float64, device="cuda")
    phi1 = torch.empty(n1, dtype=torch.float64, device="cuda")
    nb = C.c_int()
    hist = []
    for _ in range(3):
        for _ in range(npre):
            for p in (0, 1):
                assert hip.pinc_hip_gs_pass(ref.data_ptr(), rho.data_ptr(), L[0], p, 0, None, None, C.byref(nb),
                                            None) == 0
        assert hip.pinc_hip_residual(res.data_ptr(), ref.data_ptr(), rho.data_ptr(), L[0], None) == 0
        assert hip.pinc_hip_restrict(res.data_ptr(), rho1.data_ptr(), L[1], 0, None) == 0
        assert hip.pinc_hip_scale(rho1.data_ptr(), n1, 4.0, None) == 0
        assert hip.pinc_hip_mg_coarse(rho1.data_ptr(), phi1.data_ptr(), len(lv) - 1, arr, npre, npost, ncoarse, 0, 0,
                                      None) == 0
        assert hip.pinc_hip_prolong_add(ref.data_ptr(), phi1.data_ptr(), L[0], None) == 0
        for _ in range(npost):
            for p in (0, 1):
                assert hip.pinc_hip_gs_pass(ref.data_ptr(), rho.data_ptr(), L[0], p, 0, None, None, C.byref(nb),
                                            None) == 0
        assert hip.pinc_hip_residual(res.data_ptr(), ref.data_ptr(), rho.data_ptr(), L[0], None) == 0
        torch.cuda.synchronize()
        hist.append(float(torch.sqrt(torch.sum(res * res) / (tx * ty))))
    assert torch.equal(phi, ref)
    np.testing.assert_allclose(out[2:5], hist, rtol=1e-12)


@pytest.mark.parametrize("size", [64, 128])
def test_small_solve_spectral_cycle_matches_numpy(hip, size):
    """pinc_hip_mg_solve_small with the Fourier basis: one two-grid cycle
    (multigrid:spectralCoarse) against a numpy restatement -- red-black
    Gauss-Seidel (blk_update's order), the residual, the half-weight
    restriction x 4, the level-1 correction equation solved exactly (numpy
    FFT with the 5-point symbol, DC dropped), the bilinear prolongation --
    to 1e-12 of max |phi| (the f64 matrix-core products round differently
    from the FFT); then a full solve to an RMS residual <= 1e-10."""
    import torch
    vp = C.c_void_p
    hip.pinc_hip_mg_solve_small.argtypes = [vp, vp, vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.c_double, vp, vp, vp]
    n = size
    lv = _small_levels(n, n)
    g = np.random.default_rng(5)
    r = g.standard_normal((n, n))
    r -= r.mean()
    p0 = g.standard_normal((n, n))
    basis = torch.from_numpy(_fourier_basis(n // 2)).cuda()
    rho = torch.from_numpy(r.ravel().copy()).cuda()
    phi = torch.from_numpy(p0.ravel().copy()).cuda()
    out = _small_solve(hip, phi, rho, lv, 4, 4, 10, 1, basis)
    assert out[0] == 1
    y, x = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")

    def smooth(a, k):
        for _ in range(k):
            for colour in (0, 1):
                s = np.roll(a, -1, 1) + np.roll(a, 1, 1)
                s = s + (np.roll(a, -1, 0) + np.roll(a, 1, 0))
                a = np.where(((x + y) & 1) == colour, (s + r) * 0.25, a)
        return a

    def resid(a):
        q = -4.0 * a + (np.roll(a, -1, 1) + np.roll(a, 1, 1))
        return q + (np.roll(a, -1, 0) + np.roll(a, 1, 0)) + r

    a = smooth(p0, 4)
    q = resid(a)
    rc = (4.0 * q + (np.roll(q, -1, 1) + np.roll(q, 1, 1)) + (np.roll(q, -1, 0) + np.roll(q, 1, 0))) / 8.0
    r1 = rc[::2, ::2] * 4.0
    m = n // 2
    k = 2 * np.pi * np.fft.fftfreq(m)
    sym = (2 - 2 * np.cos(k))[:, None] + (2 - 2 * np.cos(k))[None, :]
    sym[0, 0] = 1.0
    f = np.fft.fft2(r1) / sym
    f[0, 0] = 0.0
    p1 = np.real(np.fft.ifft2(f))
    # bilinear prolongation (prol_low: y first, then x along the lowest odd
    # dimension)
    pf = np.zeros((n, n))
    pf[::2, ::2] = p1
    pf[1::2, ::2] = 0.5 * (p1 + np.roll(p1, -1, 0))
    pf[:, 1::2] = 0.5 * (pf[:, ::2] + np.roll(pf[:, ::2], -1, 1))
    a = smooth(a + pf, 4)
    got = phi.cpu().numpy().reshape(n, n)
    assert np.max(np.abs(got - a)) <= 1e-12 * np.max(np.abs(a))
    np.testing.assert_allclose(out[2], np.sqrt(np.mean(resid(a) ** 2)), rtol=1e-9)
    # a whole solve
    out = _small_solve(hip, phi, rho, lv, 4, 4, 10, 200, basis)
    assert out[1] <= 1e-10 and 1 <= out[0] < 200
    got = phi.cpu().numpy().reshape(n, n)
    assert np.sqrt(np.mean(resid(got) ** 2)) <= 1.1e-10
