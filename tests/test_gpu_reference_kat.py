"""The reference's own particle known answers through the HIP kernels
(last part).

tests/test_oracle_kat.py runs these against the oracle on the CPU; here the
same data (tests/golden/reference_outputs.json "kat", restated from
test/pusher.test.c) goes through libpinc_hip.so's C ABI:

  * puAcc3D1 (pusher.test.c:82-121): E[p] = p over a 5x4x3 grid without
    ghosts, v0 = 100, q = m = dt = 1 -> v = (160, 161, 162) for a particle
    at a cell centre, v_x = 121.3 off centre; through pinc_hip_accelerate
    (k_accel<3, ...>, the kick the fused push inlines);
  * puDistr3D1 (pusher.test.c:123-204): four unit particles, the CIC
    fractions of 28 nodes; through pinc_hip_deposit (the LDS-boxed
    deposit kernel) and pinc_hip_deposit_cells (the cell-range deposit of
    the tiled layout);
  * testConstE (pusher.test.c:18-78): a half-step kick in uniform E, then
    move and accelerate n times, x_n = x_0 + (q/m)/2 n^2 to 1e-15; through
    pinc_hip_move_classify(doMove=1) and pinc_hip_accelerate.

The reference's grids have no ghost layers and are not periodic; the device
keeps the reference's local frame (true nodes at 1..T, slab ghost planes 0
and T+1).  So every position is shifted by +1 in each
dimension and the reference's node (j, k, l) is the device's storage node
(j, k, l + 1) (x/y stored from node 1, z from the ghost plane).  No test
position touches a node past the reference grid's edge, so the device's
periodic x/y wrap never engages.
"""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = json.loads((Path(__file__).parent / "golden" / "reference_outputs.json").read_text())["kat"]


class Geom(C.Structure):
    _fields_ = [("nd", C.c_int), ("T", C.c_int * 3), ("nloc", C.c_int), ("off", C.c_int), ("nranks", C.c_int),
                ("literal", C.c_int)]


class Pop(C.Structure):
    _fields_ = [("x", C.c_void_p * 3), ("v", C.c_void_p * 3), ("nSpecies", C.c_int), ("nd", C.c_int),
                ("iStart", C.c_long * 9), ("iStop", C.c_long * 8)]


@pytest.fixture(scope="module")
def hip(built):
    import torch
    assert torch.cuda.is_available()
    from pinc_amd import _lib
    h = _lib.HIP
    vp = C.c_void_p
    h.pinc_hip_accelerate.argtypes = [Pop, C.c_int, Geom, vp, vp, C.POINTER(C.c_int), vp]
    h.pinc_hip_deposit.argtypes = [Pop, C.c_int, Geom, vp, vp]
    h.pinc_hip_move_classify.argtypes = [Pop, C.c_int, C.c_int, vp, vp, vp, C.c_double, vp, C.c_int, vp]
    return h


def _device_pop(pos: np.ndarray, vel: np.ndarray, start: int = 0):
    """Species 0 at [start, start + n) of SoA device arrays (torch memory)."""
    import torch
    n = pos.shape[0]
    cap = start + n + 5
    xs, vs = [], []
    for d in range(3):
        a = np.zeros(cap)
        a[start:start + n] = pos[:, d]
        b = np.zeros(cap)
        b[start:start + n] = vel[:, d]
        xs.append(torch.from_numpy(a).cuda())
        vs.append(torch.from_numpy(b).cuda())
    pop = Pop((C.c_void_p * 3)(*[t.data_ptr() for t in xs]), (C.c_void_p * 3)(*[t.data_ptr() for t in vs]), 1, 3,
              (C.c_long * 9)(start, cap), (C.c_long * 8)(start + n))
    return pop, xs, vs


def _geom(T):
    return Geom(3, (C.c_int * 3)(*T), T[2], 0, 1, 0)


def _ref_to_device_grid(ref: np.ndarray, T, nvals: int) -> np.ndarray:
    """Reference value-major grid without ghosts ([l][k][j][v]) to the
    device slab [nloc+2][Ty][Tx][v]: reference plane l at device plane l+1."""
    tx, ty, tz = T
    out = np.zeros((tz + 2, ty, tx, nvals))
    out[1:tz + 1] = ref.reshape(tz, ty, tx, nvals)
    return out


@pytest.mark.parametrize("start", [0, 1, 7])
def test_puacc3d1_known_answers(hip, start):
    """pusher.test.c:82-121 through k_accel: 160/161/162 at the cell centre,
    121.3 off centre, to the reference's 1e-13 (exact here)."""
    import torch
    k = GOLD["puAcc3D1"]
    T = tuple(k["trueSize"])
    nref = 3 * int(np.prod(T))
    Es = torch.from_numpy(_ref_to_device_grid(np.arange(nref, dtype=np.float64), T, 3).ravel()).cuda()
    pos = np.array(k["pos"], dtype=np.float64) + 1.0
    vel = np.tile(np.array(k["vel0"], dtype=np.float64), (len(pos), 1))
    pop, xs, vs = _device_pop(pos, vel, start)
    part = torch.zeros(64, dtype=torch.float64, device="cuda")
    nb = C.c_int()
    assert hip.pinc_hip_accelerate(pop, 0, _geom(T), Es.data_ptr(), part.data_ptr(), C.byref(nb), None) == 0
    torch.cuda.synchronize()
    v = np.stack([t.cpu().numpy()[start:start + len(pos)] for t in vs], 1)
    assert np.all(np.abs(v[0] - np.array(k["expect_vel_p0"])) < k["tol"]), v[0]
    assert abs(v[1, 0] - k["expect_vel_p1_x"]) < k["tol"], v[1]
    # positions untouched, KE partial = sum v.(v+dv) over the particles
    p = np.stack([t.cpu().numpy()[start:start + len(pos)] for t in xs], 1)
    assert np.array_equal(p, pos)
    ke = float(part[:nb.value].sum())
    v0 = vel
    assert abs(ke - float(np.sum(v0 * v))) <= 1e-12 * abs(ke)


def _check_fractions(rho_dev: np.ndarray, T, k):
    tx, ty, tz = T
    rho = rho_dev.reshape(tz + 2, ty, tx)
    assert np.all(rho[0] == 0) and np.all(rho[tz + 1] == 0)   # nothing on the ghost planes
    ref = rho[1:tz + 1].ravel()
    for idx, frac in k["expect"].items():
        assert abs(ref[int(idx)] - frac) < k["tol"], (idx, ref[int(idx)], frac)
    untouched = np.setdiff1d(np.arange(ref.size), np.array([int(i) for i in k["expect"]]))
    assert np.all(ref[untouched] == 0)
    assert abs(ref.sum() - len(k["pos"])) < 1e-13


@pytest.mark.parametrize("start", [0, 3])
def test_pudistr3d1_known_answers(hip, start):
    """pusher.test.c:123-204 through the LDS-boxed deposit kernel: the 28
    node fractions of four unit particles (the caller's 1/q, q chain is not
    part of the kernel; unit charge)."""
    import torch
    k = GOLD["puDistr3D1"]
    T = tuple(k["trueSize"])
    pos = np.array(k["pos"], dtype=np.float64) + 1.0
    pop, xs, vs = _device_pop(pos, np.zeros_like(pos), start)   # (keep the tensors alive)
    rho = torch.zeros((T[2] + 2) * T[1] * T[0], dtype=torch.float64, device="cuda")
    assert hip.pinc_hip_deposit(pop, 0, _geom(T), rho.data_ptr(), None) == 0
    torch.cuda.synchronize()
    _check_fractions(rho.cpu().numpy(), T, k)


@pytest.mark.parametrize("qm", GOLD["constE"]["qm"])
def test_const_e_leapfrog_known_answer(hip, qm):
    """testConstE (pusher.test.c:18-78) through the move and accelerate
    kernels: E = (1, 0, 0) scaled by q/m (the field chain's Es), a half-step
    kick, then n moves and kicks; x_n - x_0 = (q/m)/2 n^2 exactly (all
    values are multiples of 1/4)."""
    import torch
    k = GOLD["constE"]
    T = (32, 32, 32)
    n = (T[2] + 2) * T[1] * T[0]
    E = np.zeros((n, 3))
    E[:, 0] = qm
    Es = torch.from_numpy(E.ravel()).cuda()
    Eh = torch.from_numpy((E * 0.5).ravel()).cuda()
    x0 = 17.0                       # the reference's 16 in the device frame
    pop, xs, vs = _device_pop(np.array([[x0, 17.0, 17.0]]), np.zeros((1, 3)))
    g = _geom(T)
    part = torch.zeros(64, dtype=torch.float64, device="cuda")
    nb = C.c_int()
    thr = (C.c_double * 9)(1, 1, 1, T[0] + 1, T[1] + 1, T[2] + 1, T[0] + 1, T[1] + 1, T[2] + 1)
    flags = torch.zeros(16, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(4, dtype=torch.int32, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert hip.pinc_hip_accelerate(pop, 0, g, Eh.data_ptr(), part.data_ptr(), C.byref(nb), None) == 0
    for step in range(1, k["steps"] + 1):
        assert hip.pinc_hip_move_classify(pop, 0, 1, thr, flags.data_ptr(), cnt.data_ptr(), 1e30, err.data_ptr(), 0,
                                          None) == 0
        assert hip.pinc_hip_accelerate(pop, 0, g, Es.data_ptr(), part.data_ptr(), C.byref(nb), None) == 0
        torch.cuda.synchronize()
        x = float(xs[0][0])
        assert abs(x - (x0 + 0.5 * qm * step * step)) < k["tol"], (qm, step, x)
        assert float(xs[1][0]) == 17.0 and float(xs[2][0]) == 17.0
    assert int(flags[0]) == 13 and int(cnt[0]) == 0 and int(err[0]) == 0   # stays in the subdomain


class PushArgs(C.Structure):
    """pinc_push_t (include/pinc_hip.h)."""
    _fields_ = [("xout", C.c_void_p * 3), ("vout", C.c_void_p * 3), ("kick", C.c_int), ("Es", C.c_void_p),
                ("rhoS", C.c_void_p), ("thr", C.c_void_p), ("flags", C.c_void_p), ("chunkCount", C.c_void_p),
                ("maxVel", C.c_double), ("errFlag", C.c_void_p), ("wrapMask", C.c_int), ("kePartial", C.c_void_p),
                ("tileWidth", C.c_int), ("cursor", C.c_void_p), ("cntNext", C.c_void_p), ("moved", C.c_void_p),
                ("spread", C.c_void_p), ("tstamp", C.c_void_p), ("diag", C.c_void_p), ("objInside", C.c_void_p),
                ("objSy", C.c_long), ("objSz", C.c_long), ("objNodes", C.c_long), ("objCount", C.c_void_p),
                ("objLo", C.c_int * 3), ("objHi", C.c_int * 3), ("emigTotal", C.c_void_p),
                ("flagsSparse", C.c_int)]


def _embedded_fractions(rho_dev: np.ndarray, T, k):
    """The reference's 5x4x3 node (j, k, l) inside a larger device slab T:
    storage node (j, k, l + 1); every other node must be zero."""
    kt = tuple(k["trueSize"])
    tx, ty, tz = T
    rho = rho_dev.reshape(tz + 2, ty, tx)
    sub = rho[1:kt[2] + 1, :kt[1], :kt[0]].copy()
    rest = rho.copy()
    rest[1:kt[2] + 1, :kt[1], :kt[0]] = 0
    assert np.all(rest == 0)
    _check_fractions(np.concatenate([np.zeros(kt[0] * kt[1]), sub.ravel(), np.zeros(kt[0] * kt[1])]), kt, k)


@pytest.mark.parametrize("start", [0, 5])
def test_pudistr3d1_known_answers_fused_push(hip, start):
    """The same fractions through the fused push kernel (k_push, the
    headline kernel: kick off, zero velocities, so the move keeps every
    particle where it is and the push deposits all four), on the reference's
    grid embedded in an 8^3 slab."""
    import torch
    k = GOLD["puDistr3D1"]
    T = (8, 8, 8)
    pos = np.array(k["pos"], dtype=np.float64) + 1.0
    pop, xs, vs = _device_pop(pos, np.zeros_like(pos), start)
    cap = pop.iStart[1]
    xo = [torch.zeros(cap, dtype=torch.float64, device="cuda") for _ in range(3)]
    vo = [torch.zeros(cap, dtype=torch.float64, device="cuda") for _ in range(3)]
    rho = torch.zeros((T[2] + 2) * T[1] * T[0], dtype=torch.float64, device="cuda")
    flags = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int32, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    thr = (C.c_double * 9)(1, 1, 1, T[0] + 1, T[1] + 1, T[2] + 1, T[0] + 1, T[1] + 1, T[2] + 1)
    a = PushArgs()
    a.xout = (C.c_void_p * 3)(*[t.data_ptr() for t in xo])
    a.vout = (C.c_void_p * 3)(*[t.data_ptr() for t in vo])
    a.kick = 0
    a.rhoS = rho.data_ptr()
    a.thr = C.cast(thr, C.c_void_p)
    a.flags = flags.data_ptr()
    a.chunkCount = cnt.data_ptr()
    a.maxVel = 1e30
    a.errFlag = err.data_ptr()
    a.tileWidth = 1
    hip.pinc_hip_push.argtypes = [Pop, C.c_int, Geom, C.POINTER(PushArgs), C.POINTER(C.c_int), C.c_void_p]
    nb = C.c_int()
    assert hip.pinc_hip_push(pop, 0, _geom(T), C.byref(a), C.byref(nb), None) == 0
    torch.cuda.synchronize()
    assert int(err[0]) == 0 and int(cnt.sum()) == 0
    n = len(pos)
    assert np.all(flags.cpu().numpy()[start:start + n] == 13)
    moved = np.stack([t.cpu().numpy()[start:start + n] for t in xo], 1)
    assert np.array_equal(moved, pos)
    _embedded_fractions(rho.cpu().numpy(), T, k)


def test_pudistr3d1_known_answers_tiled_cells(hip):
    """The same fractions through the tiled layout's cell-range deposit:
    pinc_hip_sort_tiles orders the four particles by tile and cell, then
    pinc_hip_deposit_cells sums each cell's particles (8^3 slab)."""
    import torch
    k = GOLD["puDistr3D1"]
    T = (8, 8, 8)
    pos = np.array(k["pos"], dtype=np.float64) + 1.0
    n = len(pos)
    pop, xs, vs = _device_pop(pos, np.zeros_like(pos))         # (keep the tensors alive)
    out, oxs, ovs = _device_pop(np.zeros_like(pos), np.zeros_like(pos))
    g = _geom(T)
    hip.pinc_hip_sort_tiles.argtypes = [Pop, Pop, C.c_int, Geom, C.c_int, C.c_void_p, C.c_long,
                                        C.POINTER(C.c_long), C.c_void_p]
    hip.pinc_hip_deposit_cells.argtypes = [Pop, C.c_int, Geom, C.c_int, C.c_void_p, C.c_long, C.c_void_p,
                                           C.c_void_p]
    nk = C.c_long()
    assert hip.pinc_hip_sort_tiles(pop, out, 0, g, 4, None, 0, C.byref(nk), None) != 0
    need = 2 * (nk.value + 1) + 2 * (nk.value // 4096 + 1) + 1
    work = torch.zeros(need, dtype=torch.int32, device="cuda")
    assert hip.pinc_hip_sort_tiles(pop, out, 0, g, 4, work.data_ptr(), need, C.byref(nk), None) == 0
    rho = torch.zeros((T[2] + 2) * T[1] * T[0], dtype=torch.float64, device="cuda")
    ends = work.data_ptr() + 4 * (nk.value + 1)
    assert hip.pinc_hip_deposit_cells(out, 0, g, 4, ends, n, rho.data_ptr(), None) == 0
    torch.cuda.synchronize()
    _embedded_fractions(rho.cpu().numpy(), T, k)


class ExtractWs(C.Structure):
    """pinc_extract_ws_t (include/pinc_hip.h)."""
    _fields_ = [("chunkOffset", C.c_void_p), ("scanWork", C.c_void_p), ("tail", C.c_void_p), ("holes", C.c_void_p),
                ("order", C.c_void_p), ("blockHist", C.c_void_p), ("scratch", C.c_void_p), ("buf", C.c_void_p),
                ("bufNe", C.c_void_p), ("cap", C.c_long)]


@pytest.mark.parametrize("nd_method", ["puExtractEmigrants3D", "puExtractEmigrantsND"])
def test_extract_emigrants_back_fill_order(hip, nd_method):
    """testExtractEmigrantsXD (pusher.test.c:360-545) through the HIP
    classification (k_move_classify, doMove = 0, no wrap: the reference
    layout) and the parallel back-fill extraction (k_extract_a/b, k_rank_*,
    k_fill_holes) of libpinc_hip.so: the 81 emigrant counts, every
    emigrants[ne] buffer in the reference's order (species after species,
    extraction order inside), iStop = {17, 117, 200} and the 17 survivors of
    each species in the serial back-fill's slot order, exactly.  (Both
    reference methods classify a 3-D particle alike; the device has one
    classification for any nDims, run here under each method's name.)
    The oracle's restatement passes the same checks on the CPU
    (tests/test_oracle_kat.py)."""
    import torch
    import extract_kat as X
    hip.pinc_hip_extract.argtypes = [Pop, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, ExtractWs,
                                     C.POINTER(C.c_long), C.POINTER(C.c_long), C.c_void_p]
    start = X.K["iStart"]
    total = start[-1] + 100
    p, v = X.inputs()
    xs = [torch.zeros(total, dtype=torch.float64, device="cuda") for _ in range(3)]
    vs = [torch.zeros(total, dtype=torch.float64, device="cuda") for _ in range(3)]
    stop = list(start)
    for s in X.K["species_with_particles"]:
        for d in range(3):
            xs[d][start[s]:start[s] + len(p)] = torch.from_numpy(p[:, d].copy())
            vs[d][start[s]:start[s] + len(p)] = torch.from_numpy(v[:, d].copy())
        stop[s] = start[s] + len(p)
    pop = Pop((C.c_void_p * 3)(*[t.data_ptr() for t in xs]), (C.c_void_p * 3)(*[t.data_ptr() for t in vs]), 3, 3,
              (C.c_long * 9)(*(start + [total])), (C.c_long * 8)(*stop))
    t = X.K["expect_thresholds"]
    hi = 8 + 1.0                                                    # local frame: true nodes 1..8
    thr = (C.c_double * 9)(*t[:3], *t[3:], hi, hi, hi)
    flags = torch.zeros(total, dtype=torch.uint8, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    cap = 64
    records = {}
    counts = np.zeros((27, 3), dtype=np.int64)
    keep = []
    for s in range(3):
        cnt = torch.zeros(4, dtype=torch.int32, device="cuda")
        i32 = lambda n: torch.zeros(n, dtype=torch.int32, device="cuda")
        ws_t = [i32(8), i32(8), i32(cap + 1), i32(cap + 1), i32(cap), i32(28 * 4 + 28), i32(128),
                torch.zeros(6 * cap, dtype=torch.float64, device="cuda"), torch.zeros(cap, dtype=torch.uint8,
                                                                                     device="cuda")]
        keep += ws_t
        ws = ExtractWs(*[a.data_ptr() for a in ws_t], cap)
        assert hip.pinc_hip_move_classify(pop, s, 0, thr, flags.data_ptr(), cnt.data_ptr(), 1e30, err.data_ptr(),
                                          0, None) == 0
        ne_emig = C.c_long()
        ne_count = (C.c_long * 28)()
        assert hip.pinc_hip_extract(pop, s, flags.data_ptr(), cnt.data_ptr(), 13, 27, ws, C.byref(ne_emig),
                                    ne_count, None) == 0
        torch.cuda.synchronize()
        pop.iStop[s] -= ne_emig.value
        buf = ws_t[7].cpu().numpy().reshape(6, cap)
        base = 0
        for ne in range(28):
            n = ne_count[ne]
            if ne < 27:
                counts[ne, s] = n
            if n:
                records.setdefault(ne, []).append(buf[:, base:base + n].T.copy())
            base += n
    assert int(err[0]) == 0
    assert list(pop.iStop)[:3] == X.K["expect_iStop"]

    def recs(ne):
        r = records.get(ne, [])
        return np.concatenate(r) if r else np.zeros((0, 6))

    def survivors(s):
        a, b = start[s], pop.iStop[s]
        return (np.stack([x.cpu().numpy()[a:b] for x in xs], 1), np.stack([x.cpu().numpy()[a:b] for x in vs], 1))

    X.check(counts, recs, survivors)
