"""The oracle against the reference's own unit-test known answers.

Each case restates an assertion of the reference's test suite
(test/pusher.test.c, test/grid.test.c) as data in
tests/golden/reference_outputs.json and checks the oracle's C restatement of
the same function against it.  CPU only.
"""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

import orc

GOLD = json.loads((Path(__file__).parent / "golden" / "reference_outputs.json").read_text())["kat"]


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _lib():
    return orc._load()


@pytest.mark.parametrize("use3d", [1, 0], ids=["puAcc3D1", "puAccND1"])
def test_puacc_interpolation(use3d):
    k = GOLD["puAcc3D1"]
    lib = _lib()
    ts = np.array(k["trueSize"], dtype=np.int32)
    E = np.arange(3 * int(np.prod(ts)), dtype=np.float64)
    pos = np.array(k["pos"], dtype=np.float64).ravel()
    vel = np.tile(np.array(k["vel0"], dtype=np.float64), len(k["pos"]))
    ke = np.zeros(1)
    lib.orc_kat_acc(3, _ptr(ts), 0, _ptr(E), len(k["pos"]), _ptr(pos), _ptr(vel), k["charge"], k["mass"], use3d,
                    _ptr(ke))
    assert np.all(np.abs(vel[:3] - np.array(k["expect_vel_p0"])) < k["tol"]), vel[:3]
    assert abs(vel[3] - k["expect_vel_p1_x"]) < k["tol"], vel[3]


@pytest.mark.parametrize("use3d", [1, 0], ids=["puDistr3D1", "puDistrND1"])
def test_pudistr_fractions(use3d):
    k = GOLD["puDistr3D1"]
    lib = _lib()
    ts = np.array(k["trueSize"], dtype=np.int32)
    rho = np.zeros(int(np.prod(ts)))
    pos = np.array(k["pos"], dtype=np.float64).ravel()
    lib.orc_kat_distr(3, _ptr(ts), 0, _ptr(rho), len(k["pos"]), _ptr(pos), 1.0, use3d)
    for idx, frac in k["expect"].items():
        assert abs(rho[int(idx)] - frac) < k["tol"], (idx, rho[int(idx)], frac)
    # all the charge is deposited (4 unit particles)
    assert abs(rho.sum() - 4.0) < 1e-13


def test_rank_neighbor_maps():
    k = GOLD["puRankNeighbor"]
    lib = _lib()
    ns = np.array(k["nSubdomains"], dtype=np.int32)
    sub = np.array(k["subdomain"], dtype=np.int32)
    for ne, rank in k["neighbor_to_rank"].items():
        assert lib.orc_kat_neighbor_to_rank(_ptr(ns), _ptr(sub), int(ne)) == rank
    for rank, ne in k["rank_to_neighbor"].items():
        assert lib.orc_kat_rank_to_neighbor(_ptr(ns), _ptr(sub), int(rank)) == ne
    for ne, rec in k["reciprocal_3d"].items():
        assert lib.orc_kat_reciprocal(int(ne), 3) == rec


def _neighborhood(thr, alloc):
    lib = _lib()
    text = ("[grid]\nnDims=3\ntrueSize=10,11,12\nnGhostLayers=0,0,0,0,0,0\nstepSize=1,1,1\n"
            "boundaries=PERIODIC,PERIODIC,PERIODIC,PERIODIC,PERIODIC,PERIODIC\nnSubdomains=1,1,1\n"
            f"thresholds={','.join(map(str, thr))}\nnEmigrantsAlloc={','.join(map(str, alloc))}\n")
    t = np.zeros(6)
    a = np.zeros(27, dtype=np.int64)
    lib.orc_kat_neighborhood(text.encode(), _ptr(t), _ptr(a))
    return t, a


def test_create_neighborhood():
    k = GOLD["gCreateNeighborhood"]
    t, a = _neighborhood(k["thresholds_ini"], k["alloc_full"])
    assert np.allclose(t, k["expect_thresholds"], atol=1e-15, rtol=0)
    assert a.tolist() == k["expect_alloc_full"]
    _, a = _neighborhood(k["thresholds_ini"], k["alloc_smart"])
    assert a.tolist() == k["expect_alloc_smart"]
    _, a = _neighborhood(k["thresholds_ini"], k["alloc_equal"])
    assert a.tolist() == k["expect_alloc_equal"]


def test_const_e_leapfrog():
    """testConstE: half-step kick then move/accelerate; positions follow
    x0 + (q/m)/2 n^2 exactly (all values are multiples of 1/4)."""
    k = GOLD["constE"]
    lib = _lib()
    ts = np.array([32, 32, 32], dtype=np.int32)
    E = np.zeros(3 * int(np.prod(ts)))
    E[0::3] = 1.0
    for qm in k["qm"]:
        q, m = (qm, 1.0) if abs(qm) >= 1 else (1.0, 1.0 / qm)
        x0 = 16.0
        pos = np.array([x0, 16.0, 16.0])
        vel = np.zeros(3)
        ke = np.zeros(1)
        Eh = E * 0.5
        lib.orc_kat_acc(3, _ptr(ts), 0, _ptr(Eh), 1, _ptr(pos), _ptr(vel), q, m, 1, _ptr(ke))
        for n in range(1, k["steps"] + 1):
            pos += vel
            lib.orc_kat_acc(3, _ptr(ts), 0, _ptr(E), 1, _ptr(pos), _ptr(vel), q, m, 1, _ptr(ke))
            assert abs(pos[0] - (x0 + 0.5 * (q / m) * n * n)) < k["tol"], (qm, n, pos[0])



@pytest.mark.parametrize("use3d", [1, 0], ids=["puExtractEmigrants3D", "puExtractEmigrantsND"])
def test_extract_emigrants_back_fill_order(use3d):
    """testExtractEmigrantsXD (pusher.test.c:360-545): the 81 emigrant
    counts, every emigrants[ne] buffer in order, iStop = {17, 117, 200} and
    the 17 survivors of each species in the serial back-fill's slot order
    (thresholds restated for the current upper rule, tests/extract_kat.py)."""
    import extract_kat as X
    lib = _lib()
    start = np.array(X.K["iStart"] + [300], dtype=np.int64)
    stop = start[:3].copy()
    pos = np.zeros((300, 3))
    vel = np.zeros((300, 3))
    p, v = X.inputs()
    for s in X.K["species_with_particles"]:
        pos[start[s]:start[s] + len(p)] = p
        vel[start[s]:start[s] + len(p)] = v
        stop[s] = start[s] + len(p)
    cap = 16
    counts = np.zeros(27 * 3, dtype=np.int64)
    bufs = np.zeros((27, cap, 6))
    thr = np.zeros(6)
    lib.orc_kat_extract(X.grid_ini_text().encode(), 3, _ptr(start), _ptr(stop), _ptr(pos), _ptr(vel), use3d,
                        _ptr(counts), _ptr(bufs), cap, _ptr(thr))
    np.testing.assert_array_equal(thr, X.K["expect_thresholds"])
    np.testing.assert_array_equal(stop, X.K["expect_iStop"])
    counts = counts.reshape(27, 3)
    X.check(counts, lambda ne: bufs[ne, :counts[ne].sum()],
            lambda s: (pos[start[s]:stop[s]], vel[start[s]:stop[s]]))
