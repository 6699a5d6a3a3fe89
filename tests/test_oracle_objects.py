"""The immersed-object restatement (oracle/orc_obj.c, object.c; SURVEY.md
8(f) item 1, config C5) checked by its invariants.

The reference's object.c does not compile and no test in
the reference covers it, so this is parity against the algorithm, not
against reference outputs ("parity unpinned" for C5).  Checked here:
  - lookup tables: interior = true nodes of the mask; surface = true nodes
    with 1..7 of their 8 cell-corner nodes (offsets {0,-1}^3) in the
    object, restated independently with numpy;
  - capacitance correction: after oApplyCapacitanceMatrix and the second
    solve the surface is an equipotential at phi_c, and the correction
    charge sums to zero;
  - collection: no particle is left with its cell's lower node inside,
    removed charge equals the charge counted, spread evenly over the
    surface nodes of rhoObj.
"""
import numpy as np
import pytest

import orc
from pinc_amd import configs


def _sphere(T, c, r):
    z, y, x = np.meshgrid(*[np.arange(t, dtype=float) for t in (T[2], T[1], T[0])], indexing="ij")
    return (((x - c[0]) ** 2 + (y - c[1]) ** 2 + (z - c[2]) ** 2) <= r * r).astype(float)


def _world(T=(16, 16, 16), levels=3):
    cfg = configs.config("cold3d", true_size=T, nsub=(1, 1, 1))
    cfg["multigrid"]["mgLevels"] = str(levels)
    return orc.World(configs.write_ini(cfg))


def _node(T, x, y, z):
    # padded (ghost 1) node index, x fastest
    return (x + 1) + (T[0] + 2) * ((y + 1) + (T[1] + 2) * (z + 1))


def test_lookup_tables():
    T = (16, 16, 16)
    w = _world(T)
    w.init()
    mask = _sphere(T, (7.3, 8.1, 7.7), 4.2)
    ob = orc.Objects(w, mask)
    assert ob.n == 1
    z, y, x = np.nonzero(mask)
    assert np.array_equal(np.sort(ob.interior()), np.sort(_node(T, x, y, z)))
    # surface: count the object's nodes among (x-a, y-b, z-c), a,b,c in {0,1}
    cnt = np.zeros_like(mask)
    for a in (0, 1):
        for b in (0, 1):
            for c in (0, 1):
                cnt += np.roll(mask, (c, b, a), axis=(0, 1, 2))
    zs, ys, xs = np.nonzero((cnt > 0) & (cnt < 8))
    assert np.array_equal(np.sort(ob.surface()), np.sort(_node(T, xs, ys, zs)))
    assert len(ob.surface()) > 50


def test_capacitance_equipotential():
    T = (16, 16, 16)
    w = _world(T)
    w.init()
    w.init_fields()
    mask = _sphere(T, (8.0, 8.0, 8.0), 2.5)
    ob = orc.Objects(w, mask)
    ob.capacitance()
    sf = ob.surface()
    rng = np.random.default_rng(3)
    rho = w.grid(0)
    rho[1:-1, 1:-1, 1:-1, 0] = rng.standard_normal((16, 16, 16))
    w.set_grid(0, rho)
    w.op("solve")
    phi0 = w.grid(1).ravel()[sf].copy()
    before = w.grid(0).ravel().copy()
    pc = ob.apply()[0]
    corr = w.grid(0).ravel() - before
    assert abs(corr.sum()) <= 1e-9 * np.abs(corr).max()
    assert np.count_nonzero(corr) <= len(sf)
    w.op("solve")
    phi = w.grid(1).ravel()[sf]
    spread = np.abs(phi - pc).max()
    assert spread <= 1e-6 * np.abs(w.grid(1)).max(), (spread, pc)
    # before the correction the surface was far from an equipotential
    assert np.ptp(phi0) > 1e4 * spread


def test_collect_removes_inside_particles():
    T = (16, 16, 16)
    w = _world(T)
    w.init()
    mask = _sphere(T, (8.0, 8.0, 8.0), 3.0)
    ob = orc.Objects(w, mask)
    inside = set(ob.interior().tolist())
    q = w.species()[0]
    n0, charge_in = [], 0.0
    for s in range(2):
        pos, _, _ = w.particles(s)
        j = pos.astype(np.int64)
        nodes = j[:, 0] + (T[0] + 2) * (j[:, 1] + (T[1] + 2) * j[:, 2])
        k = np.isin(nodes, list(inside))
        n0.append((len(pos), int(k.sum())))
        charge_in += q[s] * k.sum()
    assert n0[0][1] > 0
    ob.collect()
    for s in range(2):
        pos, _, _ = w.particles(s)
        j = pos.astype(np.int64)
        nodes = j[:, 0] + (T[0] + 2) * (j[:, 1] + (T[1] + 2) * j[:, 2])
        assert not np.isin(nodes, list(inside)).any()
        assert len(pos) == n0[s][0] - n0[s][1]
    assert ob.collected(0) == pytest.approx(charge_in, rel=1e-12, abs=1e-12)
    ro = ob.rho_obj().ravel()
    sf = ob.surface()
    assert ro.sum() == pytest.approx(charge_in, rel=1e-9, abs=1e-9)
    assert np.allclose(ro[sf], charge_in / len(sf))


def test_object_steps_run():
    T = (16, 16, 16)
    w = _world(T)
    w.init()
    mask = _sphere(T, (8.0, 8.0, 8.0), 2.5)
    ob = orc.Objects(w, mask)
    ob.init_collect()
    w.init_fields()
    ob.capacitance()
    ob.step(3)
    ke, pe = w.energy()
    assert np.isfinite(ke) and np.isfinite(pe)


@pytest.mark.parametrize("reference", [False, True])
def test_collected_charge_divisor(reference):
    """object.c:476-478 spreads object a's collected charge with
    1/lookupSurfaceOffset[a+1], the cumulative surface count of objects
    0..a: object 0 keeps its charge, every later object loses the fraction
    its predecessors' surfaces take.  The build (pinc_obj.c) and this
    checker divide by the object's own surface count (a named correction,
    DESIGN.md section 11): rhoObj over each object's surface sums to the
    charge it collected."""
    T = (24, 16, 16)
    w = _world(T)
    w.init()
    mask = _sphere(T, (6.0, 8.0, 8.0), 3.0) + 2 * _sphere(T, (17.0, 8.0, 8.0), 3.5)
    ob = orc.Objects(w, mask)
    assert ob.n == 2
    ob.reference_divisor(reference)
    ob.collect()
    ro = ob.rho_obj().ravel()
    n0, n1 = len(ob.surface(0)), len(ob.surface(1))
    s0, s1 = ro[ob.surface(0)].sum(), ro[ob.surface(1)].sum()
    c0, c1 = ob.collected(0), ob.collected(1)
    assert abs(c0) > 0 and abs(c1) > 0
    assert s0 == pytest.approx(c0, rel=1e-12)
    if reference:
        assert s1 == pytest.approx(c1 * n1 / (n0 + n1), rel=1e-12)
        assert abs(s1) < abs(c1)
    else:
        assert s1 == pytest.approx(c1, rel=1e-12)
