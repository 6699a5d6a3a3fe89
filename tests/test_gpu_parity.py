"""GPU parity tests: the MI355X path (libpinc) against the CPU oracle.

Tolerances (floating point, fp64):
  * particle positions after a move from identical state: bit-exact;
  * particle counts, emigrant counts and particle order: exact;
  * rho after deposit: 1e-13 relative to max|rho| (atomic summation order);
  * phi, E after a solve: 1e-9 relative to max|phi| (the MG converges to an
    RMS residual of 1e-10; rounding differs by summation order);
  * velocities after acceleration: 1e-9 relative to the velocity scale;
  * KE/PE of multi-step runs: 1e-8 relative.
"""
import numpy as np
import pytest

import orc
from pinc_amd import configs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sim_cls(built):
    from pinc_amd import Sim
    return Sim


def _ini(name, **kw):
    return configs.write_ini(configs.config(name, **kw))


def _rel(a, b):
    scale = max(np.max(np.abs(b)), 1e-300)
    return np.max(np.abs(a - b)) / scale


def test_init_state_identical(sim_cls):
    """Lattice + perturbation + first migration: same particles, same order,
    bit-exact positions (population.c:172-276, pusher.c:782-1035)."""
    ini = _ini("cold3d")
    w = orc.World(ini)
    w.init()
    with sim_cls(ini) as s:
        s.op("init_particles")
        for sp in range(2):
            assert s.count(sp) == w.count(sp)
            pg, vg = s.particles(sp)
            po, vo, _ = w.particles(sp)
            np.testing.assert_array_equal(pg, po)
            np.testing.assert_array_equal(vg, vo)


def test_step_operators(sim_cls):
    """Each operator of one step, from identical state."""
    ini = _ini("cold3d")
    w = orc.World(ini)
    w.init()
    w.init_fields()
    with sim_cls(ini) as s:
        s.init()
        # same state after the half step?
        for sp in range(2):
            pg, vg = s.particles(sp)
            po, vo, _ = w.particles(sp)
            np.testing.assert_array_equal(pg, po)
            assert _rel(vg, vo) < 1e-9
        # force identical state, then compare each operator
        for sp in range(2):
            po, vo, _ = w.particles(sp)
            s.set_particles(sp, po, vo)
        s.op("move")
        w.op("move")
        for sp in range(2):
            np.testing.assert_array_equal(s.particles(sp)[0], w.particles(sp)[0])
        s.op("extract")
        w.op("extract")
        np.testing.assert_array_equal(s.emigrants(), w.emigrants())
        s.op("migrate")
        w.op("migrate")
        for sp in range(2):
            assert s.count(sp) == w.count(sp)
            np.testing.assert_array_equal(s.particles(sp)[0], w.particles(sp)[0])
            np.testing.assert_array_equal(s.particles(sp)[1], w.particles(sp)[1])
        s.op("distr")
        w.op("distr")
        rg, ro = s.grid(0), w.grid(0)
        inner = (slice(1, -1),) * 3
        # electrons and ions nearly cancel: bound the error by the size of
        # one species' contribution (|q| x particles per node)
        q, _ = s.species()
        ppc = s.count(0) / ro[inner].size
        assert np.max(np.abs(rg[inner] - ro[inner])) < 1e-13 * abs(q[0]) * ppc * 8
        s.op("solve")
        w.op("solve")
        pg, po = s.grid(1), w.grid(1)
        assert _rel(pg[inner], po[inner]) < 1e-9
        s.op("efield")
        w.op("efield")
        eg, eo = s.grid(2), w.grid(2)
        assert _rel(eg, eo) < 1e-8
        # identical E for the accelerator check
        s.set_grid(2, eo)
        s.op("acc")
        w.op("acc")
        for sp in range(2):
            vg = s.particles(sp)[1]
            vo = w.particles(sp)[1]
            assert np.max(np.abs(vg - vo)) <= 1e-12 * max(np.max(np.abs(vo)), 1e-30)


@pytest.mark.parametrize("name,steps", [("cold3d", 3), ("langmuir2d", 3), ("langmuir1d", 3)])
def test_energy_history(sim_cls, name, steps):
    ini = _ini(name)
    ke_o, pe_o, cyc_o = orc.run_steps(ini, [], steps)
    with sim_cls(ini) as s:
        s.init()
        for n in range(steps):
            s.step()
            ke, pe, _ = s.energy()
            assert abs(ke - ke_o[n]) <= 1e-8 * abs(ke_o[n])
            assert abs(pe - pe_o[n]) <= 1e-8 * abs(pe_o[n])
        # V-cycle counts follow the reference's convergence loop
        assert abs(s.cycles - cyc_o[-1]) <= steps


def test_reference_known_values(sim_cls):
    """KE(1), PE(1) of langmuirCold.ini at 32x16x16 recorded from the
    reference: 0.97536794508303382, 32.140625756280251."""
    with sim_cls(_ini("cold3d")) as s:
        s.init()
        s.step()
        ke, pe, _ = s.energy()
    assert abs(ke - 0.97536794508303382) < 1e-9
    assert abs(pe - 32.140625756280251) < 1e-7


@pytest.mark.parametrize("name,kw", [("cold3d", {}), ("warm", {"true_size": (32, 32, 32), "ppc": 8,
                                                               "nalloc_pc": 16, "levels": 3})])
def test_native_mg_same_solution(sim_cls, name, kw):
    """multigrid:native=1 (correction scheme with the coarse h^2 factor; not
    the reference's algorithm) solves the same discrete problem: phi agrees
    with the oracle's reference-algorithm solution to within what the
    1e-10 RMS-residual stop allows, in a handful of V-cycles."""
    cfg = configs.config(name, **kw)
    maxwell = name == "warm"
    ini_p = configs.write_ini(cfg)
    cfg["multigrid"]["native"] = "1"
    ini_n = configs.write_ini(cfg)
    w = orc.World(ini_p)
    w.init(perturb=not maxwell, maxwell=maxwell, seed=7)
    w.init_fields()
    w.step()
    with sim_cls(ini_n, maxwell=maxwell, perturb=not maxwell, seed=7) as s:
        s.init()
        for sp in range(2):
            po, vo, _ = w.particles(sp)
            s.set_particles(sp, po, vo)
        c0 = s.cycles
        s.op("distr")
        s.op("solve")
        pg = s.grid(1)
        cyc_native = s.cycles - c0
    c0 = w.cycles
    w.op("distr")
    w.op("solve")
    po = w.grid(1)
    cyc_ref = w.cycles - c0
    inner = (slice(1, -1),) * 3
    err = _rel(pg[inner], po[inner])
    assert err < 1e-6, err
    assert cyc_native <= 12, (cyc_native, cyc_ref)


@pytest.mark.parametrize("case,coarse", [("3d", 0), ("3d", 1), ("c2", 1)])
def test_native_mg_graph_replay(sim_cls, case, coarse):
    """multigrid:graph=1 (the V-cycle captured once into a HIP graph and
    replayed) gives the solution and cycle count of direct launches over
    several steps (the graph is reused across solves).  coarse = 1: with the
    exact level-1 solve (multigrid:spectralCoarse), whose rocFFT execution
    and copies are captured into the graph too; "c2" is the
    bench's C2 line (2-D 128^2, spectral coarse solve on) with the graph
    and, as the bench runs it, with the whole solve in one workgroup
    (multigrid:oneCU: the level-1 correction on the f64 matrix cores).  The
    kernels are the same (the one-workgroup solve: the same operators); the
    deposit's atomics make rho differ by rounding between any two runs, so
    phi is compared to 1e-9 of its scale and the cycle count to 1 (2 over
    the three steps' solves for the one-workgroup solve, whose coarse
    correction rounds differently)."""
    if case == "c2":
        cfg = configs.bench_config("c2", 128)
        kw = dict(perturb=True)
        variants = [("0", "0"), ("1", "0"), ("0", "1")]
    else:
        cfg = configs.config("warm", true_size=(32, 32, 64), ppc=8, nalloc_pc=16, levels=4)
        cfg["multigrid"]["native"] = "1"
        cfg["multigrid"]["spectralCoarse"] = str(coarse)
        kw = dict(maxwell=True, perturb=False, seed=3)
        variants = [("0", "0"), ("1", "0")]
    out = {}
    for graph, one in variants:
        cfg["multigrid"]["graph"] = graph
        cfg["multigrid"]["oneCU"] = one
        with sim_cls(configs.write_ini(cfg), **kw) as s:
            s.init()
            for _ in range(3):
                s.step()
            out[graph, one] = (s.grid(1).copy(), s.cycles, s.energy()[:2])
    ref = out["0", "0"]
    scale = np.abs(ref[0]).max()
    for v in variants[1:]:
        np.testing.assert_allclose(out[v][0], ref[0], rtol=0, atol=1e-9 * scale)
        assert abs(ref[1] - out[v][1]) <= (2 if v[1] == "1" else 1), (v, ref[1], out[v][1])
        np.testing.assert_allclose(out[v][2], ref[2], rtol=1e-9)


@pytest.mark.parametrize("layout", ["sorted", "scattered", "mixed"])
def test_deposit_layouts(sim_cls, layout):
    """puDistr3D1 on particle orders that exercise both deposit paths: the
    LDS-tiled one (spatially coherent chunks) and the global-atomic one
    (chunks whose node box exceeds the LDS tile)."""
    ini = _ini("cold3d")
    w = orc.World(ini)
    w.init()
    rng = np.random.default_rng(11)
    with sim_cls(ini) as s:
        s.op("init_particles")
        for sp in range(2):
            po, vo, _ = w.particles(sp)
            n = len(po)
            lo, hi = 1.0, np.array([32.9, 16.9, 16.9])
            pos = lo + rng.random((n, 3)) * (hi - lo)
            if layout == "sorted":
                pos = pos[np.lexsort((pos[:, 0], pos[:, 1], pos[:, 2]))]
            elif layout == "mixed":
                pos[: n // 2] = pos[: n // 2][np.lexsort((pos[: n // 2, 0], pos[: n // 2, 1], pos[: n // 2, 2]))]
            s.set_particles(sp, pos, vo)
            w.set_particles(sp, pos, vo)
        s.op("distr")
        w.op("distr")
        rg, ro = s.grid(0), w.grid(0)
        inner = (slice(1, -1),) * 3
        q, _ = s.species()
        ppc = s.count(0) / ro[inner].size
        assert np.max(np.abs(rg[inner] - ro[inner])) < 1e-13 * abs(q[0]) * ppc * 8


def _sorted_rows(a):
    a = np.asarray(a)
    return a[np.lexsort(a.T[::-1])]


_WARM32 = {"true_size": (32, 32, 32), "ppc": 8, "nalloc_pc": 16, "levels": 3}


@pytest.mark.parametrize("name,kw,maxwell,sched", [("cold3d", {}, False, {"sortInterval": "2"}),
                                                   ("warm", _WARM32, True, {"sortInterval": "2"}),
                                                   ("warm", _WARM32, True, {"sortFraction": "0.03", "sortMax": "3"}),
                                                   ("langmuir2d", {}, False, {"sortInterval": "2"}),
                                                   ("langmuir2d", {}, False, {"sortFraction": "0.01"})])
def test_tiled_layout(sim_cls, name, kw, maxwell, sched):
    """population:layout=tiled (particles re-sorted by tile every
    sortInterval moves, or per species once sortFraction of them left their
    cell; not the reference's order) gives the same particles and energies as
    the reference layout: the set of positions after the first move is
    bit-identical, energies follow the oracle to 1e-8."""
    cfg = configs.config(name, **kw)
    ini_ref = configs.write_ini(cfg)
    cfg["population"]["layout"] = "tiled"
    cfg["population"].update(sched)
    ini_t = configs.write_ini(cfg)
    steps = 5
    w = orc.World(ini_ref)
    w.init(perturb=not maxwell, maxwell=maxwell, seed=5)
    w.init_fields()
    with sim_cls(ini_t, maxwell=maxwell, perturb=not maxwell, seed=5) as s:
        s.init()
        for sp in range(2):
            po, vo, _ = w.particles(sp)
            pg, vg = s.particles(sp)
            np.testing.assert_array_equal(_sorted_rows(pg), _sorted_rows(po))
            # identical state (the half-step velocities agree to ~1e-12 only)
            s.set_particles(sp, po, vo)
        s.op("move")
        w.op("move")
        w.op("extract")
        w.op("migrate")
        for sp in range(2):
            assert s.count(sp) == w.count(sp)
            np.testing.assert_array_equal(_sorted_rows(s.particles(sp)[0]), _sorted_rows(w.particles(sp)[0]))
        for op in ("extract", "migrate", "distr", "solve", "efield", "acc"):
            s.op(op)
        for op in ("distr", "solve", "efield", "acc"):
            w.op(op)
        for n in range(steps):
            s.step()
            w.step()
            ke, pe, _ = s.energy()
            ke_o, pe_o = w.energy()
            assert abs(ke - ke_o) <= 1e-8 * abs(ke_o), (n, ke, ke_o)
            assert abs(pe - pe_o) <= 1e-8 * abs(pe_o), (n, pe, pe_o)
            for sp in range(2):
                assert s.count(sp) == w.count(sp)


@pytest.mark.parametrize("then", ["read", "drop"])
def test_pending_sorting_push_survives_an_e_write(sim_cls, then):
    """a sorting puAcc leaves the move pending and re-derives the
    kicked velocities from its E on demand.  main.c rescales E right after
    the initial half-step puAcc (gMul(E, 2.0)); any such write of E first
    materialises the pending kick (pinc_grid_touch), so reading the
    population afterwards, or dropping the move, gives the velocities of the
    E the push kicked with -- bit-identical to a run without the write
    (tools/debug/pending_e.py compares both with the unfused operators)."""
    cfg = configs.config("warm", **_WARM32)
    cfg["population"].update({"layout": "tiled", "sortInterval": "1", "fused": "1"})
    ini = configs.write_ini(cfg)
    out = []
    for write in (False, True):
        with sim_cls(ini, maxwell=True, perturb=False, seed=11) as s:
            s.init()
            s.op("acc")
            if write:
                s.set_grid(2, s.grid(2) * 2.0)
            if then == "drop":
                s.op("extract")
            out.append([s.particles(sp) for sp in range(2)])
    # (as sets, by position then velocity: the sorting pushes of the two runs
    # order particles sharing a lattice site arbitrarily)
    for sp in range(2):
        (p0, v0), (p1, v1) = out[0][sp], out[1][sp]
        o0 = np.lexsort(np.vstack([v0.T[::-1], p0.T[::-1]]))
        o1 = np.lexsort(np.vstack([v1.T[::-1], p1.T[::-1]]))
        np.testing.assert_array_equal(p0[o0], p1[o1])
        np.testing.assert_array_equal(v0[o0], v1[o1])


def test_pending_sorting_push_read_and_dropped(sim_cls):
    """A fused puAcc whose push sorts (tiled layout, sortInterval 1) leaves
    the move pending with the kicked velocities in slot order.  Reading the
    particles then (pSyncToHost), and dropping the move (an extract without a
    move), must give the state of the unfused operators: positions unmoved
    and bit-identical, velocities kicked -- and bit-identical to those the
    push commits at the next move.  (The fused run's first sorting
    push is preceded by a sort of the lattice-ordered population, so the two
    runs hold the particles in different orders: compared as sets, sorted by
    position and velocity.)"""
    cfg = configs.config("warm", **_WARM32)
    cfg["population"]["layout"] = "tiled"
    cfg["population"]["sortInterval"] = "1"
    out = {}
    for fused in ("0", "1"):
        cfg["population"]["fused"] = fused
        ini = configs.write_ini(cfg)
        with sim_cls(ini, maxwell=True, perturb=False, seed=11) as s:
            s.init()
            s.op("acc")
            read = [s.particles(sp) for sp in range(2)]
            s.op("extract")
            out[fused] = {"read": read, "dropped": [s.particles(sp) for sp in range(2)], "em": s.emigrants()}
    for key in ("read", "dropped"):
        for sp in range(2):
            (p1, v1), (p0, v0) = out["1"][key][sp], out["0"][key][sp]
            # (by position, then velocity: particles may share a lattice site)
            o1 = np.lexsort(np.vstack([v1.T[::-1], p1.T[::-1]]))
            o0 = np.lexsort(np.vstack([v0.T[::-1], p0.T[::-1]]))
            np.testing.assert_array_equal(p1[o1], p0[o0])
            assert np.abs(v1[o1] - v0[o0]).max() <= 1e-12 * np.abs(v0).max(), (key, sp)
    np.testing.assert_array_equal(out["1"]["em"], out["0"]["em"])
    # the read while the sorted move is pending re-applies the kick
    # (pinc_pending_vel): bit-identical to the velocities the push committed
    cfg["population"]["fused"] = "1"
    with sim_cls(configs.write_ini(cfg), maxwell=True, perturb=False, seed=11) as s:
        s.init()
        s.op("acc")
        pending = [s.particles(sp)[1] for sp in range(2)]
        s.op("move")
        moved = [s.particles(sp)[1] for sp in range(2)]
    for sp in range(2):
        a, b = pending[sp], moved[sp]
        np.testing.assert_array_equal(a[np.lexsort(a.T[::-1])], b[np.lexsort(b.T[::-1])])


@pytest.mark.parametrize("name,kw,maxwell", [("cold3d", {}, False),
                                             ("warm", {"true_size": (32, 32, 32), "ppc": 8, "nalloc_pc": 16}, True),
                                             ("langmuir2d", {}, False), ("langmuir1d", {}, False)])
def test_fused_push_equals_separate_operators(sim_cls, name, kw, maxwell):
    """population:fused=1 (default: puAcc's kick, the next puMove's drift,
    the classification and the deposit of the particles that stay in one
    pass) against fused=0 (one kernel per reference operator), 3 steps.
    Each run's deposit sums in a different order (atomics), so the field and
    through it the particles differ by rounding only: same counts, same
    order, positions to 1e-13 of the grid size, velocities to 1e-10 of
    max|v|, rho to 1e-12 of one species' charge scale (|q| ppc 8, as
    test_deposit_layouts: the net charge cancels), energies to 1e-9."""
    cfg = configs.config(name, **kw)
    out = {}
    for fused in ("0", "1"):
        cfg["population"]["fused"] = fused
        ini = configs.write_ini(cfg)
        with sim_cls(ini, maxwell=maxwell, perturb=not maxwell, seed=7) as s:
            s.init()
            s.step(3)
            out[fused] = {"parts": [s.particles(sp) for sp in range(2)], "rho": s.grid(0), "e": s.energy()[:2]}
            q, _ = s.species()
            rho_scale = abs(q[0]) * s.count(0) / np.prod(out[fused]["rho"].shape[:-1]) * 8
    L = max(int(t) for t in cfg["grid"]["trueSize"].split(","))
    for sp in range(2):
        (p1, v1), (p0, v0) = out["1"]["parts"][sp], out["0"]["parts"][sp]
        assert p1.shape == p0.shape
        assert np.abs(p1 - p0).max() <= 1e-13 * L
        assert np.abs(v1 - v0).max() <= 1e-10 * max(np.abs(v0).max(), 1e-300)
    assert np.abs(out["1"]["rho"] - out["0"]["rho"]).max() <= 1e-12 * rho_scale
    for a, b in zip(out["1"]["e"], out["0"]["e"]):
        assert abs(a - b) <= 1e-9 * abs(b)


@pytest.mark.parametrize("name,fused", [("langmuir2d", "1"), ("langmuir2d", "0"), ("cold3d", "1")])
def test_literal_mainc_energy_history(sim_cls, name, fused):
    """The literal main.c loop (rho's ghosts folded twice, main.c:226,232,
    plus the extra solve): energies follow the checker's literal loop to
    1e-8 (the device wraps x/y at deposit, so the double fold is reproduced
    by weighting periodic ghost nodes 2^g; see literal_ghost_weights)."""
    cfg = configs.config(name)
    cfg["population"]["fused"] = fused
    ini = configs.write_ini(cfg)
    steps = 5
    ke_o, pe_o, _ = orc.run_steps(ini, [], steps, literal=True)
    with sim_cls(ini, literal=True) as s:
        s.init()
        for n in range(steps):
            s.step()
            ke, pe, _ = s.energy()
            assert abs(ke - ke_o[n]) <= 1e-8 * abs(ke_o[n]), (n, ke, ke_o[n])
            assert abs(pe - pe_o[n]) <= 1e-8 * abs(pe_o[n]), (n, pe, pe_o[n])


@pytest.mark.parametrize("sort_interval", ["8", "1000000"], ids=["sorting", "no_sort"])
def test_literal_loop_tiled_one_rank_crossing_z(sim_cls, sort_interval):
    """the literal loop (rho folded twice, main.c:226,232) on one
    rank in the tiled layout, where the slab dimension wraps in place, with a
    warm plasma whose particles cross the z boundary.  The fused push must
    leave slab-ghost deposits on their own planes (a periodic image would
    move weight between ghost plane 0 and true plane T, which the double
    fold counts differently).  rho after every step against the checker's
    literal loop to 1e-12 of one species' charge scale, energies to 1e-8."""
    cfg = configs.config("warm", true_size=(16, 16, 16), ppc=16, nalloc_pc=24, vth=0.15, levels=3)
    cfg["population"].update({"layout": "tiled", "sortInterval": sort_interval})
    ini = configs.write_ini(cfg)
    steps = 6
    w = orc.World(ini, [], True)
    w.init(False, True, 11)
    w.init_fields()
    with sim_cls(ini, literal=True, maxwell=True, perturb=False, seed=11) as s:
        s.init()
        q, _ = s.species()
        for n in range(steps):
            s.step()
            w.step()
            r, ro = s.grid(0), w.grid(0)
            scale = abs(q[0]) * 16 * 8
            assert np.abs(r[1:-1, 1:-1, 1:-1] - ro[1:-1, 1:-1, 1:-1]).max() <= 1e-12 * scale, n
            ke, pe, _ = s.energy()
            ke_o, pe_o = w.energy()
            assert abs(ke - ke_o) <= 1e-8 * abs(ke_o), (n, ke, ke_o)
            assert abs(pe - pe_o) <= 1e-8 * abs(pe_o), (n, pe, pe_o)
        # electrons sit in the half cells at both z ends (they wrap there)
        zs = s.particles(0)[0][:, 2]
        assert np.sum(zs < 1.5) > 0 and np.sum(zs > 16.5) > 0
    w.close()


@pytest.mark.parametrize("case", ["cold3d", "langmuir2d", "shard"])
def test_fused_negated_efield_equals_operators(sim_cls, case):
    """regular()'s step computes E with the negation of gMul(E, -1)
    (main.c:247) inside gFinDiff1st's pass (pinc_fin_diff_neg): E is bit
    for bit the one of gFinDiff1st, gHaloOp(E), gMul(E, -1) run as separate
    operators, on one rank's grid and on the sharded solver's extended slab
    (one rank, multigrid:shard = 1)."""
    if case == "shard":
        cfg = configs.config("warm", true_size=(32, 32, 32), ppc=2, nalloc_pc=4, levels=3)
        cfg["multigrid"].update({"native": "1", "shard": "1"})
        ini = configs.write_ini(cfg)
    else:
        ini = _ini(case)
    out = {}
    with sim_cls(ini) as s:
        s.init()
        s.op("distr")
        s.op("solve")
        for op in ("efield", "efield_fused", "efield"):  # same phi (the deposit's atomics differ between runs)
            s.op(op)
            out.setdefault(op, []).append(s.grid(2).copy())
    assert np.array_equal(out["efield"][0], out["efield_fused"][0])
    assert np.array_equal(out["efield"][1], out["efield_fused"][0])
    assert np.abs(out["efield"][0]).max() > 0
