"""Multigrid parity at the configs' sizes.

One charge density (tests/mg_history.py: seeded normal noise per true node,
the same array on both sides, SHA-256 checked) goes through
  * the device's parity mode (the reference's mgVRecursive/mgSolveRaw,
    multigrid.c:1496-1556, 1688-1724) and the oracle's restatement of it
    (oracle/orc_mg.c), and
  * the device's native mode (correction scheme with the coarse h^2 factor,
    DESIGN.md section 6) and the oracle's restatement of THAT algorithm
    (oracle/orc_native.c),
and the RMS residual after every V-cycle is compared, together with the
cycle count and the final potential.  The oracle's side is committed
(tests/golden/mg_history/, made by tests/golden/make_mg_fixtures.py), so
the GPU box does not re-run the CPU solves.  The two sides differ only in the
summation order of the neutralisation means and of the norm, so the
histories agree to round-off until the residual itself approaches
round-off.
"""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent))
import mg_history  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _built(built):  # the checker's thread count is set there (conftest.py)
    return built


GOLDEN = Path(__file__).resolve().parent / "golden" / "mg_history"


def _fixture(name: str) -> dict:
    """The oracle's side, committed (tests/golden/make_mg_fixtures.py): the
    residual after every V-cycle and phi on every k-th node."""
    import json
    return json.loads((GOLDEN / f"{name}.json").read_text())


def _compare(g, o, rtol_hist, rtol_phi, tail_floor=1e-8):
    assert g["rho_sha256"] == o["rho_sha256"]
    hg, ho = np.array(g["residual"][-1]), np.array(o["residual"])
    assert abs(len(hg) - len(ho)) <= 1, (len(hg), len(ho))
    n = min(len(hg), len(ho))
    sel = ho[:n] > tail_floor   # above round-off of the norm
    rel = np.abs(hg[:n] - ho[:n]) / ho[:n]
    assert np.all(rel[sel] < rtol_hist), rel[sel].max()
    k = o["phi_stride"]
    pg = g["phi"][::k, ::k, ::k].ravel()
    assert np.max(np.abs(pg - np.array(o["phi_sub"]))) <= rtol_phi * o["phi_max"]
    assert abs(np.max(np.abs(g["phi"])) - o["phi_max"]) <= rtol_phi * o["phi_max"]


def test_parity_mode_matches_oracle_at_128():
    """C3's grid with the reference's own five levels: 121 cycles on both
    sides; residual history to 1e-6, phi to 1e-9 of its maximum."""
    o = _fixture("parity_128")
    g = mg_history.run("gpu", 128, 5, 3000, o["seed"], o["amp"])
    assert g["residual"][-1][-1] <= 1e-10 and o["residual"][-1] <= 1e-10
    _compare(g, o, 1e-6, 1e-9)


def test_parity_mode_matches_oracle_at_256_first_cycles():
    """C4's grid with five levels: the reference algorithm does not converge
    there (the residual falls to 5e-6 at cycle 210 and
    then grows).  The device follows the oracle cycle by cycle: the first 40
    cycles and phi after them to 1e-8 / 1e-9."""
    o = _fixture("parity_256_40")
    g = mg_history.run("gpu", 256, 5, 40, o["seed"], o["amp"])
    assert len(g["residual"][0]) == len(o["residual"]) == 40
    _compare(g, o, 1e-8, 1e-9, tail_floor=0.0)


def test_parity_mode_follows_oracle_through_the_256_minimum():
    """The same solve for 300 cycles, through the minimum at cycle 210 and
    into the growth, against the oracle's 3000-cycle history: the two
    agree to 1e-6 relative on every cycle (the divergence is the
    algorithm's, not the device's)."""
    o = _fixture("parity_256_3000")
    g = mg_history.run("gpu", 256, 5, 300, o["seed"], o["amp"])
    assert g["rho_sha256"] == o["rho_sha256"]
    hg, ho = np.array(g["residual"][0]), np.array(o["residual"][:300])
    assert len(hg) == 300
    assert np.argmin(hg) == np.argmin(ho)
    assert np.max(np.abs(hg - ho) / ho) < 1e-6


@pytest.mark.parametrize("size", [128, 256])
def test_native_mode_matches_native_oracle(size):
    """Native mode against its CPU restatement: same cycle count (+-1),
    residual history to 1e-6 above 1e-8, phi to 1e-9 of its maximum."""
    o = _fixture(f"native_{size}")
    g = mg_history.run("gpu", size, 5, 200, o["seed"], o["amp"], native=True)
    assert g["residual"][-1][-1] <= 1e-10 and o["residual"][-1] <= 1e-10
    assert len(g["residual"][-1]) <= 12
    _compare(g, o, 1e-6, 1e-9)


def test_native_and_parity_modes_reach_the_same_potential():
    """Both algorithms solve the same discrete problem: at 128^3 their
    converged potentials agree to 1e-7 of the maximum (both stop at an RMS
    residual of 1e-10, which bounds the error through the Laplacian's
    smallest eigenvalue on this grid)."""
    a = mg_history.run("gpu", 128, 5, 3000, 20261016, 1.0)
    b = mg_history.run("gpu", 128, 5, 200, 20261016, 1.0, native=True)
    assert np.max(np.abs(a["phi"] - b["phi"])) <= 1e-7 * np.max(np.abs(a["phi"]))


@pytest.mark.parametrize("name,native", [("c2", True), ("c2", False), ("langmuir1d", True)])
def test_nd_solve_matches_oracle(name, native):
    """1-D and 2-D multigrid (mgGSND / halfWeightND / bilinearND; C2's
    128^2 grid), native mode -- whose coarse levels run in the
    single-workgroup kernel -- and parity mode, against the oracle on the
    same rho: same cycle count (+-1), phi to 1e-9 of its maximum."""
    import orc
    from pinc_amd import Sim, configs
    cfg = configs.config(name)
    if native:
        cfg["multigrid"]["native"] = "1"
    ini = configs.write_ini(cfg)
    try:
        w = orc.World(ini)
        shape = w.grid(0).shape
        rho = np.zeros(shape)
        inner = tuple(slice(1, -1) for _ in shape[:-1]) + (0,)
        rho[inner] = np.random.default_rng(7).standard_normal(rho[inner].shape)
        w.mg_limit(4000, 4000)
        w.set_grid(0, rho)
        w.op("solve")
        ho = w.mg_history()
        po = w.grid(1)[inner].copy()
        w.close()
        with Sim(ini, perturb=False) as s:
            s.mg_limit(4000, 4000)
            s.set_grid(0, rho)
            s.op("solve")
            hg = s.mg_history()
            pg = s.grid(1)[inner].copy()
    finally:
        os.unlink(ini)
    assert ho[-1] <= 1e-10 and hg[-1] <= 1e-10
    assert abs(len(ho) - len(hg)) <= 1, (len(ho), len(hg))
    if native:
        assert len(hg) <= 12
    assert np.max(np.abs(pg - po)) <= 1e-9 * np.max(np.abs(po))


@pytest.mark.parametrize("layout,coarse", [("reference", 0), ("tiled", 0), ("reference", 1), ("tiled", 1)])
def test_extrapolated_guess_matches_oracle(layout, coarse):
    """multigrid:extrapolate (native mode, an extension: each solve starts
    from 2 phi_n - phi_(n-1) instead of phi_n, pinc_hip_extrapolate) on a
    warm 32^3 plasma: the device follows the oracle's restatement
    (oracle/orc_native.c) step by step -- energies to 1e-8, the V-cycle
    count per solve +-1 -- and needs no more cycles in total than the plain
    warm start of the same run.  coarse = 1: multigrid:spectralCoarse, the
    level-1 correction solved exactly (rocFFT with the 7-point symbol; the
    oracle's orc_discrete_poisson) -- a two-grid cycle."""
    import orc
    from pinc_amd import Sim, configs
    cfg = configs.config("warm", true_size=(32, 32, 32), ppc=8, nalloc_pc=16, levels=3)
    cfg["multigrid"]["native"] = "1"
    cfg["multigrid"]["spectralCoarse"] = str(coarse)
    ini_plain = configs.write_ini(cfg)
    cfg["multigrid"]["extrapolate"] = "1"
    ini_o = configs.write_ini(cfg)
    if layout == "tiled":
        cfg["population"]["layout"] = "tiled"
        cfg["population"]["sortInterval"] = "2"
    ini_g = configs.write_ini(cfg)
    steps = 8
    try:
        # the plain warm start first (one simulation per process at a time)
        with Sim(ini_plain, maxwell=True, perturb=False, seed=5) as p:
            p.init()
            cp0 = p.cycles
            p.step(steps)
            plain = p.cycles - cp0
        w = orc.World(ini_o)
        w.init(perturb=False, maxwell=True, seed=5)
        w.init_fields()
        with Sim(ini_g, maxwell=True, perturb=False, seed=5) as s:
            s.init()
            c0, co0 = s.cycles, w.cycles
            for n in range(steps):
                cs, co = s.cycles, w.cycles
                s.step()
                w.step()
                assert abs((s.cycles - cs) - (w.cycles - co)) <= 1, (n, s.cycles - cs, w.cycles - co)
                ke, pe, _ = s.energy()
                ke_o, pe_o = w.energy()
                assert abs(ke - ke_o) <= 1e-8 * abs(ke_o), (n, ke, ke_o)
                assert abs(pe - pe_o) <= 1e-8 * abs(pe_o), (n, pe, pe_o)
            assert s.cycles - c0 <= plain, (s.cycles - c0, plain)
            assert abs((s.cycles - c0) - (w.cycles - co0)) <= steps // 4 + 1
        w.close()
    finally:
        for f in (ini_plain, ini_o, ini_g):
            os.unlink(f)


def test_speculative_first_sweep_is_bit_identical():
    """multigrid:speculate (default on): while the host reads a cycle's
    norm, the next cycle's first double sweep (phi -> res) already runs when
    the last solve of the same role needed more cycles.  A sequence of solves
    whose cycle counts go up and down (so some sweeps ahead are used and some
    dropped) gives bit-identical potentials and residual histories to the
    synchronous loop."""
    from pinc_amd import configs
    from pinc_amd.sim import Sim
    rhos = [mg_history.make_rho(128, seed, amp) for seed, amp in
            [(1, 1.0), (1, 1.0), (2, 1.0), (3, 1e-3), (4, 10.0), (4, 10.0), (5, 1.0)]]
    out = {}
    for spec in ("0", "1"):
        cfg = configs.config("warm", true_size=(128, 128, 128), ppc=1, nalloc_pc=2, levels=5)
        cfg["multigrid"].update({"native": "1", "extrapolate": "1", "spectralCoarse": "1", "speculate": spec})
        ini = configs.write_ini(cfg)
        try:
            with Sim(ini, perturb=False) as s:
                s.mg_limit(0, 100)
                hist, phis = [], []
                for r in rhos:
                    s.set_grid(0, r)
                    s.op("solve")
                    hist.append(s.mg_history().tolist())
                    phis.append(s.grid(1)[1:-1, 1:-1, 1:-1].copy())
        finally:
            os.unlink(ini)
        out[spec] = (hist, phis)
    counts = [len(h) for h in out["1"][0]]
    assert len(set(counts)) > 1, counts           # the counts vary
    assert out["0"][0] == out["1"][0]
    for a, b in zip(out["0"][1], out["1"][1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("coarse", [0, 1])
def test_one_cu_solve_matches_multi_launch_and_oracle(coarse):
    """multigrid:oneCU (native mode, one rank, C2's 2-D 128^2): every cycle
    of a solve and its convergence test in one workgroup
    (pinc_hip_mg_solve_small), against the per-level launches of the same
    cycle and the oracle's native solve on the same rho.

    coarse = 0: the V-cycle (k_gs_pass, k_residual, k_restrict,
    k_mg_coarse, k_prolong_add in the per-level form): the same operators in
    the same expression order, so for the same cycle count phi is
    bit-identical (only the norm's summation order differs: histories to
    1e-12).  coarse = 1: multigrid:spectralCoarse, the two-grid cycle whose
    level-1 correction the workgroup solves exactly through the real Fourier
    basis on the f64 matrix cores, against rocFFT on the per-level path: the
    same discrete problem in another rounding (cycle counts +-1, phi to 1e-9
    of its maximum, as against the oracle).  A sequence of warm-started
    solves whose counts differ, a cycle cap (mgSetLimit) and a history longer
    than one launch's 60 entries."""
    import orc
    from pinc_amd import Sim, configs
    cfg = configs.config("c2")
    cfg["multigrid"]["native"] = "1"
    cfg["multigrid"]["spectralCoarse"] = str(coarse)
    gen = np.random.default_rng(11)
    out = {}
    for one in ("0", "1", "oracle"):
        cfg["multigrid"]["oneCU"] = "0" if one == "oracle" else one
        ini = configs.write_ini(cfg)
        try:
            if one == "oracle":
                s = orc.World(ini)
            else:
                s = Sim(ini, perturb=False)
            shape = s.grid(0).shape
            inner = tuple(slice(1, -1) for _ in shape[:-1]) + (0,)
            if not out:
                base = np.zeros(shape)
                base[inner] = gen.standard_normal(base[inner].shape)
                rhos = [base * a for a in (1.0, 1.0, 1e-3, 10.0)] + [base[::-1].copy()]
            hist, phis = [], []
            s.mg_limit(0, 100)
            for r in rhos:
                s.set_grid(0, r)
                s.op("solve")
                hist.append(s.mg_history().tolist())
                phis.append(s.grid(1)[inner].copy())
            s.mg_limit(3, 100)
            s.set_grid(0, rhos[3] * 7.0)
            s.op("solve")
            hist.append(s.mg_history().tolist())
            phis.append(s.grid(1)[inner].copy())
            s.close()
        finally:
            os.unlink(ini)
        out[one] = (hist, phis)
    (h0, p0), (h1, p1), (ho, po) = out["0"], out["1"], out["oracle"]
    counts = [len(h) for h in h1]
    assert len(set(counts[:-1])) > 1, counts
    assert counts[-1] == 3
    for k, (a, b, pa, pb) in enumerate(zip(h0, h1, p0, p1)):
        if coarse:
            assert abs(len(a) - len(b)) <= 1, (k, len(a), len(b))
            assert np.max(np.abs(pb - pa)) <= 1e-9 * np.max(np.abs(pa)), k
        else:
            assert len(a) == len(b), (k, len(a), len(b))
            assert np.allclose(a, b, rtol=1e-12, atol=0), k
            assert np.array_equal(pa, pb), k
    for k, (a, b, pa, pb) in enumerate(zip(ho, h1, po, p1)):
        assert abs(len(a) - len(b)) <= 1, (k, len(a), len(b))
        assert np.max(np.abs(pb - pa)) <= 1e-9 * np.max(np.abs(pa)), k
