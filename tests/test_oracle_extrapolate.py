"""The checker's restatement of multigrid:extrapolate (oracle/orc_native.c,
the device's pinc_mg.c guess_begin / guess_end), on the
CPU: the extrapolated initial guesses change how many V-cycles a solve
takes, not what it converges to.  Each case runs in a few seconds.
"""
import numpy as np
import pytest

import orc
from pinc_amd import configs


def _sphere(T, c, r):
    z, y, x = np.meshgrid(*[np.arange(t, dtype=float) for t in (T[2], T[1], T[0])], indexing="ij")
    return (((x - c[0]) ** 2 + (y - c[1]) ** 2 + (z - c[2]) ** 2) <= r * r).astype(float)


def _warm(extrapolate, objects=None, second="response"):
    cfg = configs.config("warm", true_size=(32, 32, 32), ppc=8, nalloc_pc=16, levels=3)
    cfg["multigrid"]["native"] = "1"
    cfg["multigrid"]["extrapolate"] = str(extrapolate)
    if objects:
        cfg["population"]["fused"] = "0"
        cfg["objects"] = {"sphere": ",".join(map(str, objects)), "secondGuess": second}
    return configs.write_ini(cfg)


def _cycles_per_step(w, step, steps):
    c = [w.cycles]
    for _ in range(steps):
        step()
        c.append(w.cycles)
    return list(np.diff(c))


def test_series_guess_same_run_fewer_cycles():
    """No objects: 2 phi_n - phi_(n-1) from the third solve on.  Same
    energies as the warm start to the solver tolerance, and no solve needs
    more V-cycles (at this size: 4 each with the warm start, 3 from the
    second step on)."""
    runs = {}
    for ex in (0, 1):
        w = orc.World(_warm(ex))
        w.init(perturb=False, maxwell=True, seed=5)
        w.init_fields()
        cyc = _cycles_per_step(w, w.step, 8)
        runs[ex] = (cyc, w.energy())
        w.close()
    (c0, e0), (c1, e1) = runs[0], runs[1]
    assert all(b <= a for a, b in zip(c0, c1)), (c0, c1)
    assert sum(c1) < sum(c0)
    for a, b in zip(e0, e1):
        assert abs(a - b) <= 1e-9 * abs(a)


def test_discrete_poisson_is_the_seven_point_inverse():
    """orc_discrete_poisson (the symbol of the device's
    pinc_hip_fft_set_symbol(plan, 1)): on a neutral random rho its result
    satisfies -(sum of the 6 neighbours - 6 phi) = rho to round-off, has
    zero mean, and equals numpy's FFT with the same symbol."""
    import ctypes as C
    L = (12, 10, 8)
    rho = np.random.default_rng(3).standard_normal(L[::-1])
    rho -= rho.mean()
    phi = np.zeros_like(rho)
    Lc = (C.c_int * 3)(*L)
    orc.LIB.orc_discrete_poisson(3, Lc, rho.ctypes.data, phi.ctypes.data)
    lap = sum(np.roll(phi, s, axis=a) for a in range(3) for s in (1, -1)) - 6 * phi
    assert np.max(np.abs(-lap - rho)) <= 1e-12 * np.max(np.abs(rho))
    assert abs(phi.mean()) <= 1e-14 * np.max(np.abs(phi))
    k = np.meshgrid(*[2 * np.pi * np.fft.fftfreq(n) for n in L[::-1]], indexing="ij")
    sym = sum(2 - 2 * np.cos(kk) for kk in k)
    sym[0, 0, 0] = 1.0
    f = np.fft.fftn(rho) / sym
    f[0, 0, 0] = 0.0
    assert np.max(np.abs(np.fft.ifftn(f).real - phi)) <= 1e-12 * np.max(np.abs(phi))


@pytest.mark.parametrize("second", ["response", "spectral"])
def test_object_guesses_same_run(second):
    """With an object (two solves per step: FIRST from the last two steps'
    first solutions, SECOND from this step's first plus the last correction
    response; the capacitance matrix's solves keep the warm start): the same
    particles and energies as the warm start to the solver tolerance, and
    never more V-cycles in total.  With secondGuess = spectral the second
    solve starts from the first solution plus the exact discrete response to
    this step's correction charge (orc_discrete_poisson)."""
    T, sp = (32, 32, 32), (16.3, 15.6, 17.1, 4.2)
    runs = {}
    for ex in (0, 1):
        w = orc.World(_warm(ex, sp, second))
        w.init(perturb=False, maxwell=True, seed=5)
        ob = orc.Objects(w, _sphere(T, sp[:3], sp[3]))
        ob.capacitance()
        ob.init_collect()
        w.init_fields()
        cyc = _cycles_per_step(w, ob.step, 6)
        runs[ex] = (cyc, w.energy(), [w.count(s) for s in range(2)], ob.collected(0))
        ob.close()
        w.close()
    (c0, e0, n0, q0), (c1, e1, n1, q1) = runs[0], runs[1]
    assert n0 == n1 and q0 == q1
    assert sum(c1) <= sum(c0), (c0, c1)
    if second == "spectral":
        # the second solve of every step after the first needs one cycle
        assert sum(c1[1:]) <= sum(c0[1:]) - (len(c0) - 1), (c0, c1)
    for a, b in zip(e0, e1):
        assert abs(a - b) <= 1e-7 * abs(a)


def test_spectral_coarse_same_run():
    """multigrid:spectralCoarse (the level-1 correction solved exactly by
    orc_discrete_poisson, a two-grid cycle): the same energies as the full
    V-cycle to the solver tolerance, with no more V-cycles per solve."""
    runs = {}
    for sc in ("0", "1"):
        cfg = configs.config("warm", true_size=(32, 32, 32), ppc=8, nalloc_pc=16, levels=3)
        cfg["multigrid"]["native"] = "1"
        cfg["multigrid"]["extrapolate"] = "1"
        cfg["multigrid"]["spectralCoarse"] = sc
        w = orc.World(configs.write_ini(cfg))
        w.init(perturb=False, maxwell=True, seed=5)
        w.init_fields()
        runs[sc] = (_cycles_per_step(w, w.step, 6), w.energy())
        w.close()
    (c0, e0), (c1, e1) = runs["0"], runs["1"]
    assert all(b <= a for a, b in zip(c0, c1)), (c0, c1)
    for a, b in zip(e0, e1):
        assert abs(a - b) <= 1e-9 * abs(a)
