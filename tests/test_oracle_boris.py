"""Oracle restatement of the Boris pusher extension (puBoris3D1KE,
pusher.c:394-505, with the reference's indexing defect corrected: SURVEY.md
fact 7; the reference never runs it, so parity is against the algorithm's
own invariants, not against reference outputs).

With both species on one lattice and no perturbation, rho, phi and E are
exactly zero, so the initial half step is a pure rotation about B by the
angle theta with tan(theta/2) = |T|/2 (T = q/m B / 2, halved for the half
step): speeds are kept to rounding, v parallel to B is untouched, every
particle of a species turns by the same angle, and the two species' angles
are in the ratio of their q/m.
"""
import numpy as np

import orc
from pinc_amd import configs


def _world(bext):
    cfg = configs.config("cold3d")
    cfg["methods"]["acc"] = "puBoris3D1KE"
    cfg["fields"]["BExt"] = bext
    w = orc.World(configs.write_ini(cfg))
    w.init(perturb=False, maxwell=True, seed=3)
    return w


def test_boris_half_step_is_a_rotation_about_b():
    w = _world("0,0,1e-4")
    v0 = [w.particles(s)[1].copy() for s in range(2)]
    w.init_fields()
    th = []
    for s in range(2):
        v1 = w.particles(s)[1]
        # rho cancels to rounding (E ~ 1e-19): v parallel to B is kept
        np.testing.assert_allclose(v1[:, 2], v0[s][:, 2], rtol=0, atol=1e-15 * np.abs(v0[s]).max())
        n0, n1 = np.linalg.norm(v0[s], axis=1), np.linalg.norm(v1, axis=1)
        assert np.max(np.abs(n1 / n0 - 1)) < 1e-14
        d = np.angle(np.exp(1j * (np.arctan2(v1[:, 1], v1[:, 0]) - np.arctan2(v0[s][:, 1], v0[s][:, 0]))))
        assert np.ptp(d) < 1e-12 * max(1.0, abs(d[0])) + 1e-15
        th.append(d[0])
    # tan(theta/2) is proportional to q/m: electrons (-1, 1) and ions (1, 1836)
    ratio = np.tan(th[0] / 2) / np.tan(th[1] / 2)
    assert abs(ratio / -1836.0 - 1) < 1e-9, ratio


def test_boris_oblique_field_keeps_speed_and_parallel_velocity():
    b = np.array([1e-4, -2e-4, 3e-4])
    w = _world(",".join(map(repr, b)))
    v0 = [w.particles(s)[1].copy() for s in range(2)]
    w.init_fields()
    bh = b / np.linalg.norm(b)
    for s in range(2):
        v1 = w.particles(s)[1]
        np.testing.assert_allclose(np.linalg.norm(v1, axis=1), np.linalg.norm(v0[s], axis=1), rtol=1e-14)
        np.testing.assert_allclose(v1 @ bh, v0[s] @ bh, rtol=0, atol=1e-15 * np.abs(v0[s]).max())


def test_boris_zero_field_is_the_leapfrog_kick():
    """BExt = 0: T = S = 0 and Boris reduces to two half kicks; particles and
    PE follow puAcc3D1KE to rounding over a few steps (KE is defined
    differently: |v+|^2 at the mid step for Boris, v(n-1/2).v(n+1/2) for
    the leapfrog)."""
    cfg = configs.config("cold3d")
    ini_a = configs.write_ini(cfg)
    cfg["methods"]["acc"] = "puBoris3D1KE"
    ini_b = configs.write_ini(cfg)
    out = []
    for ini in (ini_a, ini_b):
        w = orc.World(ini)
        w.init(perturb=True, maxwell=False, seed=1)
        w.init_fields()
        w.step(3)
        out.append((w.energy(), w.particles(0)[1].copy()))
    (ka, pa), va = out[0]
    (kb, pb), vb = out[1]
    assert abs(pa - pb) <= 1e-10 * abs(pa)
    assert abs(ka - kb) <= 0.05 * abs(ka)
    np.testing.assert_allclose(vb, va, rtol=0, atol=1e-14 * np.abs(va).max())
