"""The checker's spectral Poisson solve (oracle/orc_mg.c, restating
spectral.c:14-115 and its N-D extension) against known answers.

FFTW is absent here, so the reference's sSolve cannot run; the 1-D solver is
pinned by the analytic answer of the reference's own sMode driver
(spectral.c:150-175: rho = sin(2 pi j/N) gives phi = (N/2 pi)^2 rho), the
N-D extension by single Fourier modes, and the two implementations (exact
1-D r2c/c2r restatement, separable N-D DFT with rank gathering) against
each other.  Multi-rank emulation must not change the result.
"""
import numpy as np
import pytest

import orc
from pinc_amd import configs


def _world(cfg):
    ini = configs.write_ini(cfg)
    return orc.World(ini), ini


def _true(a, nd):
    """true nodes of a reference-layout scalar grid (ghost 1 per side)"""
    sl = tuple([slice(1, -1)] * nd) + (0,)
    return a[sl]


def _set_true(w, which, vals, rank=0):
    g = w.grid(which, rank)
    nd = g.ndim - 1
    g[tuple([slice(1, -1)] * nd) + (0,)] = vals
    w.set_grid(which, g, rank)


def test_smode_known_answer_1d():
    cfg = configs.config("langmuir1d")
    cfg["methods"]["poisson"] = "sSolver"
    w, _ = _world(cfg)
    N = 32
    j = np.arange(N)
    rho = np.sin(2 * np.pi * j / N)
    _set_true(w, 0, rho)
    w.op("solve")
    phi = _true(w.grid(1), 1)
    np.testing.assert_allclose(phi, (N / (2 * np.pi)) ** 2 * rho, rtol=0, atol=1e-12 * (N / (2 * np.pi)) ** 2)
    w.close()


@pytest.mark.parametrize("size,nsub", [((16, 8, 8), (1, 1, 1)), ((16, 8, 4), (1, 1, 2)), ((8, 8, 4), (1, 2, 2))])
def test_single_mode_3d(size, nsub):
    cfg = configs.config("cold3d", true_size=size, nsub=nsub)
    cfg["methods"]["poisson"] = "sSolver"
    w, _ = _world(cfg)
    L = [size[d] * nsub[d] for d in range(3)]
    m = (1, 2, 1)
    k2 = sum((2 * np.pi * m[d] / L[d]) ** 2 for d in range(3))
    for r in range(w.nranks):
        sub = [(r // int(np.prod(nsub[:d]))) % nsub[d] for d in range(3)]
        z, y, x = np.meshgrid(*[np.arange(size[d]) + sub[d] * size[d] for d in (2, 1, 0)], indexing="ij")
        rho = np.cos(2 * np.pi * (m[0] * x / L[0] + m[1] * y / L[1] + m[2] * z / L[2]))
        _set_true(w, 0, rho, r)
    w.op("solve")
    for r in range(w.nranks):
        sub = [(r // int(np.prod(nsub[:d]))) % nsub[d] for d in range(3)]
        z, y, x = np.meshgrid(*[np.arange(size[d]) + sub[d] * size[d] for d in (2, 1, 0)], indexing="ij")
        rho = np.cos(2 * np.pi * (m[0] * x / L[0] + m[1] * y / L[1] + m[2] * z / L[2]))
        np.testing.assert_allclose(_true(w.grid(1, r), 3), rho / k2, rtol=0, atol=1e-12 / k2)
    w.close()


def test_nd_path_matches_1d_restatement():
    """1-D with two emulated ranks takes the separable N-D path; it must
    agree with the exact r2c/c2r restatement of spectral.c on one rank."""
    rng = np.random.default_rng(3)
    N = 32
    rho = rng.standard_normal(N)
    out = []
    for nsub, ts in ((1, 32), (2, 16)):
        cfg = configs.config("langmuir1d")
        cfg["methods"]["poisson"] = "sSolver"
        cfg["grid"]["nSubdomains"] = str(nsub)
        cfg["grid"]["trueSize"] = str(ts)
        w, _ = _world(cfg)
        for r in range(nsub):
            _set_true(w, 0, rho[r * ts:(r + 1) * ts], r)
        w.op("solve")
        out.append(np.concatenate([_true(w.grid(1, r), 1) for r in range(nsub)]))
        w.close()
    np.testing.assert_allclose(out[1], out[0], rtol=0, atol=1e-12 * np.abs(out[0]).max())
    # and against numpy's FFT restatement of the same operator
    spec = np.fft.rfft(rho)
    n = np.arange(1, N // 2 + 1)
    spec[0] = 0
    spec[1:] *= (N / (2 * np.pi * n)) ** 2 / N * N
    np.testing.assert_allclose(out[0], np.fft.irfft(spec, N), rtol=0, atol=1e-12 * np.abs(out[0]).max())


def test_spectral_langmuir1d_frequency():
    """C1 with the spectral solver: the Langmuir oscillation stays within 1%
    of omega_pe (the reference's 1-D spectral path is what sSolver_set
    allows; SURVEY.md 8(d) estimator)."""
    from test_oracle_golden import ke_peak_omega
    cfg = configs.config("langmuir1d")
    cfg["methods"]["poisson"] = "sSolver"
    ini = configs.write_ini(cfg)
    ke, pe, _ = orc.run_steps(ini, [], 150)
    om = ke_peak_omega(ke, 0.2)
    assert abs(om - 1.0) < 0.01, om
