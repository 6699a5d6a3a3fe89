"""The oracle's multigrid on the reference's own sine fixture (CPU).

mgModeErrorScaling (multigrid.c:1734-1790) and mgMode (:1856-1900) are the
reference's known-answer harness for the Poisson solve: rho from gFillSin,
phi and E compared with gFillSinSol / gFillSinESol (grid.c:1563-1688), the
order of the error read from successive grid doublings
(script/framework/mgErrorScaling.py:28-60).  tests/mg_sine.py restates the
fixture and the discrete closed form; the same checks run through the HIP
multigrid in tests/test_gpu_mg_sine.py.
"""
import math

import pytest

import mg_sine

SIZES = (16, 32, 64)


@pytest.fixture(scope="module")
def runs(built):
    out = {}
    for native in (False, True):
        for d in (1, 3):
            for norm in (0, 1):
                for n in SIZES:
                    r = mg_sine.solve("oracle", n, d, norm, native=native)
                    out[native, d, norm, n] = (r, mg_sine.errors(r, n, d, norm), mg_sine.exact_bound(r, n, norm))
    return out


@pytest.mark.parametrize("native", [False, True], ids=["parity", "native"])
@pytest.mark.parametrize("d", [1, 3], ids=["x_mgModeErrorScaling", "z_mgMode"])
@pytest.mark.parametrize("norm", [0, 1], ids=["phi_norm", "E_norm"])
def test_oracle_solves_the_discrete_sine_exactly(runs, native, d, norm):
    """phi and E equal the 7-point closed form A sin(kJ), A sin k cos(kJ)
    to what the stop rule guarantees (mg_sine.exact_bound); with norm = 1
    (unit-scale potential) that is below 1e-9 of the maximum."""
    for n in SIZES:
        r, e, bound = runs[native, d, norm, n]
        assert e["phi_exact"] <= bound, (n, e, bound)
        assert e["E_exact"] <= bound, (n, e, bound)
        if norm == 1:
            assert e["phi_exact"] <= 1e-9 and e["E_exact"] <= 1e-9, (n, e)


@pytest.mark.parametrize("native", [False, True], ids=["parity", "native"])
@pytest.mark.parametrize("d", [1, 3], ids=["x", "z"])
def test_oracle_error_falls_fourfold_per_doubling(runs, native, d):
    """mgErrorScaling.py's measurement: the RMS error against gFillSinSol
    (norm 0) and against gFillSinESol (norm 1) falls 4x per doubling of the
    grid (second order; exactly (A - 1) = k^2/12 + O(k^4))."""
    for key, norm in (("phi_sol_rms", 0), ("E_sol_rms", 1)):
        errs = [runs[native, d, norm, n][1][key] for n in SIZES]
        for a, b in zip(errs, errs[1:]):
            assert 3.9 < a / b < 4.1, (key, errs)
        # and the value is the closed form's discretisation error
        n = SIZES[-1]
        k = 2 * math.pi / n
        A = (k if norm else k * k) / (2 - 2 * math.cos(k))
        amp = abs(A - 1) if norm == 0 else abs(A * math.sin(k) - 1)
        # (to within the solver's own error, mg_sine.exact_bound x max|phi|)
        tol = runs[native, d, norm, n][2] * A * (1 if norm == 0 else math.sin(k))
        assert abs(errs[-1] - amp / math.sqrt(2)) <= tol, (errs[-1], amp / math.sqrt(2), tol)


def test_reference_norm0_e_comparison_does_not_converge(runs):
    """mgModeErrorScaling itself fills rho with norm = 0 and still compares
    E with gFillSinESol: E is then ~k cos(kJ), so that error tends to the
    RMS of cos (1/sqrt 2) instead of falling -- the harness is only
    consistent with norm = 1 for E, which the tests above use."""
    errs = [runs[False, 1, 0, n][1]["E_sol_rms"] for n in SIZES]
    assert errs[0] < errs[1] < errs[2] < 1 / math.sqrt(2)
