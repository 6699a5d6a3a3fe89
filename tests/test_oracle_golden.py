"""The oracle against outputs of the reference itself (SURVEY.md Appendix B,
recorded from the reference's own C sources; tests/golden/reference_outputs.json).

These pin the oracle; the GPU parity tests then compare the MI355X path with
the pinned oracle.  CPU only, each case runs in a few seconds.
"""
import json
from pathlib import Path

import numpy as np
import pytest

import orc
from pinc_amd import configs

GOLD = json.loads((Path(__file__).parent / "golden" / "reference_outputs.json").read_text())["standin_build_runs"]


def ke_peak_omega(ke, dt):
    """Langmuir frequency from parabolic-interpolated kinetic-energy peaks:
    KE peaks twice per plasma period, so omega = pi / (T_steps * dt)
    ('Langmuir validation')."""
    t = []
    for i in range(1, len(ke) - 1):
        if ke[i] > ke[i - 1] and ke[i] >= ke[i + 1]:
            a, b, c = ke[i - 1], ke[i], ke[i + 1]
            den = a - 2 * b + c
            t.append(i + (0.5 * (a - c) / den if den != 0 else 0.0))
    assert len(t) >= 2, "fewer than two KE peaks"
    return np.pi / (np.mean(np.diff(t)) * dt)


def _run(name, steps, literal=False, **kw):
    cfg = configs.config(name, **kw)
    ini = configs.write_ini(cfg)
    try:
        ke, pe, cyc = orc.run_steps(ini, [], steps, literal=literal)
    finally:
        Path(ini).unlink()
    return ke, pe, cyc, float(cfg["time"]["timeStep"])


def test_cold3d_first_step_exact():
    g = GOLD["cold3d_1rank"]
    ke, pe, _, _ = _run("cold3d", 1)
    assert ke[0] == g["KE1"]
    assert pe[0] == g["PE1"]


def test_langmuir2d_energy_and_frequency():
    g = GOLD["langmuir2d"]
    ke, _, _, dt = _run("langmuir2d", 150)
    assert np.allclose(ke[:3], g["KE"], rtol=0, atol=5e-9)
    assert abs(ke_peak_omega(ke, dt) - g["omega_150"]) < 5e-6


def test_langmuir2d_literal_mainc():
    g = GOLD["langmuir2d"]
    ke, _, _, dt = _run("langmuir2d", 150, literal=True)
    assert abs(ke[0] - g["literal_KE1"]) < 5e-9
    assert abs(ke_peak_omega(ke, dt) - g["literal_omega_150"]) < 5e-6


def test_langmuir1d_cycles_and_frequency():
    g = GOLD["langmuir1d"]
    ke, _, cyc, dt = _run("langmuir1d", 150)
    assert cyc[-1] == g["cycles_150"]
    assert abs(ke_peak_omega(ke, dt) - g["omega_150"]) < 5e-6


def test_c2_first_step():
    g = GOLD["c2"]
    ke, _, _, _ = _run("c2", 1)
    assert abs(ke[0] - g["KE1"]) < 5e-8 * 10
    ke, _, _, _ = _run("c2", 1, literal=True)
    assert abs(ke[0] - g["literal_KE1"]) < 5e-8 * 10


def test_rank_independence_4_ranks():
    """4 emulated ranks (1x2x2 of 32x16x16) against 1 rank of 32^3."""
    g = GOLD["cold3d_4rank"]
    ke4, pe4, _, _ = _run("cold3d", 3, nsub=(1, 2, 2))
    ke1, pe1, _, _ = _run("cold3d", 3, true_size=(32, 32, 32))
    assert abs(ke4[0] - g["KE1"]) < 5e-9 and abs(pe4[0] - g["PE1"]) < 5e-9
    assert np.max(np.abs(ke4 - ke1) / np.abs(ke1)) < 1e-10
    assert np.max(np.abs(pe4 - pe1) / np.abs(pe1)) < 1e-11


@pytest.mark.slow
def test_c2_frequency():
    g = GOLD["c2"]
    ke, _, _, dt = _run("c2", 150)
    assert abs(ke_peak_omega(ke, dt) - g["omega_150"]) < 5e-6
