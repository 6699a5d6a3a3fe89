"""The drop-in C path and process teardown.

* tests/c_driver/pinc_main.c is a C caller in the shape of the reference's
  main.c:19-48: iniOpen(argc, argv) with key=value overrides, then
  select(ini, "methods:mode", regular_set) and the run mode.  It links
  libpinc.so only: no Python, no torch.  On the GPU its per-step
  "KE .. PE .." STATUS lines (regular(), main.c:197-274) must match the
  oracle's energy history, and it must exit 0.
* Python processes that import pinc_amd before or after torch must exit 0
  (round 1 hid an abort at exit behind the import order, ADVICE r01: two
  ROCm stacks in one process, see pinc_amd/_lib.py).
"""
import os
import re
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests" / "c_driver"))

HAVE_GPU = Path("/dev/kfd").exists()


def _driver(built):
    import build as cbuild
    return cbuild.build()


def _energies(stdout: str):
    ke, pe = [], []
    for m in re.finditer(r"^STATUS: KE (\S+) PE (\S+)$", stdout, flags=re.M):
        ke.append(float(m.group(1)))
        pe.append(float(m.group(2)))
    return np.array(ke), np.array(pe)


@pytest.mark.skipif(HAVE_GPU, reason="checks the no-GPU error path")
def test_c_driver_fails_loudly_without_gpu(built):
    """No CPU fallback: without a device the run mode ends in msg(ERROR)."""
    from pinc_amd import configs
    exe = _driver(built)
    ini = configs.write_ini(configs.config("cold3d"))
    try:
        r = subprocess.run([str(exe), ini, "time:nTimeSteps=1"], capture_output=True, text=True, timeout=60)
    finally:
        os.unlink(ini)
    assert r.returncode != 0
    assert "ERROR" in r.stderr and "hip" in r.stderr.lower()


@pytest.mark.gpu
@pytest.mark.parametrize("name,over", [
    ("cold3d", ["time:nTimeSteps=4"]),
    ("langmuir2d", ["time:nTimeSteps=4"]),
    ("c3small", ["time:nTimeSteps=3"]),
])
def test_c_driver_regular_matches_oracle(built, name, over):
    import orc
    from pinc_amd import configs
    exe = _driver(built)
    if name == "c3small":
        # a Langmuir perturbation along x (0.005 cells), so that the energies
        # are physical rather than round-off of a cold lattice
        cfg = configs.config("c3", true_size=(32, 32, 32), ppc=4)
        cfg["population"]["perturbAmplitude"] = "1e-3,0,0,0,0,0"
        cfg["population"]["perturbMode"] = "1,0,0,0,0,0"
    else:
        cfg = configs.config(name)
    ini = configs.write_ini(cfg)
    try:
        env = dict(os.environ)
        env.pop("PINC_QUIET", None)
        r = subprocess.run([str(exe), ini, *over], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
        assert "completed successfully" in r.stdout
        ke, pe = _energies(r.stdout)
        nsteps = int(over[0].split("=")[1])
        assert len(ke) == nsteps
        ke_o, pe_o, _ = orc.run_steps(ini, over, nsteps, perturb=True)
    finally:
        os.unlink(ini)
    np.testing.assert_allclose(ke, ke_o, rtol=1e-8)
    np.testing.assert_allclose(pe, pe_o, rtol=1e-8)


_PROG = r"""
import sys
sys.path.insert(0, {root!r})
order = {order!r}
if order == "torch_first":
    import torch
    x = torch.ones(4, device="cuda")
from pinc_amd import Sim, configs
if order == "pinc_first":
    import torch
    x = torch.ones(4, device="cuda")
ini = configs.write_ini(configs.config("c3", true_size=(16, 16, 16), ppc=2))
with Sim(ini) as s:
    s.init()
    s.step(2)
    ke, pe, _ = s.energy()
torch.cuda.synchronize()
print("ok", ke, pe, float(x.sum()))
"""


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["pinc_first", "torch_first"])
def test_process_exits_cleanly_in_either_import_order(built, order):
    """A spectral (rocFFT) run next to torch, in both import orders: the
    process must exit 0 (no abort in the runtimes' teardown)."""
    r = subprocess.run([sys.executable, "-c", _PROG.format(root=str(ROOT), order=order)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout[-1500:], r.stderr[-3000:])
    assert r.stdout.startswith("ok")


def _sphere_mask(T, c, r):
    z, y, x = np.meshgrid(*[np.arange(t, dtype=float) for t in (T[2], T[1], T[0])], indexing="ij")
    return (((x - c[0]) ** 2 + (y - c[1]) ** 2 + (z - c[2]) ** 2) <= r * r).astype(float)


@pytest.mark.gpu
@pytest.mark.parametrize("fused,layout", [(1, "reference"), (0, "reference"), (1, "tiled")])
def test_reference_object_api_matches_checker(built, fused, layout):
    """main.c's object loop driven through the reference's own API
    (tests/c_driver/pinc_objmain.c: oAlloc, oComputeCapacitanceMatrix,
    oCollectObjectCharge into the caller's rhoObj, gAddTo, solve,
    oApplyCapacitanceMatrix, solve), which never attaches the object to the
    population up front.  With population:fused = 1 the first collection
    must discard the push's deposit (it tested no object) and attach the
    object for the pushes after it (particles inside were
    counted twice, in rhoS and rhoObj).  Counts exact, energies to 1e-7
    against the checker (tolerances of tests/test_gpu_objects.py)."""
    import orc
    from pinc_amd import configs
    import build as cbuild
    exe = cbuild.build("pinc_objmain")
    T, sphere, steps = (16, 16, 16), (8.0, 8.0, 8.0, 2.5), 4
    cfg = configs.config("cold3d", true_size=T, nsub=(1, 1, 1))
    cfg["multigrid"]["mgLevels"] = "3"
    cfg["population"]["fused"] = "0"
    cfg["objects"] = {"sphere": ",".join(map(str, sphere))}
    cfg["time"]["nTimeSteps"] = str(steps)
    ini = configs.write_ini(cfg)
    cfg["population"]["fused"] = str(fused)
    if layout == "tiled":
        cfg["population"]["layout"] = "tiled"
        cfg["population"]["sortInterval"] = "2"
    ini_dev = configs.write_ini(cfg)
    try:
        env = dict(os.environ)
        env.pop("PINC_QUIET", None)
        r = subprocess.run([str(exe), ini_dev], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
        ke, pe = _energies(r.stdout)
        n = [int(m.group(1)) for m in re.finditer(r"^STATUS: N (\d+)$", r.stdout, flags=re.M)]
        assert len(ke) == steps and len(n) == steps
        w = orc.World(ini)
        w.init()
        ob = orc.Objects(w, _sphere_mask(T, sphere[:3], sphere[3]))
        ob.capacitance()
        ob.init_collect()
        w.init_fields()
        for k in range(steps):
            ob.step()
            ke_o, pe_o = w.energy()
            assert n[k] == w.count(0) + w.count(1), (k, n[k])
            assert abs(ke[k] - ke_o) <= 1e-7 * abs(ke_o), (k, ke[k], ke_o)
            assert abs(pe[k] - pe_o) <= 1e-7 * abs(pe_o), (k, pe[k], pe_o)
        assert ob.collected(0) != 0.0
        w.close()
    finally:
        os.unlink(ini)
        os.unlink(ini_dev)
