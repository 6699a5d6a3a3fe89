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


# ------------------------------------------------- main.c call for call --
def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mainc_cfg(nsub=(1, 1, 1), per_rank=(16, 16, 16), ppc=8, order=1):
    from pinc_amd import configs
    cfg = configs.config("cold3d", true_size=per_rank, nsub=nsub)
    cfg["multigrid"]["mgLevels"] = "3"
    cfg["population"]["nParticles"] = f"{ppc} pc"
    cfg["population"]["nAlloc"] = f"{2 * ppc} pc"
    # a Langmuir perturbation along x, so the energies are physical
    cfg["population"]["perturbAmplitude"] = "1e-3,0,0,0,0,0"
    # main.c always reads <files:output>test.grid.h5 (main.c:126-127); these
    # runs have no mask file and opt in to running without objects
    cfg["objects"] = {"optional": "1"}
    if order == 0:
        cfg["methods"]["acc"] = "puAccND0KE"
        cfg["methods"]["distr"] = "puDistrND0"
    return cfg


def _rank_lines(stdout: str):
    rows = re.findall(r"^STATUS: rank (\d+) KE (\S+) PE (\S+) N (\d+)$", stdout, flags=re.M)
    return np.array([[float(k), float(p), int(n)] for _, k, p, n in rows]).reshape(-1, 3)


def _run_mainc(ini, over, nranks, timeout=300):
    """pinc_mainc on nranks processes sharing the GPU (PINC_TRANSPORT=host):
    per-rank (KE, PE, N) rows per step, and the processes' outputs."""
    import build as cbuild
    exe = cbuild.build("pinc_mainc")
    env = dict(os.environ)
    env.pop("PINC_QUIET", None)
    if nranks > 1:
        env.update(PINC_WORLD_SIZE=str(nranks), PINC_TRANSPORT="host", PINC_MASTER_ADDR="127.0.0.1",
                   PINC_MASTER_PORT=str(_free_port()), PINC_BOOT_TIMEOUT="120")
    procs = []
    for r in range(nranks):
        e = dict(env)
        if nranks > 1:
            e["PINC_RANK"] = str(r)
        procs.append(subprocess.Popen([str(exe), ini, *over], env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=timeout))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for r, (p, (o, e)) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, (r, p.returncode, o[-2000:], e[-3000:])
    return [_rank_lines(o) for o, _ in outs], outs


def _history(path, name):
    from pinc_amd import _lib
    import ctypes as C
    buf = np.zeros(4096)
    n = _lib.HOST.pinc_h5_read(str(path).encode(), name.encode(), 0, buf.ctypes.data_as(C.c_void_p), buf.size)
    assert n > 0, (path, name, n)
    return buf[:n].reshape(-1, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("nranks,order", [(1, 1), (2, 1), (1, 0), (2, 0)])
def test_mainc_loop_matches_oracle_literal(built, tmp_path, nranks, order):
    """The reference's main.c loop, call for call (tests/c_driver/pinc_mainc.c:
    rho folded twice per step, both asserts, every output file, the objects'
    calls with no mask file), on 1 and 2 ranks launched as processes that take
    their world from PINC_RANK/PINC_WORLD_SIZE and share the GPU over the TCP
    host transport.  CIC and NGP (puAccND0KE/puDistrND0).  Energies summed
    over the ranks against the oracle's literal loop (main.c:226-240) to 1e-8;
    the history file holds the same sums (xyWrite MPI_SUM); rank 0 prints the
    Timer."""
    import orc
    from pinc_amd import configs
    steps = 4
    cfg = _mainc_cfg(nsub=(1, 1, nranks), order=order)
    ini = configs.write_ini(cfg)
    over = [f"time:nTimeSteps={steps}", f"files:output={tmp_path}/"]
    try:
        rows, outs = _run_mainc(ini, over, nranks)
        ke_o, pe_o, _ = orc.run_steps(ini, over[:1], steps, literal=True, perturb=True)
    finally:
        os.unlink(ini)
    for r in rows:
        assert r.shape == (steps, 3), r.shape
    ke = sum(r[:, 0] for r in rows)
    pe = sum(r[:, 1] for r in rows)
    np.testing.assert_allclose(ke, ke_o, rtol=1e-8)
    np.testing.assert_allclose(pe, pe_o, rtol=1e-8)
    # tMsg(t->total, ...) (main.c:276): with core.h's Timer layout (total
    # first) the value is the run's loop time, not a clock reading
    m = re.search(r"TIMER: Time spent:\s+([0-9.]+)(s|ms|us|ns)", outs[0][0])
    assert m, outs[0][0][-2000:]
    secs = float(m.group(1)) * {"s": 1.0, "ms": 1e-3, "us": 1e-6, "ns": 1e-9}[m.group(2)]
    assert 0.0 < secs < 300.0, m.group(0)
    assert "no objects" in outs[0][1]  # oReadH5 found no <output>test.grid.h5
    hk = _history(tmp_path / "history.xy.h5", "/energy/kinetic/total")
    hp = _history(tmp_path / "history.xy.h5", "/energy/potential/total")
    np.testing.assert_array_equal(hk[:, 0], np.arange(1, steps + 1))
    np.testing.assert_allclose(hk[:, 1], ke, rtol=1e-12)
    np.testing.assert_allclose(hp[:, 1], pe, rtol=1e-12)
    for f in ("rho.grid.h5", "rhoObj.grid.h5", "phi.grid.h5", "E.grid.h5", "pop.pop.h5"):
        assert (tmp_path / f).exists(), f


@pytest.mark.gpu
def test_mainc_loop_reads_object_mask(built, tmp_path):
    """main.c's object path through the reference's file API: the mask is
    <files:output>test.grid.h5 /Object [nz,ny,nx,1] (oOpenH5(..., "test") +
    oReadH5, object.c:717-756), and the literal loop with the capacitance
    correction runs against the checker's literal object step: counts exact,
    energies to 1e-7 (tests/test_gpu_objects.py's tolerances)."""
    import orc
    from pinc_amd import configs, _lib
    import ctypes as C
    steps = 4
    T = (16, 16, 16)
    sphere = (8.0, 8.0, 8.0, 2.5)
    cfg = _mainc_cfg()
    ini = configs.write_ini(cfg)
    mask = _sphere_mask(T, sphere[:3], sphere[3])
    dims = np.array([T[2], T[1], T[0], 1], dtype=np.int64)
    m = np.ascontiguousarray(mask.reshape(T[2], T[1], T[0], 1))
    rc = _lib.HOST.pinc_h5_write(str(tmp_path / "test.grid.h5").encode(), b"/Object", 4,
                                 dims.ctypes.data_as(C.c_void_p), m.ctypes.data_as(C.c_void_p))
    assert rc == 0
    over = [f"time:nTimeSteps={steps}", f"files:output={tmp_path}/"]
    try:
        rows, outs = _run_mainc(ini, over, 1)
        w = orc.World(ini, over[:1], True)
        w.init()
        ob = orc.Objects(w, mask)
        ob.capacitance()
        ob.init_collect()
        w.init_fields()
        for k in range(steps):
            ob.step()
            ke_o, pe_o = w.energy()
            assert rows[0][k, 2] == w.count(0) + w.count(1), (k, rows[0][k], w.count(0) + w.count(1))
            assert abs(rows[0][k, 0] - ke_o) <= 1e-7 * abs(ke_o), (k, rows[0][k, 0], ke_o)
            assert abs(rows[0][k, 1] - pe_o) <= 1e-7 * abs(pe_o), (k, rows[0][k, 1], pe_o)
        assert ob.collected(0) != 0.0
        w.close()
    finally:
        os.unlink(ini)
    assert "1 object(s)" in outs[0][0]


@pytest.mark.gpu
def test_mainc_velocity_assert_ends_run(built, tmp_path):
    """pVelAssertMax (main.c:206) with a bound the first kick exceeds ends the
    run with msg(ERROR) and a non-zero status, as population.c:342-365."""
    import build as cbuild
    from pinc_amd import configs
    exe = cbuild.build("pinc_mainc")
    cfg = _mainc_cfg()
    cfg["population"]["maxVel"] = "1e-12"
    ini = configs.write_ini(cfg)
    try:
        r = subprocess.run([str(exe), ini, "time:nTimeSteps=2", f"files:output={tmp_path}/"], capture_output=True,
                           text=True, timeout=300)
    finally:
        os.unlink(ini)
    assert r.returncode != 0
    assert "travels too fast" in r.stderr


@pytest.mark.gpu
def test_mainc_missing_object_mask_ends_run(built, tmp_path):
    """main.c reads its object mask unconditionally (main.c:126-127,
    object.c:727-756); without the file the reference's H5Dopen fails, so a
    mistyped files:output ends the run here too unless the ini opts in with
    objects:optional = 1."""
    import build as cbuild
    from pinc_amd import configs
    exe = cbuild.build("pinc_mainc")
    cfg = _mainc_cfg()
    del cfg["objects"]
    ini = configs.write_ini(cfg)
    try:
        r = subprocess.run([str(exe), ini, "time:nTimeSteps=1", f"files:output={tmp_path}/"], capture_output=True,
                           text=True, timeout=300)
    finally:
        os.unlink(ini)
    assert r.returncode != 0
    assert "no object mask" in r.stderr


@pytest.mark.gpu
def test_regular_two_ranks_from_launcher_env(built):
    """regular() (tests/c_driver/pinc_main.c, main.c's main()) on 2 processes
    whose world comes from PINC_RANK/PINC_WORLD_SIZE (the single-add loop),
    over the TCP host transport: rank 0's KE/PE lines, summed over the ranks,
    against the oracle's 2-slab run to 1e-8."""
    import orc
    import build as cbuild
    from pinc_amd import configs
    exe = cbuild.build("pinc_main")
    steps = 4
    cfg = _mainc_cfg(nsub=(1, 1, 2))
    ini = configs.write_ini(cfg)
    over = [f"time:nTimeSteps={steps}"]
    env = dict(os.environ, PINC_WORLD_SIZE="2", PINC_TRANSPORT="host", PINC_MASTER_ADDR="127.0.0.1",
               PINC_MASTER_PORT=str(_free_port()))
    env.pop("PINC_QUIET", None)
    try:
        procs = [subprocess.Popen([str(exe), ini, *over], env=dict(env, PINC_RANK=str(r)), stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, text=True) for r in range(2)]
        outs = [p.communicate(timeout=300) for p in procs]
        for p, (o, e) in zip(procs, outs):
            assert p.returncode == 0, (p.returncode, o[-2000:], e[-3000:])
        ke, pe = _energies(outs[0][0])
        assert len(ke) == steps
        assert not _energies(outs[1][0])[0].size  # msg(STATUS) prints on rank 0 only
        ke_o, pe_o, _ = orc.run_steps(ini, over, steps, perturb=True)
    finally:
        os.unlink(ini)
    np.testing.assert_allclose(ke, ke_o, rtol=1e-8)
    np.testing.assert_allclose(pe, pe_o, rtol=1e-8)
