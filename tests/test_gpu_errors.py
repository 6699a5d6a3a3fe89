"""Error paths of the hot path.

The reference stops a run through msg(ERROR, ...) -> exit(EXIT_FAILURE)
(io.c:170-217) when
  * a velocity exceeds population:maxVel (pVelAssertMax, population.c:342-365,
    signed comparison, called every step at main.c:206);
  * a particle is outside its local frame after migration
    (pPosAssertInLocalFrame, population.c:316-340, main.c:219);
and leaves two overflows unchecked: the emigrant buffers (the TODO at
pusher.c:776,858) and the import into a full population (pusher.c:967-985).
Here the first two stop with msg(ERROR) (also in the fused push, whose
kernel keeps a bad particle away from the deposit), the emigrant buffer
grows instead of overflowing (same result as a large buffer, bit for bit),
and an import overflow stops with msg(ERROR).  Each scenario runs in a
subprocess (tests/err_worker.py) and must end with a non-zero exit code and
the right message.
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
WORKER = str(ROOT / "tests" / "err_worker.py")


def _run(args, timeout=240):
    return subprocess.run([sys.executable, WORKER, *args], capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
@pytest.mark.parametrize("layout,fused", [("reference", 1), ("reference", 0), ("tiled", 1), ("tiled", 0)])
def test_maxvel_exceeded_stops_run(built, layout, fused):
    r = _run(["maxvel", "--layout", layout, "--fused", str(fused)])
    assert r.returncode != 0 and "REACHED-END" not in r.stdout, (r.stdout[-800:], r.stderr[-800:])
    assert "ERROR" in r.stderr and "maxVel" in r.stderr, r.stderr[-800:]


@pytest.mark.gpu
@pytest.mark.parametrize("layout,fused", [("reference", 1), ("reference", 0), ("tiled", 1), ("tiled", 0)])
def test_particle_outside_local_frame_stops_run(built, layout, fused):
    r = _run(["frame", "--layout", layout, "--fused", str(fused)])
    assert r.returncode != 0 and "REACHED-END" not in r.stdout, (r.stdout[-800:], r.stderr[-800:])
    assert "ERROR" in r.stderr and "out of bounds" in r.stderr, r.stderr[-800:]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_population_overflow_on_migration_stops_run(built):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", WORKER, "overflow"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    assert r.returncode != 0, out[-2000:]
    assert "population overflow on migration" in out, out[-2000:]


@pytest.mark.gpu
def test_emigrant_buffer_grows_instead_of_overflowing(built):
    """grid:nEmigrantsAlloc far below the number of emigrants: the device
    extract grows its buffers and ends with the oracle run's emigrant counts
    (exact) and particles (same order; positions to 1e-9, the E field that
    moved them differs in summation order) with buffers large enough (the
    reference would write past them)."""
    import orc
    from pinc_amd import Sim, configs
    cfg = configs.config("warm", true_size=(16, 16, 16), ppc=8, nalloc_pc=12)
    cfg["multigrid"]["mgLevels"] = "3"
    big = configs.write_ini(cfg)
    cfg["grid"]["nEmigrantsAlloc"] = "1,1,1"
    tiny = configs.write_ini(cfg)
    try:
        w = orc.World(big)
        w.init(perturb=False, maxwell=True, seed=11)
        w.init_fields()
        with Sim(tiny, perturb=False, maxwell=True, seed=11) as s:
            s.init()
            for _ in range(3):
                s.step()
                w.step()
                em = s.emigrants()
                assert em.max() > 10  # far beyond the one record per direction allocated
                np.testing.assert_array_equal(em, w.emigrants())
                for sp in range(2):
                    pg, vg = s.particles(sp)
                    po, vo, _ = w.particles(sp)
                    assert pg.shape == po.shape
                    np.testing.assert_allclose(pg, po, rtol=0, atol=1e-9)
    finally:
        os.unlink(big)
        os.unlink(tiny)


def test_oracle_emigrant_buffer_overflow_is_an_error(built):
    """The checker refuses to write past grid:nEmigrantsAlloc (orc_die), so a
    run that would overflow the reference's buffers cannot pass silently."""
    from pinc_amd import configs
    cfg = configs.config("warm", true_size=(16, 16, 16), ppc=8, nalloc_pc=12)
    cfg["multigrid"]["mgLevels"] = "3"
    cfg["grid"]["nEmigrantsAlloc"] = "1,1,1"
    ini = configs.write_ini(cfg)
    prog = ("import sys; sys.path.insert(0, %r); import orc; w = orc.World(%r); "
            "w.init(perturb=False, maxwell=True, seed=11); w.init_fields(); w.step(); print('REACHED-END')"
            % (str(ROOT / "oracle"), ini))
    try:
        r = subprocess.run([sys.executable, "-c", prog], capture_output=True, text=True, timeout=120)
    finally:
        os.unlink(ini)
    assert r.returncode != 0 and "REACHED-END" not in r.stdout
    assert "overflow" in r.stderr
