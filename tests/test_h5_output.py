"""The reference's output files.

Layouts follow grid.c:1161-1270 (.grid.h5), population.c:497-698 (.pop.h5
and the energy datasets) and io.c:566-734 (history.xy.h5).  h5py is not
installed, so files are read back through the library's own run-time HDF5
binding (pinc_h5_read).  The reference's writer needs parallel HDF5 and
does not build here, so the layout is pinned by the reference source text
(dataset names, dims order, attributes), not by reference-written files.
"""
import ctypes as C
import os
from pathlib import Path

import numpy as np
import pytest
# torch's HIP runtime comes up before the native library (see conftest.built)
import torch  # noqa: F401

from pinc_amd import configs

ROOT = Path(__file__).resolve().parent.parent


def _host():
    from pinc_amd._lib import HOST
    return HOST


def _need_h5():
    from pinc_amd.sim import h5_available
    if not h5_available():
        pytest.skip("no libhdf5 on this machine (PINC_HDF5_LIB)")


def test_history_rows_roundtrip(tmp_path):
    """xyOpenH5 / xyCreateDataset / xyWrite (io.c:651-734): an extendible
    [n, 2] dataset per series, one (x, y) row appended per write."""
    _need_h5()
    from pinc_amd.sim import h5_read
    H = _host()
    H.iniFromString.restype = C.c_void_p
    H.iniFromString.argtypes = [C.c_char_p]
    H.xyOpenH5.restype = C.c_longlong
    H.xyOpenH5.argtypes = [C.c_void_p, C.c_char_p]
    H.xyCreateDataset.argtypes = [C.c_longlong, C.c_char_p]
    H.xyWrite.argtypes = [C.c_longlong, C.c_char_p, C.c_double, C.c_double, C.c_int]
    H.xyCloseH5.argtypes = [C.c_longlong]
    H.iniClose.argtypes = [C.c_void_p]
    ini = H.iniFromString(f"[files]\noutput = {tmp_path}/run\n".encode())
    h = H.xyOpenH5(ini, b"history")
    assert h > 0
    H.xyCreateDataset(h, b"/energy/kinetic/total")
    H.xyCreateDataset(h, b"/a/b/c")
    rows = [(1.0, 2.5), (2.0, -1.25), (3.0, 1e300)]
    for x, y in rows:
        H.xyWrite(h, b"/energy/kinetic/total", x, y, 0)
    H.xyWrite(h, b"/a/b/c", 7.0, 8.0, 1)
    H.xyCloseH5(h)
    H.iniClose(ini)
    f = tmp_path / "run_history.xy.h5"   # prefix + '_' + name + .xy.h5 (io.c:571-576)
    assert f.exists()
    np.testing.assert_array_equal(h5_read(f, "/energy/kinetic/total"), np.array(rows))
    np.testing.assert_array_equal(h5_read(f, "/a/b/c"), np.array([[7.0, 8.0]]))


@pytest.mark.gpu
def test_grid_pop_history_files(built, tmp_path):
    """main.c's output of one step: rho/phi/E datasets equal the true nodes
    of the device grids, positions (global frame) and velocities equal the
    population, the history rows equal the energies."""
    _need_h5()
    from pinc_amd import Sim
    from pinc_amd.sim import h5_read
    cfg = configs.config("cold3d")
    cfg["files"] = {"output": str(tmp_path) + "/"}
    ini = configs.write_ini(cfg)
    with Sim(ini) as s:
        s.init()
        s.step()
        s.open_output()
        s.write_output(1)
        s.sync()
        ke, pe, kes = s.energy()
        grids = {name: s.grid(w) for w, name in enumerate(["rho", "phi", "E"])}
        parts = [s.particles(sp) for sp in range(s.nspecies)]
        nd = s.ndims
    # closed with the simulation
    for name, g in grids.items():
        f = tmp_path / f"{name}.grid.h5"      # '/'-terminated prefix: no separator
        a = h5_read(f, "/n=1.0")
        true = g[1:-1, 1:-1, 1:-1, :]          # [z, y, x, v] true nodes
        assert a.shape == true.shape, (name, a.shape, true.shape)
        np.testing.assert_array_equal(a, true)
        assert h5_read(f, "Quantity denormalization factor", attr=True)[0] == 1.0
        assert h5_read(f, "Axis denormalization factor", attr=True)[0] > 0
    f = tmp_path / "pop.pop.h5"
    for sp, (pos, vel) in enumerate(parts):
        p = h5_read(f, f"/pos/specie {sp}/n=1.0")
        v = h5_read(f, f"/vel/specie {sp}/n=1.5")
        assert p.shape == (pos.shape[0], nd)
        # global frame: local + subdomain*trueSize - nGhost (gAllocMpi offset)
        np.testing.assert_array_equal(p, pos - 1.0)
        np.testing.assert_array_equal(v, vel)
    assert h5_read(f, "Velocity denormalization factor", attr=True)[0] > 0
    f = tmp_path / "history.xy.h5"
    np.testing.assert_allclose(h5_read(f, "/energy/kinetic/total"), [[1.0, ke]], rtol=0, atol=0)
    np.testing.assert_allclose(h5_read(f, "/energy/potential/total"), [[1.0, pe]], rtol=0, atol=0)
    for sp in range(len(parts)):
        np.testing.assert_allclose(h5_read(f, f"/energy/kinetic/specie {sp}"), [[1.0, kes[sp]]], rtol=0, atol=0)


def _sorted_rows(a):
    return a[np.lexsort(a.T[::-1])]


@pytest.mark.gpu
def test_two_rank_files_match_one_rank(built, tmp_path):
    """z-slabs on two ranks (host transport, one GPU): rank 0 writes the
    all-gathered datasets, which match a one-rank run of the same problem
    (grids to the multi-rank tolerance, particles as sets, bit-exact)."""
    _need_h5()
    import socket
    import subprocess
    import sys
    from pinc_amd import Sim
    from pinc_amd.sim import h5_read
    cfg1 = configs.config("cold3d", true_size=(16, 16, 16), nsub=(1, 1, 1))
    cfg1["multigrid"]["mgLevels"] = "3"
    cfg1["files"] = {"output": str(tmp_path / "one") + "/"}
    with Sim(configs.write_ini(cfg1)) as s:
        s.init()
        s.step()
        s.write_output(1)
    cfg2 = configs.config("cold3d", true_size=(16, 16, 8), nsub=(1, 1, 2))
    cfg2["multigrid"]["mgLevels"] = "3"
    cfg2["files"] = {"output": str(tmp_path / "two") + "/"}
    ini2 = configs.write_ini(cfg2)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", str(ROOT / "tests" / "h5_worker.py"),
                        "--ini", ini2], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    for name in ("rho", "phi", "E"):
        a = h5_read(tmp_path / "one" / f"{name}.grid.h5", "/n=1.0")
        b = h5_read(tmp_path / "two" / f"{name}.grid.h5", "/n=1.0")
        assert a.shape == b.shape == (16, 16, 16, a.shape[-1])
        scale = np.max(np.abs(a))
        assert np.max(np.abs(a - b)) <= 1e-9 * scale, name
    for sp in range(2):
        for kind, n in (("pos", "1.0"), ("vel", "1.5")):
            a = h5_read(tmp_path / "one" / "pop.pop.h5", f"/{kind}/specie {sp}/n={n}")
            b = h5_read(tmp_path / "two" / "pop.pop.h5", f"/{kind}/specie {sp}/n={n}")
            assert a.shape == b.shape
        pa = np.hstack([h5_read(tmp_path / "one" / "pop.pop.h5", f"/pos/specie {sp}/n=1.0"),
                        h5_read(tmp_path / "one" / "pop.pop.h5", f"/vel/specie {sp}/n=1.5")])
        pb = np.hstack([h5_read(tmp_path / "two" / "pop.pop.h5", f"/pos/specie {sp}/n=1.0"),
                        h5_read(tmp_path / "two" / "pop.pop.h5", f"/vel/specie {sp}/n=1.5")])
        # same particles: the move runs in each rank's local frame, so the
        # positions round differently than on one rank (1e-12); rows are
        # matched through positions rounded to 1e-6
        def order(p):
            k = np.round(p[:, :3] * 1e6)
            return p[np.lexsort(k.T[::-1])]
        ra, rb = order(pa), order(pb)
        assert np.max(np.abs(ra[:, :3] - rb[:, :3])) <= 1e-12
        assert np.max(np.abs(ra[:, 3:] - rb[:, 3:])) <= 1e-9
    for ser in ("/energy/kinetic/total", "/energy/potential/total"):
        a = h5_read(tmp_path / "one" / "history.xy.h5", ser)
        b = h5_read(tmp_path / "two" / "history.xy.h5", ser)
        np.testing.assert_allclose(a, b, rtol=1e-8)
