"""Multi-rank parity on one GPU: two processes run the z-slab decomposition
(grid:nSubdomains=1,1,2) with the host transport over gloo (RCCL refuses two
ranks on one device), against the oracle's two-rank emulation.

The same host code runs with RCCL on a multi-GPU node; only the three
collectives in pinc_comm.c differ.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import orc
from pinc_amd import configs

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sorted_rows(a):
    a = np.asarray(a)
    return a[np.lexsort(a.T[::-1])]


@pytest.mark.parametrize("layout,poisson", [("reference", "mgSolver"), ("tiled", "mgSolver"),
                                            ("reference", "sSolver"), ("reference", "mgShard")])
def test_two_ranks_one_gpu(built, tmp_path, layout, poisson):
    """mgShard: native multigrid with level 0 sharded over the two slabs
    (8 halo planes, smoothing in chunks of 3 iterations) against the
    oracle's native solve."""
    cfg = configs.config("cold3d", true_size=(16, 16, 8), nsub=(1, 1, 2))
    cfg["multigrid"]["mgLevels"] = "3"
    if poisson == "mgShard":
        cfg["multigrid"]["native"] = "1"
        cfg["multigrid"]["shard"] = "1"
        poisson = "mgSolver"
    cfg["methods"]["poisson"] = poisson
    ini_ref = configs.write_ini(cfg)
    if layout == "tiled":
        cfg["population"]["layout"] = "tiled"
        cfg["population"]["sortInterval"] = "2"
    ini = configs.write_ini(cfg)
    steps = 3
    w = orc.World(ini_ref)
    assert w.nranks == 2
    w.init()
    w.init_fields()
    state = tmp_path / "state"
    for r in range(2):
        d = {}
        for sp in range(2):
            d[f"pos{sp}"], d[f"vel{sp}"], _ = w.particles(sp, rank=r)
        np.savez(f"{state}_r{r}.npz", **d)
    out = tmp_path / "out"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "tests" / "mp_worker.py"),
           "--ini", ini, "--state", str(state), "--out", str(out), "--steps", str(steps)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]

    for op in ("move", "extract", "migrate"):
        w.op(op)
    for r in range(2):
        g = np.load(f"{out}_r{r}.npz")
        for sp in range(2):
            po, vo, _ = w.particles(sp, rank=r)
            if layout == "reference":
                # same particles in the same order (receive order of puMigrate)
                np.testing.assert_array_equal(g[f"pos{sp}"], po)
                np.testing.assert_array_equal(g[f"vel{sp}"], vo)
            else:
                np.testing.assert_array_equal(_sorted_rows(g[f"pos{sp}"]), _sorted_rows(po))
        if layout == "reference":
            np.testing.assert_array_equal(g["emigrants"], w.emigrants(rank=r))
    for op in ("distr", "solve", "efield", "acc"):
        w.op(op)
    e_o = [w.energy()]
    for _ in range(steps):
        w.step()
        e_o.append(w.energy())
    res = [json.loads(Path(f"{out}_r{r}.json").read_text()) for r in range(2)]
    for r in range(2):
        e = np.array(res[r]["energy"])[1:]   # after full steps
        eo = np.array(e_o)[1:]
        assert np.all(np.abs(e - eo) <= 1e-8 * np.abs(eo)), (r, e, eo)
        assert res[r]["counts"] == [w.count(sp, rank=r) for sp in range(2)]
