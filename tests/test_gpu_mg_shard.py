"""Sharded multigrid level 0.

Native mode with multigrid:shard = 1 keeps level 0 as each rank's z-slab
extended by hz halo planes on each side, refreshed from the neighbouring
slabs before every chunk of smoothing iterations; the coarser levels are
all-gathered and solved on every rank.  The potential is the same discrete
solution as the replicated solve's, reached through the same operations:
only the summation order of the neutralisation means and of the residual
norm differs (per-slab partial sums, then summed over the ranks).  Checked
against the oracle's restatement of native mode (oracle/orc_native.c) on the
same charge density, at one rank (the halo is the slab's own periodic image)
and at two ranks on one GPU over the host transport (gloo), through the fused
sweeps and through the colour-by-colour passes.
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent))
import mg_history  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module", autouse=True)
def _built(built):
    return built


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _check_hist(hg, ho, rtol=1e-6, floor=1e-8):
    hg, ho = np.asarray(hg), np.asarray(ho)
    assert abs(len(hg) - len(ho)) <= 1, (len(hg), len(ho))
    n = min(len(hg), len(ho))
    sel = ho[:n] > floor
    assert np.all(np.abs(hg[:n] - ho[:n])[sel] < rtol * ho[:n][sel]), (hg[:n], ho[:n])


@pytest.mark.parametrize("size", [128, 256])
def test_one_rank_shard_matches_native_oracle(size):
    """One rank, shard forced: the extended slab (24 halo planes, fused
    two-iteration sweeps) against the oracle's native solve."""
    g = mg_history.run("gpu", size, 5, 200, 20261016, 1.0, native=True, shard="1")
    assert g["shard_halo"] == 24
    o = mg_history.run("oracle", size, 5, 200, 20261016, 1.0, native=True)
    assert g["residual"][-1][-1] <= 1e-10 and o["residual"][-1][-1] <= 1e-10
    _check_hist(g["residual"][-1], o["residual"][-1])
    assert np.max(np.abs(g["phi"] - o["phi"])) <= 1e-9 * np.max(np.abs(o["phi"]))


@pytest.mark.parametrize("shard", ["1", "0"])
def test_spectral_coarse_matches_native_oracle(shard):
    """multigrid:spectralCoarse at 128^3 (the level-1 correction solved
    exactly by rocFFT with the 7-point symbol; a two-grid cycle), on the
    sharded extended slab (shard forced, one rank) and replicated, against
    the oracle's restatement (orc_discrete_poisson): residual history per
    cycle, phi to 1e-9 of its maximum."""
    g = mg_history.run("gpu", 128, 5, 200, 20261016, 1.0, native=True, shard=shard, spectral_coarse=True)
    o = mg_history.run("oracle", 128, 5, 200, 20261016, 1.0, native=True, spectral_coarse=True)
    assert g["residual"][-1][-1] <= 1e-10 and o["residual"][-1][-1] <= 1e-10
    _check_hist(g["residual"][-1], o["residual"][-1])
    assert np.max(np.abs(g["phi"] - o["phi"])) <= 1e-9 * np.max(np.abs(o["phi"]))


def _two_ranks(size, levels, tmp_path, fused_min=None, cycles=60, solves=2, world=2, spectral_coarse=False):
    out = tmp_path / "shard"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    if fused_min is not None:
        env["PINC_MG_FUSED_MIN"] = str(fused_min)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "tests" / "shard_worker.py"),
           "--size", str(size), "--levels", str(levels), "--cycles", str(cycles), "--solves", str(solves),
           "--out", str(out)] + (["--spectral-coarse"] if spectral_coarse else [])
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return [dict(np.load(f"{out}_r{r}.npz")) for r in range(world)]


def _oracle_two_ranks(size, levels, cycles=60, solves=2, world=2, spectral_coarse=False):
    import orc
    ini = mg_history.ini_for(size, levels, True, nranks=world, spectral_coarse=spectral_coarse)
    rho = mg_history.make_rho(size, 20261016, 1.0)
    try:
        w = orc.World(ini)
        assert w.nranks == world
        w.mg_limit(cycles, cycles)
        hists = []
        for _ in range(solves):
            for r in range(world):
                w.set_grid(0, mg_history.rank_slab(rho, r, world), rank=r)
            w.op("solve")
            hists.append(w.mg_history())
        phi = [w.grid(1, rank=r)[..., 0].copy() for r in range(world)]
        w.op("efield")
        E = [w.grid(2, rank=r).copy() for r in range(world)]
        w.close()
    finally:
        os.unlink(ini)
    return hists, phi, E


@pytest.mark.parametrize("size,levels,fused_min", [(64, 4, None), (64, 4, 1), (128, 5, None)])
def test_two_ranks_shard_matches_oracle(tmp_path, size, levels, fused_min):
    """Two z-slabs, halo planes exchanged over the host transport: every
    rank's residual history equals the oracle's two-rank native solve (1e-6
    above 1e-8), the potential to 1e-9 of its maximum, E to 1e-8; the second
    solve (warm start from the first's potential) too."""
    g = _two_ranks(size, levels, tmp_path, fused_min)
    ho, po, Eo = _oracle_two_ranks(size, levels)
    for r in range(2):
        assert int(g[r]["halo"]) > 0
        for k in range(2):
            _check_hist(g[r][f"hist{k}"], ho[k])
        scale = max(np.max(np.abs(p[1:-1])) for p in po)
        assert np.max(np.abs(g[r]["phi"][1:-1] - po[r][1:-1])) <= 1e-9 * scale
        inner = (slice(1, -1),) * 3
        escale = max(np.max(np.abs(e[inner])) for e in Eo)
        assert np.max(np.abs(g[r]["E"][inner] - Eo[r][inner])) <= 1e-8 * escale
    assert g[0]["hist0"][-1] <= 1e-10


def test_four_ranks_shard_matches_oracle(tmp_path):
    """Four z-slabs of 32 planes at 128^3 -- one rank's level-0 geometry at
    C4 on 8 GPUs (24 halo planes, 80-plane extended slab), and distinct
    z-1 / z+1 neighbours -- against the oracle's four-rank native solve."""
    world = 4
    g = _two_ranks(128, 5, tmp_path, world=world)
    ho, po, Eo = _oracle_two_ranks(128, 5, world=world)
    scale = max(np.max(np.abs(p[1:-1])) for p in po)
    for r in range(world):
        assert int(g[r]["halo"]) == 24
        for k in range(2):
            _check_hist(g[r][f"hist{k}"], ho[k])
        assert np.max(np.abs(g[r]["phi"][1:-1] - po[r][1:-1])) <= 1e-9 * scale


@pytest.mark.parametrize("world", [2, 4])
def test_ranks_decomposed_level1_matches_oracle(tmp_path, world):
    """multigrid:spectralCoarse on the sharded level 0 with the level-1 solve
    decomposed as well (the reference keeps every level
    on its subdomain, multigrid.c:128-180, 1496-1556): each rank's restricted
    residual planes go through the slab-distributed transform with the
    7-point symbol, one level-1 halo plane comes from each neighbour, and
    only the owned level-0 planes are corrected.  No all-gather in the
    solve: the transposes replace it.  Against the oracle's native solve with
    the exact level-1 solve (orc_discrete_poisson), 128^3 in 2 and 4 z-slabs:
    residual history per cycle, phi to 1e-9 of its maximum, E to 1e-8."""
    g = _two_ranks(128, 5, tmp_path, world=world, spectral_coarse=True)
    ho, po, Eo = _oracle_two_ranks(128, 5, world=world, spectral_coarse=True)
    scale = max(np.max(np.abs(p[1:-1])) for p in po)
    inner = (slice(1, -1),) * 3
    escale = max(np.max(np.abs(e[inner])) for e in Eo)
    for r in range(world):
        assert int(g[r]["halo"]) > 0
        # the level-1 all-gather is gone; the transposes carry level 1
        assert g[r]["comm_allgather"][0] == 0, g[r]["comm_allgather"]
        assert g[r]["comm_spectral_transpose"][0] > 0
        for k in range(2):
            _check_hist(g[r][f"hist{k}"], ho[k])
        assert np.max(np.abs(g[r]["phi"][1:-1] - po[r][1:-1])) <= 1e-9 * scale
        assert np.max(np.abs(g[r]["E"][inner] - Eo[r][inner])) <= 1e-8 * escale
    assert g[0]["hist0"][-1] <= 1e-10


def test_shard_off_below_threshold(tmp_path):
    """multigrid:shard defaults to auto: one rank solves replicated."""
    ini = mg_history.ini_for(32, 3, True)
    from pinc_amd import Sim
    try:
        with Sim(ini, perturb=False) as s:
            assert s.mg_shard == 0
    finally:
        os.unlink(ini)
