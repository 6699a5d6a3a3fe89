"""The push's two host-side shortcuts change no result:

  * PINC_EXTRACT_SKIP (default on): a species whose last push flagged no
    particle to leave skips its extraction (pinc_pusher.c extract);
  * PINC_FLAGS_SPARSE (default on): when a species' flags are all the centre
    (the extraction puts the extracted ones back), the push writes only its
    leavers' flags (pinc_flags_before_write).

Each switch setting runs in its own process (the library reads them when
its context is created), from the same seeded device initialisation, with
the bench's flags (tiled layout, adaptive in-push sort, fused push):

  * C5's immersed sphere on one rank (the push flags collected particles as
    sinks, so species take turns having leavers and none; the object loop
    extracts them);
  * C4 on two z-slabs over the host transport (emigrants cross every step).

The device path is not bit-reproducible from run to run (the charge
deposit sums with atomics, the in-push sort ranks with LDS atomics), so
runs are compared the way two runs of one setting agree: every step's
emigrant counts exactly, the collected charge exactly, the particle counts
exactly, the energies to 1e-11 relative, and each particle component as a
sorted list (the marginal distributions, order-free) to 1e-9 of its scale.
A particle extracted wrongly, lost or duplicated changes a count or moves a
sorted component by a whole cell.
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from pinc_amd import configs

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
WORKER = str(Path(__file__).resolve().parent / "switch_worker.py")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(ini, out, skip, sparse, world, steps):
    env = dict(os.environ, PINC_EXTRACT_SKIP=str(skip), PINC_FLAGS_SPARSE=str(sparse), PINC_QUIET="1",
               MASTER_ADDR="127.0.0.1")
    if world == 1:
        cmd = [sys.executable, WORKER, "--ini", ini, "--out", out, "--steps", str(steps)]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), WORKER, "--ini", ini, "--out", out,
               "--steps", str(steps)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    files = [out + ".npz"] if world == 1 else [f"{out}.r{k}.npz" for k in range(world)]
    return [dict(np.load(f)) for f in files]


@pytest.mark.parametrize("case", ["c5_one_rank", "c4_two_slabs"])
def test_extract_skip_and_sparse_flags_change_nothing(built, tmp_path, case):
    if case == "c5_one_rank":
        cfg = configs.bench_config("c5", size=32, ppc=8)
        cfg["objects"]["sphere"] = "16,16,16,5"        # (S/32 would be one cell)
        world, variants = 1, [(1, 1), (0, 0), (1, 0), (0, 1)]
    else:
        cfg = configs.bench_config("c4", size=64, ppc=4, world=2)
        world, variants = 2, [(1, 1), (0, 0)]
    steps = 6
    ini = configs.write_ini(cfg)
    try:
        runs = {v: _run(ini, str(tmp_path / f"run_{v[0]}{v[1]}"), *v, world, steps) for v in variants}
    finally:
        os.unlink(ini)
    base = runs[variants[0]]
    if case == "c5_one_rank":
        # the sphere collected particles (the push's sink flags: leavers)
        assert base[0]["collected"][0] != 0.0
    else:
        assert sum(r["emigrants"] for r in base).sum() > 0
    for v, other in runs.items():
        for r, (a, b) in enumerate(zip(base, other)):
            assert set(a) == set(b)
            what = f"{case} rank {r}, skip,sparse = {v} against {variants[0]}"
            np.testing.assert_array_equal(a["emigrants"], b["emigrants"], err_msg=what)
            np.testing.assert_array_equal(a["collected"], b["collected"], err_msg=what)
            np.testing.assert_allclose(a["energy"], b["energy"], rtol=1e-11, atol=0, err_msg=what)
            for k in a:
                if k.startswith(("pos", "vel")):
                    assert a[k].shape == b[k].shape, (what, k)
                    scale = max(np.max(np.abs(a[k])), 1e-300)
                    np.testing.assert_allclose(np.sort(a[k], axis=0), np.sort(b[k], axis=0), rtol=0,
                                               atol=1e-9 * scale, err_msg=f"{what}: {k}")
