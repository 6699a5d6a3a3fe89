"""Immersed object on the device (pinc_obj.c, k_objects.hip; object.c,
config C5) against the checker (oracle/orc_obj.c), one subdomain.

Same init order on both sides: lattice + migrate, capacitance matrix (one
solve per surface node), removal of the particles that start inside
(charge dropped, main.c:163-166), initial fields, then main.c's loop with
collection, rho += rhoObj, solve, capacitance correction, solve.

Tolerances: particle counts and the removal order are bit-exact (integer
work, the emigrant back-fill); the capacitance columns come from two MG
runs that agree to solver tolerance, so fields and energies are compared
to 1e-7 relative.  Parity is against the corrected algorithm (the
reference's object.c does not compile; parity unpinned against it).
"""
import os

import numpy as np
import pytest

import orc
from pinc_amd import configs

pytestmark = pytest.mark.gpu


def _sphere(T, c, r):
    z, y, x = np.meshgrid(*[np.arange(t, dtype=float) for t in (T[2], T[1], T[0])], indexing="ij")
    return (((x - c[0]) ** 2 + (y - c[1]) ** 2 + (z - c[2]) ** 2) <= r * r).astype(float)


@pytest.mark.parametrize("T,sphere,layout,fused", [((16, 16, 16), (8.0, 8.0, 8.0, 2.5), "reference", 0),
                                                   ((32, 16, 16), (20.3, 7.6, 9.1, 3.2), "reference", 0),
                                                   ((32, 16, 16), (20.3, 7.6, 9.1, 3.2), "tiled", 0),
                                                   ((16, 16, 16), (8.0, 8.0, 8.0, 2.5), "reference", 1),
                                                   ((32, 16, 16), (20.3, 7.6, 9.1, 3.2), "tiled", 1),
                                                   ((32, 16, 16), (30.5, 7.6, 15.2, 3.2), "reference", 1)])
def test_object_steps_match_checker(built, T, sphere, layout, fused):
    """fused = 1: the push tests the particles that stay against the object
    and flags them for the next extract (PINC_NE_SINK), the flag pass runs
    on the immigrants only; removal order differs from the checker's two
    back-fills (extract, then collect), so particles compare as sets.  The
    third fused case puts the sphere across the periodic x and z boundaries
    (immigrants land in it)."""
    from pinc_amd import Sim
    cfg = configs.config("cold3d", true_size=T, nsub=(1, 1, 1))
    cfg["multigrid"]["mgLevels"] = "3"
    cfg["population"]["fused"] = "0"
    cfg["objects"] = {"sphere": ",".join(map(str, sphere))}
    ini = configs.write_ini(cfg)
    cfg["population"]["fused"] = str(fused)
    if layout == "tiled":
        cfg["population"]["layout"] = "tiled"
        cfg["population"]["sortInterval"] = "2"
    ini_dev = configs.write_ini(cfg)
    w = orc.World(ini)
    w.init()
    ob = orc.Objects(w, _sphere(T, sphere[:3], sphere[3]))
    ob.capacitance()
    ob.init_collect()
    w.init_fields()
    steps = 3
    with Sim(ini_dev) as s:
        s.init()
        for sp in range(2):
            assert s.count(sp) == w.count(sp)
        for k in range(steps):
            ob.step()
            s.step()
            ke_o, pe_o = w.energy()
            ke, pe, _ = s.energy()
            for sp in range(2):
                assert s.count(sp) == w.count(sp), (k, sp)
            assert abs(ke - ke_o) <= 1e-7 * abs(ke_o), (k, ke, ke_o)
            assert abs(pe - pe_o) <= 1e-7 * abs(pe_o), (k, pe, pe_o)
        for sp in range(2):
            pg, vg = s.particles(sp)
            po, vo, _ = w.particles(sp)
            if layout == "tiled" or fused:
                # sorted by tile: compare as sets (positions to 1e-9)
                def order(p, v):
                    k = np.lexsort(np.round(p * 1e6).T[::-1])
                    return p[k], v[k]
                pg, vg = order(pg, vg)
                po, vo = order(po, vo)
            assert np.max(np.abs(pg - po)) <= 1e-9
            assert np.max(np.abs(vg - vo)) <= 1e-9 * max(1.0, np.abs(vo).max())
        phi_g = s.grid(1)[1:-1, 1:-1, 1:-1]
        phi_o = w.grid(1)[1:-1, 1:-1, 1:-1]
        assert np.max(np.abs(phi_g - phi_o)) <= 1e-7 * np.abs(phi_o).max()
    # the object is charged: electrons fall in faster than ions
    assert ob.collected(0) != 0.0


def test_object_mask_file_equals_sphere(built, tmp_path):
    """objects:file (the reference's /Object dataset [nz, ny, nx, 1],
    object.c:727-756) gives the same run as the generated sphere."""
    from pinc_amd import Sim
    from pinc_amd._lib import HOST
    T, sphere = (16, 16, 16), (7.5, 8.2, 8.9, 3.1)
    mask = np.ascontiguousarray(_sphere(T, sphere[:3], sphere[3])[..., None])
    f = str(tmp_path / "obj.grid.h5")
    dims = np.array(mask.shape, dtype=np.int64)
    assert HOST.pinc_h5_write(f.encode(), b"/Object", 4, dims.ctypes.data, mask.ctypes.data) == 0
    res = []
    for key, val in (("sphere", ",".join(map(str, sphere))), ("file", f)):
        cfg = configs.config("cold3d", true_size=T, nsub=(1, 1, 1))
        cfg["multigrid"]["mgLevels"] = "3"
        cfg["population"]["fused"] = "0"
        cfg["objects"] = {key: val}
        with Sim(configs.write_ini(cfg)) as s:
            s.init()
            s.step(2)
            res.append((s.count(0), s.count(1), *s.energy()[:2]))
    # same removals; energies to the run-to-run spread of the atomic deposit
    assert res[0][:2] == res[1][:2]
    for a, b in zip(res[0][2:], res[1][2:]):
        assert abs(a - b) <= 1e-10 * abs(a)


@pytest.mark.parametrize("capacitance,fused,guess,world,shard", [
    ("solve", 0, None, 2, None), ("green", 0, None, 2, None), ("solve", 1, None, 2, None),
    ("solve", 1, "spectral", 2, None),
    # the sharded level 0 with an object: surface
    # potentials read from the owning slabs and summed over the ranks, the
    # spectral second guess slab-distributed
    ("solve", 1, "spectral", 2, "1"), ("solve", 1, "response", 2, "1"), ("green", 1, "spectral", 4, "1")])
def test_object_two_slabs_match_one(built, tmp_path, capacitance, fused, guess, world, shard):
    """Two (or four) z-slabs (host transport, one GPU): the object's lookups
    are global, charge corrections land in the owning slab and the collected
    charge is summed over the ranks; counts and energies match a one-rank
    run.  Replicated solve: phi is read from its global view.  shard = 1:
    the native multigrid's level 0 stays distributed,
    each rank reads the surface nodes of its slab and the potentials are
    summed over the ranks; the one-rank run it is compared with solves
    replicated.  green: the unit charge of the translated response sits on
    the rank holding global node (0,0,0) and the response is read from the
    potential (all-gathered once when sharded).  fused: the push collects the
    particles that stay, the flag pass the immigrants (the sphere straddles
    a slab boundary).  spectral: native multigrid with the extrapolated
    guesses and the spectral second guess (replicated: every rank transforms
    the gathered global rho; sharded: the slab-distributed transform of the
    owned planes)."""
    import json
    import os
    import socket
    import subprocess
    import sys
    from pathlib import Path
    from pinc_amd import Sim
    root = Path(__file__).resolve().parent.parent
    zb = 8 * world // 2
    sphere = f"8.2,7.7,{zb + 0.4},3.3"   # straddles the slab boundary at z = zb
    steps = 4 if guess else 3

    def cfg(nsub, T, shard_mode):
        c = configs.config("cold3d", true_size=T, nsub=nsub)
        c["multigrid"]["mgLevels"] = "3"
        c["population"]["fused"] = str(fused)
        c["objects"] = {"sphere": sphere, "capacitance": capacitance}
        if guess:
            c["multigrid"]["native"] = "1"
            c["multigrid"]["extrapolate"] = "1"
            c["objects"]["secondGuess"] = guess
        if shard_mode is not None:
            c["multigrid"]["shard"] = shard_mode
        return configs.write_ini(c)

    one = {"energy": [], "counts": []}
    with Sim(cfg((1, 1, 1), (16, 16, 8 * world), None)) as s:
        s.init()
        for _ in range(steps):
            s.step()
            ke, pe, _ = s.energy()
            one["energy"].append([ke, pe])
            one["counts"].append([s.count(0), s.count(1)])
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    out = tmp_path / "two.json"
    env = dict(os.environ, PYTHONPATH=str(root))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
                        "--master-addr=127.0.0.1", f"--master-port={port}", str(root / "tests" / "obj_worker.py"),
                        "--ini", cfg((1, 1, world), (16, 16, 8), shard), "--out", str(out), "--steps", str(steps)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    two = json.loads(out.read_text())
    if shard:
        assert two["mg_shard"] > 0
    assert two["counts"] == one["counts"]
    for a, b in zip(one["energy"], two["energy"]):
        assert abs(a[0] - b[0]) <= 1e-7 * abs(a[0]) and abs(a[1] - b[1]) <= 1e-7 * abs(a[1]), (a, b)


def test_two_objects_match_checker(built, tmp_path):
    """Two objects (mask values 1 and 2, from an objects:file mask): one
    capacitance matrix each, per-object charge collection and correction,
    against the checker's multi-object restatement."""
    from pinc_amd import Sim
    from pinc_amd._lib import HOST
    T = (32, 16, 16)
    mask = _sphere(T, (8.2, 7.9, 8.1), 2.6) + 2 * _sphere(T, (23.4, 8.3, 7.6), 3.1)
    assert mask.max() == 2
    f = str(tmp_path / "two.grid.h5")
    m4 = np.ascontiguousarray(mask[..., None])
    dims = np.array(m4.shape, dtype=np.int64)
    assert HOST.pinc_h5_write(f.encode(), b"/Object", 4, dims.ctypes.data, m4.ctypes.data) == 0
    cfg = configs.config("cold3d", true_size=T, nsub=(1, 1, 1))
    cfg["multigrid"]["mgLevels"] = "3"
    cfg["population"]["fused"] = "0"
    cfg["objects"] = {"file": f}
    ini = configs.write_ini(cfg)
    w = orc.World(ini)
    w.init()
    ob = orc.Objects(w, mask)
    assert ob.n == 2
    ob.capacitance()
    ob.init_collect()
    w.init_fields()
    with Sim(ini) as s:
        s.init()
        for k in range(3):
            ob.step()
            s.step()
            ke_o, pe_o = w.energy()
            ke, pe, _ = s.energy()
            for sp in range(2):
                assert s.count(sp) == w.count(sp), (k, sp)
            assert abs(ke - ke_o) <= 1e-7 * abs(ke_o), (k, ke, ke_o)
            assert abs(pe - pe_o) <= 1e-7 * abs(pe_o), (k, pe, pe_o)
        phi_g = s.grid(1)[1:-1, 1:-1, 1:-1]
        phi_o = w.grid(1)[1:-1, 1:-1, 1:-1]
        assert np.max(np.abs(phi_g - phi_o)) <= 1e-7 * np.abs(phi_o).max()
    assert ob.collected(0) != 0.0 and ob.collected(1) != 0.0


def test_green_capacitance_matches_solves(built):
    """objects:capacitance = green (one solve, columns by translation of the
    periodic response) gives the run of the reference's one-solve-per-node
    matrix, to the solver tolerance."""
    from pinc_amd import Sim
    res = []
    for mode in ("solve", "green"):
        cfg = configs.config("cold3d", true_size=(32, 16, 16), nsub=(1, 1, 1))
        cfg["multigrid"]["mgLevels"] = "3"
        cfg["population"]["fused"] = "0"
        cfg["objects"] = {"sphere": "20.3,7.6,9.1,3.2", "capacitance": mode}
        with Sim(configs.write_ini(cfg)) as s:
            s.init()
            s.step(3)
            res.append((s.count(0), s.count(1), *s.energy()[:2], s.grid(1)[1:-1, 1:-1, 1:-1].copy()))
    (a0, a1, ka, pa, fa), (b0, b1, kb, pb, fb) = res
    assert (a0, a1) == (b0, b1)
    assert abs(ka - kb) <= 1e-7 * abs(ka) and abs(pa - pb) <= 1e-7 * abs(pa)
    assert np.max(np.abs(fa - fb)) <= 1e-6 * np.abs(fa).max()


GOLD_MASKS = __import__("pathlib").Path(__file__).resolve().parent / "golden" / "masks"


@pytest.mark.parametrize("name", ["sphere.grid.h5", "test_boxbox.h5_backup"])
def test_reference_masks_match_checker(built, name):
    """The object masks that ship with the reference (all of them are
    committed unchanged under tests/golden/masks/; the single object and a
    two-object 32^3 file here, the checker's capacitance solves keep the
    rest out of the suite's time), read by objects:file as oReadH5 reads them
    (object.c:727-756: dataset /Object [nz, ny, nx, 1]): lookup tables,
    capacitance matrices, collection and corrections against the checker
    fed with the same mask, two steps."""
    from pinc_amd import Sim
    from pinc_amd.sim import h5_read
    f = str(GOLD_MASKS / name)
    mask = h5_read(f, "/Object")[..., 0]
    T = tuple(reversed(mask.shape))
    cfg = configs.config("cold3d", true_size=T, nsub=(1, 1, 1))
    cfg["multigrid"]["mgLevels"] = "3"
    # native multigrid on both sides (oracle/orc_native.c): the same object
    # operators with ~4 instead of ~20 V-cycles per capacitance column
    cfg["multigrid"]["native"] = "1"
    cfg["population"]["fused"] = "0"
    cfg["population"]["nParticles"] = "8 pc"
    cfg["population"]["nAlloc"] = "12 pc"
    cfg["objects"] = {"file": f}
    ini = configs.write_ini(cfg)
    w = orc.World(ini)
    w.init()
    ob = orc.Objects(w, mask)
    assert ob.n == int(mask.max())
    ob.capacitance()
    ob.init_collect()
    w.init_fields()
    with Sim(ini) as s:
        s.init()
        for sp in range(2):
            assert s.count(sp) == w.count(sp)
        for k in range(2):
            ob.step()
            s.step()
            ke_o, pe_o = w.energy()
            ke, pe, _ = s.energy()
            for sp in range(2):
                assert s.count(sp) == w.count(sp), (k, sp)
            assert abs(ke - ke_o) <= 1e-7 * abs(ke_o), (k, ke, ke_o)
            assert abs(pe - pe_o) <= 1e-7 * abs(pe_o), (k, pe, pe_o)
        phi_g = s.grid(1)[1:-1, 1:-1, 1:-1]
        phi_o = w.grid(1)[1:-1, 1:-1, 1:-1]
        assert np.max(np.abs(phi_g - phi_o)) <= 1e-7 * np.abs(phi_o).max()


@pytest.mark.parametrize("name", ["test_box64.h5_backup", "test_twobox.h5_backup"])
def test_reference_masks_64_green_equals_solve(built, name):
    """The 64^3 reference masks on the device: the capacitance matrix by one
    solve per surface node (the reference's method) and by translation
    (objects:capacitance = green) give the same run (counts exact, energies
    to the solver tolerance), and the particles inside the objects are gone."""
    from pinc_amd import Sim
    from pinc_amd.sim import h5_read
    f = str(GOLD_MASKS / name)
    mask = h5_read(f, "/Object")[..., 0]
    T = tuple(reversed(mask.shape))
    res = []
    for mode in ("solve", "green"):
        cfg = configs.config("cold3d", true_size=T, nsub=(1, 1, 1))
        cfg["multigrid"]["mgLevels"] = "4"
        cfg["multigrid"]["native"] = "1"   # ~4 V-cycles per capacitance column
        cfg["population"]["fused"] = "0"
        cfg["population"]["nParticles"] = "4 pc"
        cfg["population"]["nAlloc"] = "6 pc"
        cfg["objects"] = {"file": f, "capacitance": mode}
        with Sim(configs.write_ini(cfg)) as s:
            s.init()
            s.step(2)
            inside = 0
            for sp in range(2):
                p, _ = s.particles(sp)
                j = p.astype(np.int64) - 1   # lower node, true-node coordinates
                inside += int((mask[j[:, 2] % T[2], j[:, 1] % T[1], j[:, 0] % T[0]] > 0).sum())
            res.append((s.count(0), s.count(1), *s.energy()[:2], inside))
    (a0, a1, ka, pa, ia), (b0, b1, kb, pb, ib) = res
    assert (a0, a1) == (b0, b1)
    assert ia == 0 and ib == 0
    assert abs(ka - kb) <= 1e-7 * abs(ka) and abs(pa - pb) <= 1e-7 * abs(pa)


@pytest.mark.parametrize("fused,second", [(0, "response"), (1, "response"), (0, "spectral"), (1, "spectral")])
def test_object_extrapolated_guesses_match_checker(built, fused, second):
    """multigrid:extrapolate with an object (native mode, an extension;
    mgGuessNext): the first solve of each step starts
    from the first solutions of the last two steps, the second from this
    step's first solution plus the last step's correction response
    (objects:secondGuess = response) or plus the exact discrete response to
    this step's correction charge (= spectral: rocFFT with the 7-point
    symbol on the device, orc_discrete_poisson in the checker); the
    capacitance matrix's solves keep the warm start.  The checker restates
    the same guesses (oracle/orc_native.c): counts exact, energies and phi
    to 1e-7, V-cycles per step within 2."""
    from pinc_amd import Sim
    T, sphere = (32, 16, 16), (20.3, 7.6, 9.1, 3.2)
    cfg = configs.config("cold3d", true_size=T, nsub=(1, 1, 1))
    cfg["multigrid"]["mgLevels"] = "3"
    cfg["multigrid"]["native"] = "1"
    cfg["multigrid"]["extrapolate"] = "1"
    cfg["population"]["fused"] = "0"
    cfg["objects"] = {"sphere": ",".join(map(str, sphere)), "secondGuess": second}
    ini = configs.write_ini(cfg)
    cfg["population"]["fused"] = str(fused)
    ini_dev = configs.write_ini(cfg)
    w = orc.World(ini)
    w.init()
    ob = orc.Objects(w, _sphere(T, sphere[:3], sphere[3]))
    ob.capacitance()
    ob.init_collect()
    w.init_fields()
    with Sim(ini_dev) as s:
        s.init()
        for k in range(6):
            cs, co = s.cycles, w.cycles
            ob.step()
            s.step()
            assert abs((s.cycles - cs) - (w.cycles - co)) <= 2, (k, s.cycles - cs, w.cycles - co)
            ke_o, pe_o = w.energy()
            ke, pe, _ = s.energy()
            for sp in range(2):
                assert s.count(sp) == w.count(sp), (k, sp)
            assert abs(ke - ke_o) <= 1e-7 * abs(ke_o), (k, ke, ke_o)
            assert abs(pe - pe_o) <= 1e-7 * abs(pe_o), (k, pe, pe_o)
        phi_g = s.grid(1)[1:-1, 1:-1, 1:-1]
        phi_o = w.grid(1)[1:-1, 1:-1, 1:-1]
        assert np.max(np.abs(phi_g - phi_o)) <= 1e-7 * np.abs(phi_o).max()


def test_c5_bench_flags_match_checker(built):
    """Config C5 with the bench's exact flags (configs.bench_config("c5"):
    the sphere at the grid centre with radius S/32, fused collection in the
    push, tiled layout with the adaptive in-push sort, native multigrid with
    the extrapolated guesses, the exact level-1 solve and the spectral second
    guess, the capacitance matrix by one solve per surface node -- the
    reference's) at 64^3 x 16 ppc, 8 steps of main.c:197-274 against the
    checker's object loop (oracle/orc_obj.c with orc_native.c's guesses) on
    the same Maxwellian initial state: particle counts
    exact, KE/PE to 1e-7 (the tolerances above)."""
    from pinc_amd import Sim
    S, ppc, steps, seed = 64, 16, 8, 20260101
    cfg = configs.bench_config("c5", size=S, ppc=ppc)
    o = cfg["objects"]
    assert o["capacitance"] == "solve" and o["secondGuess"] == "spectral" and cfg["population"]["fused"] == "1"
    assert cfg["multigrid"]["extrapolate"] == "1" and cfg["multigrid"]["spectralCoarse"] == "1"
    sphere = [float(v) for v in o["sphere"].split(",")]
    ini = configs.write_ini(cfg)
    try:
        w = orc.World(ini)
        w.init(perturb=False, maxwell=True, seed=seed)
        ob = orc.Objects(w, _sphere((S, S, S), sphere[:3], sphere[3]))
        ob.capacitance()
        ob.init_collect()
        w.init_fields()
        with Sim(ini, maxwell=True, perturb=False, device_init=True, seed=seed) as s:
            s.init()
            for k in range(steps):
                ob.step()
                s.step()
                ke_o, pe_o = w.energy()
                ke, pe, _ = s.energy()
                print(f"step {k}: N {s.count(0)}+{s.count(1)} KE {ke:.13g}/{ke_o:.13g} PE {pe:.13g}/{pe_o:.13g}")
                for sp in range(2):
                    assert s.count(sp) == w.count(sp), (k, sp, s.count(sp), w.count(sp))
                assert abs(ke - ke_o) <= 1e-7 * abs(ke_o), (k, ke, ke_o)
                assert abs(pe - pe_o) <= 1e-7 * abs(pe_o), (k, pe, pe_o)
            collected = s.obj_collected
        assert collected != 0.0 and ob.collected(0) != 0.0
        w.close()
    finally:
        os.unlink(ini)
