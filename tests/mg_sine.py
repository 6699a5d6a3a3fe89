"""The reference's own known-answer harness for the Poisson solve, restated.

TEST INFRASTRUCTURE.  The reference checks its
multigrid with a sine source whose continuous solution is known:

  * mgModeErrorScaling (multigrid.c:1734-1790) fills rho with
    gFillSin(rho, 1, mpiInfo, 0) -- a sine along x -- solves, takes E with
    gFinDiff1st (no gMul(E,-1)) and compares phi with gFillSinSol and E with
    gFillSinESol; script/framework/mgErrorScaling.py:28-60 doubles the grid
    and reads the order of the error from two successive runs;
  * mgMode (multigrid.c:1856-1900) does the same with a sine along z
    (gFillSin(rho, 3, ...)) after gNeutralizeGrid(rho).

The fill functions below restate grid.c:1563-1688 for one subdomain
(subdomain[d-1] = 0, nSubdomains[d-1] = 1, the halo filled periodically as
gHaloOp(setSlice, ..., TOHALO) does):

  gFillSin(norm=0)   rho_J = k^2 sin(kJ)          k = 2 pi / T_d
  gFillSin(norm=1)   rho_J = k   sin(kJ)
  gFillSinSol        phi_J = sin(kJ)
  gFillSinESol       E_J   = cos(kJ) on component d-1, 0 on the others

For the 7-point Laplacian the discrete problem has a closed form, because a
sine is an eigenvector: -L sin(kJ) = (2 - 2 cos k) sin(kJ).  So the solver's
answer is known exactly, not only up to discretisation error:

  phi_J = A sin(kJ),  A = c / (2 - 2 cos k)   (c = k^2 or k, per norm)
  gFinDiff1st:  0.5 (phi_{J+1} - phi_{J-1}) = A sin(k) cos(kJ)

and the discretisation error against gFillSinSol is (A - 1) sin(kJ) with
A - 1 = k^2/12 + O(k^4): a factor 4 per doubling of the grid, which is what
mgErrorScaling.py measures.  With norm = 1 the same holds for E against
gFillSinESol (A sin k = 1 - k^2/12 + ...); with norm = 0, as
mgModeErrorScaling itself calls it, phi ~ 1 and E ~ k cos(kJ), so the
reference's own E comparison there does not converge -- the norm argument of
gFillSin ("If it should be normalized to give E or phi correct",
grid.c:1581-1586) selects which of the two the run checks.

Layout: the reference layout with one ghost layer, [z+2][y+2][x+2] for a
scalar and [z+2][y+2][x+2][3] for E (value-major, grid.c:413-500).
"""
from __future__ import annotations

import math
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def _coord(size: int, d: int) -> tuple[np.ndarray, tuple[int, ...]]:
    """J along dimension d (1 = x, 2 = y, 3 = z) for every padded node
    (ghost 0 holds J = -1, ghost T+1 holds J = T: the periodic halo), and the
    broadcast shape of the [z][y][x] array."""
    J = np.arange(-1, size + 1, dtype=np.float64)
    shape = [1, 1, 1]
    shape[3 - d] = size + 2
    return J, tuple(shape)


def fill_sin(size: int, d: int, norm: int) -> np.ndarray:
    """gFillSin(grid, d, mpiInfo, norm), grid.c:1563-1608."""
    k = 2 * math.pi / size
    J, shp = _coord(size, d)
    c = k if norm else k * k
    col = np.array([c * math.sin(j * k) for j in J])   # the reference's loop, sin per node
    return np.broadcast_to(col.reshape(shp), (size + 2,) * 3).copy()


def fill_sin_sol(size: int, d: int) -> np.ndarray:
    """gFillSinSol(grid, d, mpiInfo), grid.c:1610-1645."""
    k = 2 * math.pi / size
    J, shp = _coord(size, d)
    col = np.array([math.sin(j * k) for j in J])
    return np.broadcast_to(col.reshape(shp), (size + 2,) * 3).copy()


def fill_sin_esol(size: int, d: int) -> np.ndarray:
    """gFillSinESol(grid, d, mpiInfo), grid.c:1647-1688: cos(kJ) in value
    d-1 of every node ((k+d-1)%3 == 0 over the value-major slice), 0 in the
    other two."""
    k = 2 * math.pi / size
    J, shp = _coord(size, d)
    col = np.array([math.cos(j * k) for j in J])
    out = np.zeros((size + 2,) * 3 + (3,))
    out[..., d - 1] = np.broadcast_to(col.reshape(shp), (size + 2,) * 3)
    return out


def closed_form(size: int, d: int, norm: int) -> tuple[np.ndarray, np.ndarray]:
    """The discrete solution of -L phi = gFillSin(norm) and its gFinDiff1st
    (no sign flip, as mgModeErrorScaling), on the true nodes [z][y][x] and
    [z][y][x][3]."""
    k = 2 * math.pi / size
    c = k if norm else k * k
    A = c / (2.0 - 2.0 * math.cos(k))
    J = np.arange(size, dtype=np.float64)
    shp = [1, 1, 1]
    shp[3 - d] = size
    phi = np.broadcast_to((A * np.sin(k * J)).reshape(shp), (size,) * 3)
    E = np.zeros((size,) * 3 + (3,))
    E[..., d - 1] = np.broadcast_to((A * math.sin(k) * np.cos(k * J)).reshape(shp), (size,) * 3)
    return phi, E


def ini_for(size: int, levels: int, *, native: bool = False, stack: bool = False, shard: str = "auto") -> str:
    """One 3-D subdomain of size^3 (the warm family's grid keys); native:
    the native V-cycle; stack: the bench's whole solver stack
    (configs.bench_config: native, extrapolated guess, FFT coarse solve,
    the bench's smoothing counts,
    multigrid:shard as given -- 'auto' is the bench's, which keeps one rank
    replicated; '1' runs the sharded level 0 with its deep halo on one
    rank)."""
    from pinc_amd import configs
    cfg = configs.config("warm", true_size=(size, size, size), nsub=(1, 1, 1), ppc=1, nalloc_pc=2, levels=levels)
    if native or stack:
        cfg["multigrid"]["native"] = "1"
    if stack:
        cfg["multigrid"]["shard"] = shard
        cfg["multigrid"]["extrapolate"] = "1"
        cfg["multigrid"]["spectralCoarse"] = "1"
        bench_mg = configs.bench_config("c4", size=size, ppc=1)["multigrid"]
        cfg["multigrid"]["nPreSmooth"] = bench_mg["nPreSmooth"]
        cfg["multigrid"]["nPostSmooth"] = bench_mg["nPostSmooth"]
    return configs.write_ini(cfg)


def levels_for(size: int) -> int:
    """The reference's level count where it fits (input files use 4-5), the
    coarsest grid at least 4^3."""
    return max(2, min(5, int(math.log2(size)) - 1))


def solve(side: str, size: int, d: int, norm: int, *, native: bool = False, stack: bool = False,
          shard: str = "auto", solves: int = 1, scale: float = 1.0) -> dict:
    """rho = gFillSin(d, norm) through the multigrid of `side` ('oracle' or
    'gpu'), then E as the run mode does.  Returns the true-node phi, E with
    mgModeErrorScaling's sign (gFinDiff1st without gMul(E,-1): the library's
    efield op applies main.c's gMul(E,-1), undone here), the residual
    history of every solve and the cycle counts.  scale multiplies the
    source (the problem is linear; phi and E are returned divided by it)."""
    rho = fill_sin(size, d, norm) * scale
    ini = ini_for(size, levels_for(size), native=native, stack=stack, shard=shard)
    hists = []
    shard_halo = 0
    try:
        if side == "oracle":
            sys.path.insert(0, str(ROOT / "oracle"))
            import orc
            w = orc.World(ini)
            w.mg_limit(0, 4000)
            for _ in range(solves):
                w.set_grid(0, rho)
                w.op("solve")
                hists.append(w.mg_history().tolist())
            w.op("efield")
            phi = w.grid(1)[1:-1, 1:-1, 1:-1, 0].copy()
            E = -w.grid(2)[1:-1, 1:-1, 1:-1].copy()
            w.close()
        else:
            from pinc_amd.sim import Sim
            s = Sim(ini, perturb=False)
            s.mg_limit(0, 4000)
            for _ in range(solves):
                s.set_grid(0, rho)
                s.op("solve")
                hists.append(s.mg_history().tolist())
            s.op("efield")
            phi = s.grid(1)[1:-1, 1:-1, 1:-1, 0].copy()
            E = -s.grid(2)[1:-1, 1:-1, 1:-1].copy()
            shard_halo = s.mg_shard
            s.close()
    finally:
        os.unlink(ini)
    return {"phi": phi / scale, "E": E / scale, "residual": [[x / scale for x in h] for h in hists],
            "shard_halo": shard_halo}


def errors(r: dict, size: int, d: int, norm: int) -> dict:
    """The run against the closed form (solver exactness) and against the
    reference's continuous solutions (discretisation error, RMS over the true
    nodes as mgErrorScaling.py's meanE2 along its line)."""
    phi_c, E_c = closed_form(size, d, norm)
    sol = fill_sin_sol(size, d)[1:-1, 1:-1, 1:-1]
    esol = fill_sin_esol(size, d)[1:-1, 1:-1, 1:-1]
    return {
        "phi_exact": float(np.max(np.abs(r["phi"] - phi_c)) / np.max(np.abs(phi_c))),
        "E_exact": float(np.max(np.abs(r["E"] - E_c)) / np.max(np.abs(E_c))),
        "phi_sol_rms": float(np.sqrt(np.mean((r["phi"] - sol) ** 2))),
        # the component along the sine (the other two are zero in both and
        # checked by E_exact)
        "E_sol_rms": float(np.sqrt(np.mean((r["E"][..., d - 1] - esol[..., d - 1]) ** 2))),
        "last_residual": float(r["residual"][-1][-1]) if r["residual"] and r["residual"][-1] else 0.0,
    }


def exact_bound(r: dict, size: int, norm: int) -> float:
    """What the solver's stop rule guarantees about exactness, relative to
    max|phi|: the solve ends once the RMS residual is <= 1e-10 (absolute,
    multigrid.c:1698), and the residual of a sine-mode error of amplitude e
    has RMS e (2 - 2cos k)/sqrt(2) (the sine is the Laplacian's eigenvector
    of that eigenvalue), so e <= sqrt(2) r / (2 - 2cos k).  Twice that, for
    the components the V-cycle leaves off the mode (round-off)."""
    k = 2 * math.pi / size
    lam = 2.0 - 2.0 * math.cos(k)
    A = (k if norm else k * k) / lam
    r_last = max(h[-1] for h in r["residual"] if h)
    return 2.0 * math.sqrt(2.0) * r_last / lam / A + 1e-13
