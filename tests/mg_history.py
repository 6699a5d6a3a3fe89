#!/usr/bin/env python3
"""Multigrid residual history of one solve on a fixed charge density.

TEST INFRASTRUCTURE: the same rho goes through the
oracle's restatement of mgSolveRaw/mgVRecursive (multigrid.c:1496-1556,
1688-1724; oracle/orc_mg.c) and through the device solver in parity mode
(pinc_amd/host/pinc_mg.c), and the RMS residual after every V-cycle is
recorded on both sides.

    python tests/mg_history.py --side oracle --size 128 --levels 5 --cycles 200 --out f.json
    python tests/mg_history.py --side gpu    --size 256 --levels 5 --cycles 2000 --out g.json

rho: the C4 plasma's charge fluctuation, emulated as independent normal
values per true node (numpy default_rng(seed), standard normal x amp), the
same array on both sides (its SHA-256 is recorded).  phi and every coarse
level start from zero on both sides (the reference's malloc'd grids read as
zero on fresh pages).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def make_rho(size: int, seed: int, amp: float) -> np.ndarray:
    """Reference layout [z+2][y+2][x+2] (one ghost layer, value-major with
    one value) with the noise on the true nodes and zero ghosts."""
    g = np.random.default_rng(seed).standard_normal((size, size, size)) * amp
    out = np.zeros((size + 2, size + 2, size + 2))
    out[1:-1, 1:-1, 1:-1] = g
    return out


def ini_for(size: int, levels: int, native: bool, nranks: int = 1, shard: str | None = None,
            spectral: bool = False, spectral_coarse: bool = False) -> str:
    from pinc_amd import configs
    cfg = configs.config("warm", true_size=(size, size, size // nranks), nsub=(1, 1, nranks), ppc=1, nalloc_pc=2,
                         levels=levels)
    if native:
        cfg["multigrid"]["native"] = "1"
    if shard is not None:
        cfg["multigrid"]["shard"] = shard
    if spectral:
        cfg["methods"]["poisson"] = "sSolver"
    if spectral_coarse:
        cfg["multigrid"]["spectralCoarse"] = "1"
    return configs.write_ini(cfg)


def rank_slab(rho: np.ndarray, rank: int, nranks: int) -> np.ndarray:
    """This rank's planes of a reference-layout global grid (ghost planes are
    the neighbours' planes; the solvers read true nodes only)."""
    nloc = (rho.shape[0] - 2) // nranks
    return np.ascontiguousarray(rho[rank * nloc: rank * nloc + nloc + 2])


def run(side: str, size: int, levels: int, cycles: int, seed: int, amp: float, native: bool = False,
        solves: int = 1, shard: str | None = None, spectral_coarse: bool = False) -> dict:
    rho = make_rho(size, seed, amp)
    digest = hashlib.sha256(rho.tobytes()).hexdigest()
    ini = ini_for(size, levels, native, shard=shard, spectral_coarse=spectral_coarse)
    halo = 0
    t0 = time.perf_counter()
    hists = []
    try:
        if side == "oracle":
            sys.path.insert(0, str(ROOT / "oracle"))
            import orc
            w = orc.World(ini)
            w.mg_limit(cycles, cycles)
            for _ in range(solves):
                w.set_grid(0, rho)
                w.op("solve")
                hists.append(w.mg_history().tolist())
            phi = w.grid(1)[1:-1, 1:-1, 1:-1].copy()
            w.close()
        else:
            from pinc_amd.sim import Sim
            s = Sim(ini, perturb=False)
            s.mg_limit(cycles, cycles)
            for _ in range(solves):
                s.set_grid(0, rho)
                s.op("solve")
                hists.append(s.mg_history().tolist())
            phi = s.grid(1)[1:-1, 1:-1, 1:-1].copy()
            halo = s.mg_shard
            s.close()
    finally:
        os.unlink(ini)
    return {"side": side, "size": size, "levels": levels, "native": native, "cycle_cap": cycles, "seed": seed,
            "amp": amp, "shard_halo": halo, "rho_sha256": digest, "seconds": time.perf_counter() - t0, "residual": hists,
            "phi_rms": float(np.sqrt(np.mean(phi ** 2))), "phi_sample": phi[::max(1, size // 8), 3, 5].tolist(),
            "phi": phi}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", choices=["oracle", "gpu"], required=True)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--cycles", type=int, default=200)
    ap.add_argument("--seed", type=int, default=20261016)
    ap.add_argument("--amp", type=float, default=1.0)
    ap.add_argument("--native", action="store_true")
    ap.add_argument("--solves", type=int, default=1)
    ap.add_argument("--out", required=True)
    ap.add_argument("--phi-out", default=None, help="also save the final phi (.npy)")
    ap.add_argument("--phi-stride", type=int, default=1, help="save every n-th node per dimension")
    a = ap.parse_args()
    r = run(a.side, a.size, a.levels, a.cycles, a.seed, a.amp, a.native, a.solves)
    phi = r.pop("phi")
    if a.phi_out:
        k = a.phi_stride
        np.save(a.phi_out, np.ascontiguousarray(phi[::k, ::k, ::k]))
    Path(a.out).write_text(json.dumps(r))
    h = r["residual"][-1]
    print(f"{a.side} {a.size}^3 L={a.levels}: {len(h)} cycles in {r['seconds']:.1f} s, "
          f"first {h[0]:.3e} last {h[-1]:.3e} min {min(h):.3e}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
