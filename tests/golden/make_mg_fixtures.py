#!/usr/bin/env python3
"""Generate tests/golden/mg_history/*.json: the oracle's multigrid residual
histories at the configs' grids, so that the GPU tests compare against
committed numbers instead of re-running the CPU oracle on the GPU box.

TEST INFRASTRUCTURE.  Each fixture is one solve of tests/mg_history.py's
charge density (numpy default_rng(seed) standard normal per true node,
SHA-256 recorded) by the oracle (oracle/orc_mg.c: the reference's
mgVRecursive / mgSolveRaw, multigrid.c:1496-1556, 1688-1724; or
oracle/orc_native.c for native mode): the RMS residual after every V-cycle,
the maximum of the final phi and phi on every k-th node per dimension
(k = size / 16: 4096 values).

    python tests/golden/make_mg_fixtures.py            # the fast fixtures (~2 min on 8 threads)
    python tests/golden/make_mg_fixtures.py --long     # + parity mode at 256^3 for 3000 cycles (~100 min)

Without --long the 3000-cycle 256^3 fixture is taken from the oracle run
recorded in profiles/r02_mg_history.json (made by tests/mg_history.py, same
density), if that file is present.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))
SEED, AMP = 20261016, 1.0
CASES = {
    # name: size, levels, cycle cap, native
    "parity_128": (128, 5, 3000, False),
    "parity_256_40": (256, 5, 40, False),
    "native_128": (128, 5, 200, True),
    "native_256": (256, 5, 200, True),
}


def fixture(r: dict, phi: np.ndarray) -> dict:
    k = max(1, r["size"] // 16)
    return {k2: r[k2] for k2 in ("size", "levels", "native", "cycle_cap", "seed", "amp", "rho_sha256")} | {
        "residual": r["residual"][-1], "phi_max": float(np.max(np.abs(phi))), "phi_stride": k,
        "phi_sub": np.ascontiguousarray(phi[::k, ::k, ::k]).ravel().tolist(),
        "generator": "tests/golden/make_mg_fixtures.py (oracle)"}


def main() -> int:
    import mg_history
    ap = argparse.ArgumentParser()
    ap.add_argument("--long", action="store_true")
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    out = HERE / "mg_history"
    out.mkdir(exist_ok=True)
    import orc
    orc.LIB.orc_set_threads(8)
    cases = dict(CASES)
    if a.long:
        cases["parity_256_3000"] = (256, 5, 3000, False)
    for name, (size, levels, cap, native) in cases.items():
        if a.only and name != a.only:
            continue
        r = mg_history.run("oracle", size, levels, cap, SEED, AMP, native=native)
        phi = r.pop("phi")
        (out / f"{name}.json").write_text(json.dumps(fixture(r, phi)))
        print(f"{name}: {len(r['residual'][-1])} cycles, {r['seconds']:.1f} s", flush=True)
    prof = ROOT / "profiles" / "r02_mg_history.json"
    if not a.long and prof.exists() and (a.only in (None, "parity_256_3000")):
        run = json.loads(prof.read_text())["runs"]["parity_256_oracle"]
        f = {k2: run[k2] for k2 in ("size", "levels", "native", "cycle_cap", "seed", "amp", "rho_sha256")}
        f |= {"residual": run["residual"][-1], "phi_sample_z": run.get("phi_sample"),
              "generator": "tests/mg_history.py --side oracle --size 256 --levels 5 --cycles 3000 "
                           "(recorded in profiles/r02_mg_history.json; --long regenerates it)"}
        (out / "parity_256_3000.json").write_text(json.dumps(f))
        print("parity_256_3000: from", prof.name)
    return 0


if __name__ == "__main__":
    sys.exit(main())
