"""Per-cycle cost of the native multigrid solve, replicated and sharded, on
one GPU (DESIGN.md section 7's 8-GPU prediction).

  python tools/mg_shard_probe.py --out f.json

Cases (native mode, 4 V-cycles per solve, 5 timed solves after 2 warm-up):
  rep256    256^3 replicated (what every rank runs without sharding)
  shard256  256^3 on one rank with shard = 1 (extended slab of 304 planes)
  ext80     256x256x32 on one rank with shard = 1: its level 0 is an
            extended slab of 80 planes, exactly the level-0 work of one rank
            of 8 at 256^3 (the coarse levels are those of a 256x256x32 grid)
  rep_l1    128^3 replicated: levels >= 1 of the 256^3 hierarchy
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def case(name, T, shard, cycles=4, solves=9, warm=3):
    from pinc_amd import Sim, configs
    cfg = configs.config("warm", true_size=T, nsub=(1, 1, 1), ppc=1, nalloc_pc=2, levels=3)
    cfg["multigrid"]["native"] = "1"
    cfg["multigrid"]["shard"] = shard
    ini = configs.write_ini(cfg)
    try:
        with Sim(ini, perturb=False) as s:
            rho = np.zeros([T[2] + 2, T[1] + 2, T[0] + 2])
            rho[1:-1, 1:-1, 1:-1] = np.random.default_rng(1).standard_normal((T[2], T[1], T[0]))
            s.mg_limit(cycles, cycles)
            zero = np.zeros_like(rho)
            ts = []
            for k in range(warm + solves):
                s.set_grid(0, rho)
                s.set_grid(1, zero)   # cold start: every solve runs the capped cycles
                s.sync()
                t0 = time.perf_counter()
                s.op("solve")
                s.sync()
                n = len(s.mg_history())
                if k >= warm:
                    ts.append((time.perf_counter() - t0) / n)
            r = {"case": name, "T": T, "halo": s.mg_shard, "levels": s.mg_levels,
                 "ms_per_cycle": 1e3 * float(np.median(ts)), "ms_per_cycle_each": [1e3 * t for t in ts]}
    finally:
        os.unlink(ini)
    print(json.dumps(r), flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--cases", default="rep256,shard256,ext80,rep_l1")
    a = ap.parse_args()
    table = {"rep256": ((256, 256, 256), "0"), "shard256": ((256, 256, 256), "1"),
             "ext80": ((256, 256, 32), "1"), "rep_l1": ((128, 128, 128), "0")}
    res = [case(c, *table[c]) for c in a.cases.split(",")]
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
