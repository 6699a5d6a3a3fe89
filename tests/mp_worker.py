"""One rank of a multi-rank parity run (launched by tests/test_gpu_multirank.py
through torch.distributed.run; gloo moves the data, every rank on cuda:0).

Loads the oracle's initial particles for this rank, runs move + extract +
migrate and saves the particles, then runs the rest of that step and
`--steps` more, saving the rank-summed energies.
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ini", required=True)
    ap.add_argument("--state", required=True, help="prefix of the oracle state files")
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--maxwell", action="store_true")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from pinc_amd import Sim
    from pinc_amd.transport import GlooTransport
    tr = GlooTransport()
    res = {"rank": rank}
    with Sim(args.ini, rank=rank, nranks=world, device=0, transport=tr, perturb=not args.maxwell,
             maxwell=args.maxwell, seed=5) as s:
        s.init()
        st = np.load(f"{args.state}_r{rank}.npz")
        for sp in range(s.nspecies):
            s.set_particles(sp, st[f"pos{sp}"], st[f"vel{sp}"])
        for op in ("move", "extract", "migrate"):
            s.op(op)
        out = {}
        for sp in range(s.nspecies):
            out[f"pos{sp}"], out[f"vel{sp}"] = s.particles(sp)
        out["emigrants"] = s.emigrants()
        np.savez(f"{args.out}_r{rank}.npz", **out)
        for op in ("distr", "solve", "efield", "acc"):
            s.op(op)
        ke, pe, _ = s.energy()
        res["energy"] = [[ke, pe]]
        for _ in range(args.steps):
            s.step()
            ke, pe, _ = s.energy()
            res["energy"].append([ke, pe])
        res["counts"] = [s.count(sp) for sp in range(s.nspecies)]
    Path(f"{args.out}_r{rank}.json").write_text(json.dumps(res))
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
