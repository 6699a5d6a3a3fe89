"""One rank of the sharded-multigrid parity test (tests/test_gpu_mg_shard.py),
launched through torch.distributed.run; gloo moves the data (host transport),
every rank on cuda:0.

The global charge density of tests/mg_history.py is cut into this rank's
z-slab, solved `--solves` times (native mode, multigrid:shard = 1), and the
per-cycle residual history of every solve plus this rank's potential are
saved for the test to compare with the oracle's two-rank emulation.
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, required=True)
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--cycles", type=int, default=60)
    ap.add_argument("--solves", type=int, default=2)
    ap.add_argument("--seed", type=int, default=20261016)
    ap.add_argument("--out", required=True)
    ap.add_argument("--spectral", action="store_true", help="sSolver (slab-distributed) instead of the multigrid")
    ap.add_argument("--spectral-coarse", action="store_true",
                    help="multigrid:spectralCoarse (level 1 solved exactly; decomposed with the sharded level 0)")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch.distributed as dist
    dist.init_process_group("gloo")
    import mg_history
    from pinc_amd import Sim
    from pinc_amd.transport import GlooTransport
    ini = mg_history.ini_for(args.size, args.levels, True, nranks=world, shard="1", spectral=args.spectral,
                             spectral_coarse=args.spectral_coarse)
    from pinc_amd import _lib
    rho = mg_history.rank_slab(mg_history.make_rho(args.size, args.seed, 1.0), rank, world)
    out = {}
    try:
        with Sim(ini, rank=rank, nranks=world, device=0, transport=GlooTransport(), perturb=False) as s:
            if args.spectral:
                out["distributed"] = np.array(s.spectral_distributed)
            else:
                s.mg_limit(args.cycles, args.cycles)
                out["halo"] = np.array(s.mg_shard)
            _lib.comm_stats_start(1 << 12)
            for k in range(args.solves):
                s.set_grid(0, rho)
                s.op("solve")
                if not args.spectral:
                    out[f"hist{k}"] = s.mg_history()
            # collectives of the solves: calls and payload bytes per kind
            for kind, c in _lib.comm_stats_read().items():
                out[f"comm_{kind}"] = np.array([c["calls"], c["bytes"]])
            out["phi"] = s.grid(1)[..., 0].copy()
            s.op("efield")
            out["E"] = s.grid(2).copy()
    finally:
        os.unlink(ini)
    np.savez(f"{args.out}_r{rank}.npz", **out)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
