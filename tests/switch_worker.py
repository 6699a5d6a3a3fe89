"""One run of the flag/extraction switch test (tests/test_gpu_flag_switches.py):
the switches come from the environment (PINC_EXTRACT_SKIP, PINC_FLAGS_SPARSE,
read when the library's context is created), `--steps` steps from a seeded
device initialisation; every step's emigrant counts and energies, and the
final particles of this rank, go to `--out` (.npz; rank r adds .r<r>).
With WORLD_SIZE > 1 (torch.distributed.run) the ranks share cuda:0 over the
gloo host transport."""
import argparse
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ini", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (HIP runtime before the native library)
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    tr = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from pinc_amd.transport import GlooTransport
        tr = GlooTransport()
    from pinc_amd import Sim
    em, en = [], []
    with Sim(args.ini, rank=rank, nranks=world, device=0, transport=tr, maxwell=True, perturb=False,
             device_init=True, seed=20260101) as s:
        s.init()
        for _ in range(args.steps):
            s.step()
            em.append(s.emigrants())
            ke, pe, _ = s.energy()
            en.append([ke, pe])
        parts = {"collected": np.array([s.obj_collected])}
        for sp in range(s.nspecies):
            p, v = s.particles(sp)
            parts[f"pos{sp}"] = p
            parts[f"vel{sp}"] = v
    out = args.out + (f".r{rank}" if world > 1 else "")
    np.savez(out, emigrants=np.array(em), energy=np.array(en), **parts)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
