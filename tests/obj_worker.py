"""One rank of the two-slab object test (tests/test_gpu_objects.py, launched
through torch.distributed.run; gloo moves the data, every rank on cuda:0):
init with the object, `--steps` steps, rank-summed counts and energies."""
import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ini", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch  # noqa: F401  (HIP runtime before the native library)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from pinc_amd import Sim
    from pinc_amd.transport import GlooTransport
    tr = GlooTransport()
    res = {"energy": [], "counts": []}
    with Sim(args.ini, rank=rank, nranks=world, device=0, transport=tr) as s:
        s.init()
        for _ in range(args.steps):
            s.step()
            ke, pe, _ = s.energy()
            res["energy"].append([ke, pe])
            c = torch.tensor([s.count(0), s.count(1)], dtype=torch.int64)
            dist.all_reduce(c)
            res["counts"].append(c.tolist())
        res["mg_shard"] = s.mg_shard
    if rank == 0:
        Path(args.out).write_text(json.dumps(res))
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
