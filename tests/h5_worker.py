"""One rank of the multi-rank output test (tests/test_h5_output.py,
launched through torch.distributed.run; gloo moves the data, every rank on
cuda:0): init, one step, main.c's output for step 1 under --out."""
import argparse
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ini", required=True)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch  # noqa: F401  (HIP runtime before the native library)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from pinc_amd import Sim
    from pinc_amd.transport import GlooTransport
    tr = GlooTransport()
    with Sim(args.ini, rank=rank, nranks=world, device=0, transport=tr) as s:
        s.init()
        s.step()
        s.write_output(1)
        s.sync()
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
