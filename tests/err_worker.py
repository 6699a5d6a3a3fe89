"""One error-path scenario of tests/test_gpu_errors.py, in its own process
(msg(ERROR) exits the process, as the reference's io.c:214-215 does).

    err_worker.py maxvel|frame  --layout reference|tiled --fused 0|1
    err_worker.py overflow      (under torch.distributed.run, 2 ranks, gloo)

Each scenario prints "REACHED-END" if the run did NOT stop.
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def _cfg(layout: str, fused: int, nsub=(1, 1, 1), true_size=(16, 16, 16)):
    from pinc_amd import configs
    cfg = configs.config("cold3d", true_size=true_size, nsub=nsub)
    cfg["multigrid"]["mgLevels"] = "3"
    cfg["population"]["fused"] = str(fused)
    if layout == "tiled":
        cfg["population"]["layout"] = "tiled"
        cfg["population"]["sortInterval"] = "2"
    return cfg


def single(kind: str, layout: str, fused: int) -> int:
    from pinc_amd import Sim, configs
    ini = configs.write_ini(_cfg(layout, fused))
    with Sim(ini) as s:
        s.init()
        s.step()
        pos, vel = s.particles(0)
        if kind == "maxvel":
            # pVelAssertMax (population.c:342-365): vel > maxVel (= 1), signed
            vel[7, 0] = 1.5
        else:
            # pPosAssertInLocalFrame (population.c:316-340): a particle that
            # crosses more than a subdomain ends outside the local frame
            # after the periodic shift; -20 passes the signed maxVel test
            pos[7, 2] = 1.5
            vel[7, 2] = -20.0
        s.set_particles(0, pos, vel)
        for _ in range(3):
            s.step()
    os.unlink(ini)
    print("REACHED-END", flush=True)
    return 0


def overflow() -> int:
    """Two z-slabs; population:nAlloc equals the initial count, so a rank has
    no room for a single net immigrant.  Every species-0 particle of rank 1
    leaves downwards while rank 0 keeps all of its own: rank 0's import must
    stop with msg(ERROR) (pinc_pusher.c, puMigrate), where the reference
    would write past iStart[s+1] (pusher.c:967-985 has no check)."""
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from pinc_amd import Sim, configs
    from pinc_amd.transport import GlooTransport
    cfg = _cfg("reference", 0, nsub=(1, 1, 2), true_size=(16, 16, 8))
    cfg["population"]["nAlloc"] = cfg["population"]["nParticles"]
    ini = configs.write_ini(cfg)
    tr = GlooTransport()
    with Sim(ini, rank=rank, nranks=world, device=0, transport=tr) as s:
        s.init()
        pos, vel = s.particles(0)
        vel[:] = 0.0
        if rank == 1:
            pos[:, 2] = 0.5
            vel[:, 2] = -0.9
        s.set_particles(0, pos, vel)
        for op in ("move", "extract", "migrate"):
            s.op(op)
    print("REACHED-END", flush=True)
    dist.destroy_process_group()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["maxvel", "frame", "overflow"])
    ap.add_argument("--layout", default="reference")
    ap.add_argument("--fused", type=int, default=1)
    a = ap.parse_args()
    if a.kind == "overflow":
        return overflow()
    return single(a.kind, a.layout, a.fused)


if __name__ == "__main__":
    sys.exit(main())
