"""The collectives of the multi-GPU bench, checked under RCCL's matching
rules.

RCCL refuses two ranks on one GPU, so the N>1 flow runs here as bench.py's
rehearsal (--host-transport: N processes share the GPU, the collectives go
through gloo).  Gloo matches point-to-point messages by tag and would pass a
pairing that RCCL -- which matches per peer in issue order and needs every
rank to issue the same collectives in the same order -- turns into a hang.
Every rank therefore records the sequence it issues (PINC_COMM_TRACE,
pinc_amd/host/pinc_comm.c), and tools/comm_pairing.py checks it: same
collectives in the same order with the same counts on every rank, and the
k-th send of a to b meeting the k-th receive of b from a with the same byte
count.  Workloads: C4 with the sharded level 0 (halo exchanges of the
extended slab, level-1 all-gather, 8-byte allreduces), C3's slab-distributed
spectral solve (all-to-all exchanges), C5 (objects: collection sums,
replicated solve), at 2 ranks (both z neighbours are the same rank) and 4.
The 8-rank run (the driver's N = 8 geometry) is in tools/gpu_rehearse.sh,
its check in profiles/.
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,workload,args", [
    (2, "c4", ["--size", "64", "--ppc", "4", "--mg-shard", "1"]),
    (2, "c3", ["--size", "64", "--ppc", "4"]),
    (2, "c5", ["--size", "64", "--ppc", "4"]),
    (4, "c4", ["--size", "128", "--ppc", "2", "--mg-shard", "1"]),
])
def test_rehearsal_collectives_pair_under_rccl_rules(built, tmp_path, world, workload, args):
    import json
    import comm_pairing
    env = dict(os.environ, PINC_COMM_TRACE=str(tmp_path), PINC_QUIET="1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "bench.py"), "--gpus", str(world),
           "--workload", workload, "--steps", "2", "--warmup", "1", "--host-transport", "--no-cpu-baseline", *args]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=str(ROOT))
    assert p.returncode == 0, p.stdout[-1500:] + p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world
    traces = comm_pairing.load(tmp_path)
    errs, stats = comm_pairing.check(traces, world)
    assert errs == [], errs
    kinds = {k for k, _ in stats}
    assert "X" in kinds and "R" in kinds
    if workload == "c4":
        assert ("X", "ext halo") in stats  # the sharded level 0 ran
    if workload == "c3":
        # the slab-distributed solve's all-to-all transposes, not an all-gather of rho
        assert ("X", "spectral transpose") in stats and not any(k == "G" for k, _ in stats), stats
    # the N>1 bench line says where the time went:
    # per-phase max/min over the ranks, every collective kind's time, bytes
    # and calls per step, and each rank's roofline of the dominant kernel
    mr = line["multi_rank"]
    assert mr["ranks"] == world and mr["transport"].startswith("host")
    for k in ("move", "extract", "migrate", "deposit", "solve", "efield", "accelerate", "energy"):
        assert k in mr["phase_ms_per_step_max"] and k in mr["phase_ms_per_step_min"]
        assert mr["phase_ms_per_step_max"][k] >= mr["phase_ms_per_step_min"][k]
    comm = mr["comm_per_step"]
    assert set(comm) == {"halo", "ext_halo", "migrate", "allgather", "allreduce", "spectral_transpose"}
    for v in comm.values():
        assert set(v) == {"ms_per_step_max", "ms_per_step_mean", "bytes_per_step_per_rank_max", "calls_per_step"}
    assert comm["migrate"]["calls_per_step"] >= 2 and comm["migrate"]["bytes_per_step_per_rank_max"] > 0
    assert comm["halo"]["calls_per_step"] >= 1 and comm["allreduce"]["calls_per_step"] > 0
    if workload == "c4":
        assert comm["ext_halo"]["calls_per_step"] > 0 and comm["ext_halo"]["ms_per_step_max"] > 0
    if workload == "c3":
        assert comm["spectral_transpose"]["calls_per_step"] > 0
    assert mr["comm_ms_per_step_max_total"] > 0
    assert len(mr["per_rank"]) == world
    for r in mr["per_rank"]:
        assert r["particles"] > 0 and r["roofline"]["achieved_GBs"] > 0 and r["roofline"]["kernel"] == \
            line["roofline"]["kernel"]
