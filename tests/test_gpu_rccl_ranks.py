"""Several ranks over RCCL on several GPUs, against the same ranks over the
host transport (the sharded level-0 multigrid and the
slab-distributed spectral solve had only run through gloo).

RCCL refuses two ranks on one device, so this runs only where the process
sees at least two GPUs (an 8-GPU node); on the one-GPU test box it is
skipped, and the same multi-rank flow is covered by test_gpu_multirank.py,
test_gpu_mg_shard.py and the comm-pairing rehearsal over the host transport.

The bench's own N-rank flow runs twice on the same small C4-shaped problem:
once with the library's RCCL communicator (one GPU per rank, the measured
configuration) and once with every rank on GPU 0 and the collectives
through gloo.  Only the transport differs, so the energies, the particle
count and the V-cycles must agree.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent

pytestmark = pytest.mark.gpu


def _ngpus() -> int:
    try:
        import torch
        return torch.cuda.device_count()  # does not initialise the GPU
    except Exception:  # noqa: BLE001
        return 0


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(n: int, args: list[str], host: bool) -> dict:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"), "--gpus", str(n),
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline", *args]
    if host:
        cmd.append("--host-transport")
    env = dict(os.environ, PINC_QUIET="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("n,args", [
    (2, ["--size", "64", "--ppc", "8"]),
    (2, ["--workload", "c3", "--size", "64", "--ppc", "8"]),
    (4, ["--size", "64", "--ppc", "8", "--mg-shard", "1"]),
    (2, ["--workload", "c5", "--size", "64", "--ppc", "8"]),
], ids=["c4-2", "c3-spectral-2", "c4-shard-4", "c5-2"])
def test_rccl_ranks_match_host_transport(n, args):
    if _ngpus() < n:
        pytest.skip(f"needs {n} GPUs (RCCL refuses two ranks on one device)")
    rc = _bench(n, args, host=False)
    hc = _bench(n, args, host=True)
    assert rc["n_gpus"] == hc["n_gpus"] == n
    assert rc["config"]["particles"] == hc["config"]["particles"]
    for q in ("KE", "PE"):
        a, b = rc["energy"][q], hc["energy"][q]
        assert abs(a - b) <= 1e-9 * abs(b), (q, a, b)
    if "mg_cycles_per_solve" in rc:
        assert abs(rc["mg_cycles_per_solve"] - hc["mg_cycles_per_solve"]) <= 1e-9
