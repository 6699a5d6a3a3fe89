"""The multi-rank collectives' host transport on CPU with gloo, world sizes
2 and 3 (P = 2 is the case where both z neighbours are the same rank)."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3, 4])
def test_gloo_transport(world):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "tests" / "transport_worker.py")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    assert p.stdout.count(" ok") == world


def _write_traces(d, lines_by_rank):
    for r, lines in lines_by_rank.items():
        (d / f"comm_rank{r}.log").write_text("\n".join(lines) + "\n")


def test_comm_pairing_checker(tmp_path):
    """tools/comm_pairing.py applies RCCL's matching (per ordered pair, in
    issue order) to a recorded sequence.  At two ranks both z neighbours are
    the same rank: the halo's "up" send must meet the peer's "from below"
    receive because it is posted first, not because of a tag."""
    sys.path.insert(0, str(ROOT / "tools"))
    import comm_pairing as cp
    good = {0: ["X 0 halo exchange|2 s1:100 r1:100 s1:200 r1:200", "R 1 norm|1"],
            1: ["X 0 halo exchange|2 s0:100 r0:100 s0:200 r0:200", "R 1 norm|1"]}
    _write_traces(tmp_path, good)
    errs, stats = cp.check(cp.load(tmp_path), 2)
    assert errs == [] and stats[("R", "norm")] == 1
    # rank 1 posts its receives in the other order: a tag-matched transport
    # pairs them, RCCL would hand rank 0's 100-byte send to a 200-byte receive
    bad = {0: good[0], 1: ["X 0 halo exchange|2 s0:100 r0:200 s0:200 r0:100", "R 1 norm|1"]}
    _write_traces(tmp_path, bad)
    errs, _ = cp.check(cp.load(tmp_path), 2)
    assert errs and "sends [100, 200] B to rank 1" in errs[0]
    # a rank that skips a collective
    skip = {0: good[0], 1: ["R 1 norm|1"]}
    _write_traces(tmp_path, skip)
    errs, _ = cp.check(cp.load(tmp_path), 2)
    assert errs and "different numbers" in errs[0]
