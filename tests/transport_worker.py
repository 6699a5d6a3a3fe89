"""One rank of the CPU transport test (tests/test_transport_cpu.py): drives
pinc_amd.transport.GlooTransport through its C callback entry points exactly
as libpinc's pinc_comm.c calls them (z-slab neighbour exchange with paired
ops, allgather, allreduce) and checks the results."""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from pinc_amd.transport import GlooTransport
    r, P = dist.get_rank(), dist.get_world_size()
    t = GlooTransport()
    up, dn = (r + 1) % P, (r - 1 + P) % P
    # exchange: op 0 sends "up" to the upper slab and receives from the lower
    # one, op 1 the reverse (pinc_grid.c exchange_planes, pinc_pusher.c)
    n_up, n_dn = 3 + r, 5 + 2 * r            # ragged sizes, as migrant counts are
    s0 = np.full(n_up, 100.0 * r + 1)
    s1 = np.full(n_dn, 100.0 * r + 2)
    n_from_dn, n_from_up = 3 + dn, 5 + 2 * up
    r0 = np.zeros(n_from_dn)
    r1 = np.zeros(n_from_up)
    sp = (C.c_int * 2)(up, dn)
    rp = (C.c_int * 2)(dn, up)
    sb = (C.c_void_p * 2)(s0.ctypes.data, s1.ctypes.data)
    rb = (C.c_void_p * 2)(r0.ctypes.data, r1.ctypes.data)
    snb = (C.c_long * 2)(s0.nbytes, s1.nbytes)
    rnb = (C.c_long * 2)(r0.nbytes, r1.nbytes)
    assert t.struct.exchange(None, 2, sp, sb, snb, rp, rb, rnb) == 0
    assert np.all(r0 == 100.0 * dn + 1), (r, r0)
    assert np.all(r1 == 100.0 * up + 2), (r, r1)
    # all-to-all as the slab-distributed spectral solve drives it
    # (pinc_spectral.c all_to_all): op i sends block (r+i)%P to rank (r+i)%P
    # and receives block (r-i)%P from rank (r-i)%P, P-1 ops, tag i
    n = P - 1
    if n > 0:
        blk = 6
        src = np.concatenate([np.full(blk, 1000.0 * r + q) for q in range(P)])
        dst = np.zeros(blk * P)
        sp = (C.c_int * n)(*[(r + i) % P for i in range(1, P)])
        rp = (C.c_int * n)(*[(r - i + P) % P for i in range(1, P)])
        sb = (C.c_void_p * n)(*[src.ctypes.data + ((r + i) % P) * blk * 8 for i in range(1, P)])
        rb = (C.c_void_p * n)(*[dst.ctypes.data + ((r - i + P) % P) * blk * 8 for i in range(1, P)])
        nb = (C.c_long * n)(*([blk * 8] * n))
        assert t.struct.exchange(None, n, sp, sb, nb, rp, rb, nb) == 0
        dst[r * blk:(r + 1) * blk] = src[r * blk:(r + 1) * blk]
        # block p of dst is what rank p sent for this rank: value 1000 p + r
        assert np.array_equal(dst, np.concatenate([np.full(blk, 1000.0 * p + r) for p in range(P)])), (r, dst)
    # allgather of one slab per rank
    cnt = 4
    a = np.arange(cnt, dtype=np.float64) + 10.0 * r
    g = np.zeros(cnt * P)
    assert t.struct.allgather(None, a.ctypes.data, g.ctypes.data, cnt) == 0
    assert np.array_equal(g, np.concatenate([np.arange(cnt) + 10.0 * q for q in range(P)]))
    # allreduce
    v = np.array([1.0, float(r)])
    assert t.struct.allreduce_sum(None, v.ctypes.data, 2) == 0
    assert v[0] == P and v[1] == sum(range(P))
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {r} ok")
    return 0


if __name__ == "__main__":
    sys.exit(main())
