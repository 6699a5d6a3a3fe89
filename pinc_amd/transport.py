"""Host transport for the multi-rank collectives over torch.distributed.

The production path moves device buffers with RCCL over xGMI.  RCCL refuses
two ranks on one GPU, so multi-rank correctness on a single-GPU box (and the
collective logic on CPU) is exercised through this transport instead: the
host library stages device data through host memory and calls back into
Python, which moves it with a torch.distributed process group (gloo).
See pinc_set_host_transport in include/pinc.h.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

EXCHANGE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_void_p),
                       C.POINTER(C.c_long), C.POINTER(C.c_int), C.POINTER(C.c_void_p), C.POINTER(C.c_long))
ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_long)
ALLREDUCE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_long)


class HostTransportStruct(C.Structure):
    _fields_ = [("exchange", EXCHANGE), ("allgather", ALLGATHER), ("allreduce_sum", ALLREDUCE),
                ("user", C.c_void_p)]


def _u8(ptr: int, n: int):
    import torch
    return torch.from_numpy(np.ctypeslib.as_array((C.c_ubyte * n).from_address(ptr)))


def _f64(ptr: int, n: int):
    import torch
    return torch.from_numpy(np.ctypeslib.as_array((C.c_double * n).from_address(ptr)))


class GlooTransport:
    """Collectives of the hot path over the default torch.distributed group.

    exchange op i sends to sendPeer[i] with tag i and receives from
    recvPeer[i] with tag i, so a peer's send op i meets this rank's receive
    op i even when both neighbours are the same rank (P = 2)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self._exchange = EXCHANGE(self.exchange)
        self._allgather = ALLGATHER(self.allgather)
        self._allreduce = ALLREDUCE(self.allreduce_sum)
        self.struct = HostTransportStruct(self._exchange, self._allgather, self._allreduce, None)

    def exchange(self, user, n_ops, send_peer, send_buf, send_bytes, recv_peer, recv_buf, recv_bytes):
        try:
            reqs = []
            for i in range(n_ops):
                if send_bytes[i] > 0:
                    reqs.append(self.dist.isend(_u8(send_buf[i], send_bytes[i]), send_peer[i], group=self.group,
                                                tag=i))
                if recv_bytes[i] > 0:
                    reqs.append(self.dist.irecv(_u8(recv_buf[i], recv_bytes[i]), recv_peer[i], group=self.group,
                                                tag=i))
            for r in reqs:
                r.wait()
            return 0
        except Exception as e:  # an exception must not cross the C boundary
            print(f"[transport rank {self.rank}] exchange failed: {e!r}")
            return 1

    def allgather(self, user, send, recv, count):
        try:
            s = _f64(send, count)
            r = _f64(recv, count * self.size)
            self.dist.all_gather([r[i * count:(i + 1) * count] for i in range(self.size)], s, group=self.group)
            return 0
        except Exception as e:
            print(f"[transport rank {self.rank}] allgather failed: {e!r}")
            return 1

    def allreduce_sum(self, user, buf, count):
        try:
            self.dist.all_reduce(_f64(buf, count), op=self.dist.ReduceOp.SUM, group=self.group)
            return 0
        except Exception as e:
            print(f"[transport rank {self.rank}] allreduce failed: {e!r}")
            return 1
