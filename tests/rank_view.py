"""A G-rank view of a real one-rank process group (test infrastructure).

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so the one-GPU test box cannot run a
G >= 2 RCCL communicator.  RankView(dist, G, r) lets the element-partitioned code take its G >= 2 branches
(interface exchange, strip all-gather of the reduced blocks, capture agreement) as rank r of G while every
collective it issues is a REAL RCCL call on the one-rank group -- launched on the RCCL stream, waited on
through the backend's work handles, captured into hipGraphs.  The values from the G - 1 absent ranks are
stand-ins: a sum over one rank is the local tensor, an all-gather fills the absent slots with copies of the
local tensor (4-D reduced-system blocks with a boosted diagonal, so the stand-in reduced system stays
regular).  Only rank-independent properties are checkable under it: graph replay against eager execution,
the capture decisions, the collective counts.  Correctness across ranks is covered by the gloo tests.
"""
import torch


class RankView:
    def __init__(self, dist, G, r):
        self._d, self.G, self.r = dist, G, r
        self.calls = {}

    def __getattr__(self, name):       # ReduceOp, P2POp, ... come from torch.distributed
        return getattr(self._d, name)

    def _count(self, k):
        self.calls[k] = self.calls.get(k, 0) + 1

    def get_world_size(self, group=None):
        return self.G

    def get_rank(self, group=None):
        return self.r

    def get_backend(self, group=None):
        return self._d.get_backend()

    def get_global_rank(self, group, r):
        return r

    def all_reduce(self, t, op=None, group=None, async_op=False):
        self._count("all_reduce")
        kw = {} if op is None else {"op": op}
        return self._d.all_reduce(t, async_op=async_op, **kw)

    def all_gather(self, out, t, group=None, async_op=False):
        self._count("all_gather")
        work = self._d.all_gather([out[self.r]], t, async_op=async_op)
        for j, o in enumerate(out):
            if j == self.r:
                continue
            o.copy_(t)
            if t.dim() == 4:   # a reduced-system block pair (2, 2, m, m) of an absent strip: keep it regular
                eye = torch.eye(t.shape[-1], dtype=t.dtype, device=t.device) * t.abs().max()
                o[0, 0] += eye
                o[1, 1] += eye
        return work

    def broadcast(self, t, src=0, group=None, async_op=False):
        self._count("broadcast")
        return self._d.broadcast(t, src=0, async_op=async_op)

    def barrier(self, group=None):
        self._count("barrier")
        return self._d.barrier()
