"""Host-staged stand-in for RCCL, for running slab.Comm's RCCL code paths with several ranks on ONE
GPU (RCCL refuses two ranks on one device).  TEST INFRASTRUCTURE ONLY.

``StagedTransportComm`` is a ``slab.Comm`` whose ``stage`` flag is False -- so every branch the
driver's multi-GPU run takes executes as it does there: device all-gathers into device buffers, the
pinned-memory ``read_async`` with its event, ``device_sum`` through ``k_rank_sum`` (gnk_rank_sum),
``sum_device``, device-tensor halos, the tensor all-gather of ``gather_rows`` -- and only the two
transport primitives underneath (``_all_gather_into``, ``_p2p``) move the bytes through host memory
over gloo.  What is NOT exercised is RCCL's own stream semantics (its collectives are stream-ordered;
here they complete synchronously, which is stronger)."""
import torch
import torch.distributed as dist

from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm


class StagedTransportComm(Comm):
    def __init__(self, group=None):
        super().__init__(group)
        self.stage = False                # take the RCCL branches
        self.staged_calls = {"all_gather": 0, "p2p": 0}

    def _all_gather_into(self, buf, t):
        if buf.device.type == "cpu":
            return super()._all_gather_into(buf, t)
        self.staged_calls["all_gather"] += 1
        hb = torch.empty(buf.numel(), dtype=buf.dtype)
        dist.all_gather_into_tensor(hb, t.detach().to("cpu"), group=self.group)
        buf.copy_(hb.view(buf.shape))

    def _p2p(self, ops):
        self.staged_calls["p2p"] += 1
        host_ops, recv = [], []
        for op, t, peer in ops:
            h = t.detach().to("cpu").clone()
            host_ops.append((op, h, peer))
            if op is dist.irecv:
                recv.append((t, h))
        super()._p2p(host_ops)
        for t, h in recv:
            t.copy_(h)
