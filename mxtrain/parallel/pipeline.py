"""1F1B pipeline-parallel schedule (P4, M9) over point-to-point RCCL send/recv.

Replaces the DeepSpeed PipelineEngine that Megatron-DeepSpeed uses for
`--pipeline-model-parallel-size 2` (examples/megatron-deepspeed/gpt2_345m/
pretrain-ddp-tp-pp-zero1.yaml:40).  Stage s runs min(p - s - 1, m) warm-up forwards,
then alternates one forward / one backward, then drains the remaining backwards.
Activations travel as one contiguous [tokens, hidden] bf16 tensor per micro-batch
(a single xGMI p2p transfer); the activation gradient travels back the same way.
Each stage reports its gradient units to the DP optimizer only during the LAST
micro-batch's backward, so bucket reduce-scatters overlap the pipeline drain.

Transport: RCCL ``batch_isend_irecv`` by default; with ``MXTRAIN_XGMI=1`` the direct xGMI
channels of ``parallel/xgmi.py`` (XGMIP2P: the sender's ring slot read by the receiver over
xGMI, device-side sequence counters, side streams), which also run between processes
sharing one GPU -- so the 1F1B schedule executes on real HIP streams in the one-GPU tests.
"""
from __future__ import annotations

from collections import deque
from typing import TYPE_CHECKING

import torch
import torch.distributed as dist

if TYPE_CHECKING:  # pragma: no cover
    from ..training import GPTTrainer


class _P2P:
    """Posted batch of p2p ops: ``wait()`` completes them and returns the received
    tensor (None for send-only batches); the send tensor is kept alive until then."""
    __slots__ = ("reqs", "rbuf", "keep")

    def __init__(self, reqs, rbuf, keep):
        self.reqs, self.rbuf, self.keep = reqs, rbuf, keep

    def wait(self):
        for r in self.reqs:
            r.wait()
        self.reqs, self.keep = [], None
        return self.rbuf


class PipelineSchedule:
    SEND_WINDOW = 2   # outstanding posted sends before the oldest is waited for

    def __init__(self, trainer: "GPTTrainer"):
        self.tr = trainer
        self.ps = trainer.ps
        self._xp = None          # XGMIP2P channels (MXTRAIN_XGMI), built on first use
        self._xp_key = None

    def _xgmi(self, shape):
        """The xGMI p2p channels for activations of ``shape`` (None: RCCL).  Collective over
        the pipeline group, so every stage calls it at the top of run()."""
        from . import xgmi
        ps = self.ps
        dev = self.tr.device
        if not xgmi.enabled() or dev.type != "cuda" or ps.pp_group is None:
            return None
        nb = shape[0] * shape[1] * torch.empty((), dtype=self.tr.dtype).element_size()
        if self._xp_key != nb:
            g = ps.pp_group
            peers = [dist.get_group_rank(g, r) for r in (ps.prev_rank(), ps.next_rank()) if r is not None]
            self._xp = xgmi.get_p2p(g, dev, peers, nb)
            self._xp_key = nb
        return self._xp

    def _act_shape(self, B, S):
        ps = self.ps
        tokens = B * S
        if ps.sequence_parallel:
            tokens //= ps.tp
        return (tokens, self.tr.cfg.hidden_size)

    # ---------------------------------------------------------------- p2p primitives
    # Every transfer is posted without waiting; the consumer waits right before it uses
    # the tensor (a stream dependency under RCCL, not a host block); at most SEND_WINDOW
    # sends stay outstanding (their tensors referenced) before the oldest is waited for.
    # Receives are posted as early as the schedule allows -- the next forward's input
    # before this step's backward, the next backward's gradient before this backward --
    # so the transfer runs under compute.  Opposite-direction transfers that are needed
    # together (send activation / receive its gradient) are posted in one
    # batch_isend_irecv so the pair can never deadlock.
    def _buf(self, shape):
        return torch.empty(shape, dtype=self.tr.dtype, device=self.tr.device)

    def _post(self, send_t=None, send_to=None, recv_shape=None, recv_from=None):
        xp = self._xp if self._xp_key is not None else None
        if xp is not None:
            g = self.ps.pp_group
            return xp.post(send_t=send_t, send_to=dist.get_group_rank(g, send_to) if send_t is not None else None,
                           recv_buf=self._buf(recv_shape) if recv_shape is not None else None,
                           recv_from=dist.get_group_rank(g, recv_from) if recv_shape is not None else None)
        ops = []
        rbuf = None
        if send_t is not None:
            send_t = send_t.contiguous()
            ops.append(dist.P2POp(dist.isend, send_t, send_to))
        if recv_shape is not None:
            rbuf = self._buf(recv_shape)
            ops.append(dist.P2POp(dist.irecv, rbuf, recv_from))
        reqs = dist.batch_isend_irecv(ops) if ops else []
        return _P2P(reqs, rbuf, send_t)

    def _exchange(self, send_t=None, send_to=None, recv_shape=None, recv_from=None):
        """Blocking form (evaluation path): post and wait."""
        return self._post(send_t, send_to, recv_shape, recv_from).wait()

    def run(self, tokens: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        tr, ps = self.tr, self.ps
        stage = tr.stage
        nm, B, S = tokens.shape
        p, s = ps.pp, ps.pp_rank
        shape = self._act_shape(B, S)
        self._xgmi(shape)
        first, last = ps.is_first_stage, ps.is_last_stage
        prev, nxt = ps.prev_rank(), ps.next_rank()
        warm = min(p - s - 1, nm)
        remaining = nm - warm
        loss_total = torch.zeros((), dtype=torch.float32, device=tr.device)
        inflight = deque()
        # posted sends: a bounded window (each keeps its activation / gradient tensor alive
        # until waited), so memory does not grow with the number of micro-batches
        sends = deque()

        def push_send(sd):
            sends.append(sd)
            while len(sends) > self.SEND_WINDOW:
                sends.popleft().wait()
        fwd_i = 0
        bwd_i = 0

        def fwd(inp):
            nonlocal fwd_i, loss_total
            m = fwd_i
            fwd_i += 1
            if first:
                out = stage.forward(ids=tokens[m].reshape(-1), labels=labels[m].reshape(-1), B=B, S=S, micro=m)
            else:
                out = stage.forward(hidden=inp, labels=labels[m].reshape(-1), B=B, S=S, micro=m)
            if last:
                loss_total = loss_total + out.detach()
            inflight.append((inp, out))
            return out

        def bwd(out_grad):
            nonlocal bwd_i
            inp, out = inflight.popleft()
            stage.rt.unit_done = tr.opt.unit_done if bwd_i == nm - 1 else None
            bwd_i += 1
            if last:
                out.backward()
            else:
                torch.autograd.backward(out, grad_tensors=out_grad)
            return None if first else inp.grad

        def post_recv_fwd():
            return None if first else self._post(recv_shape=shape, recv_from=prev)

        def take(pend, grad=False):
            if pend is None:
                return None
            t = pend.wait()
            return t.requires_grad_(True) if grad else t

        # warm-up forwards (the next input is prefetched while this forward runs)
        nin = post_recv_fwd() if (warm > 0 or remaining > 0) else None
        for k in range(warm):
            inp = take(nin, grad=True)
            nin = post_recv_fwd() if (k + 1 < warm or remaining > 0) else None
            out = fwd(inp)
            if not last:
                push_send(self._post(send_t=out.detach(), send_to=nxt))
        # steady state: 1F1B
        inp = take(nin, grad=True) if remaining > 0 else None
        nin = None
        for i in range(remaining):
            out = fwd(inp)
            out_grad = None
            if not last:
                out_grad = self._post(send_t=out.detach(), send_to=nxt, recv_shape=shape, recv_from=nxt).wait()
            # prefetch the next forward's input before running this backward
            nin = post_recv_fwd() if i < remaining - 1 else None
            in_grad = bwd(out_grad)
            if not first:
                push_send(self._post(send_t=in_grad, send_to=prev))
            inp = take(nin, grad=True) if i < remaining - 1 else None
        # cool-down backwards (the next gradient is prefetched while this backward runs)
        ng = None if (last or warm == 0) else self._post(recv_shape=shape, recv_from=nxt)
        for k in range(warm):
            out_grad = take(ng)
            ng = None if (last or k + 1 >= warm) else self._post(recv_shape=shape, recv_from=nxt)
            in_grad = bwd(out_grad)
            if not first:
                push_send(self._post(send_t=in_grad, send_to=prev))
        for sd in sends:
            sd.wait()
        return loss_total

    @torch.no_grad()
    def run_forward_only(self, tokens: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """Evaluation: every micro-batch flows forward through the stages; the last stage
        returns the summed loss (0 elsewhere)."""
        tr, ps = self.tr, self.ps
        stage = tr.stage
        nm, B, S = tokens.shape
        shape = self._act_shape(B, S)
        self._xgmi(shape)
        first, last = ps.is_first_stage, ps.is_last_stage
        prev, nxt = ps.prev_rank(), ps.next_rank()
        loss_total = torch.zeros((), dtype=torch.float32, device=tr.device)
        for m in range(nm):
            if first:
                out = stage.forward(ids=tokens[m].reshape(-1), labels=labels[m].reshape(-1), B=B, S=S, micro=m)
            else:
                inp = self._exchange(recv_shape=shape, recv_from=prev)
                out = stage.forward(hidden=inp, labels=labels[m].reshape(-1), B=B, S=S, micro=m)
            if last:
                loss_total = loss_total + out.detach()
            else:
                self._exchange(send_t=out, send_to=nxt)
        return loss_total
