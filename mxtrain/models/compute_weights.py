"""Batched fp32 -> bf16 compute copies of a model's trainable weights (AMP-style master
weights without one cast kernel per tensor).

The detection model keeps fp32 parameters (the optimizer, Horovod all-reduce and the
tensorpack checkpoint contract see fp32) and computes in bf16.  Casting every weight
inside its module's forward costs ~2 kernels per tensor forward (cast, plus the FrozenBN
scale multiply of a folded conv) and ~2 in backward -- about 300 launches and their
Python dispatch per Mask R-CNN step, most of them a few microseconds long.  Here ONE
autograd Function produces all compute copies with multi-tensor ``_foreach`` kernels
(fold-scale multiply, then cast into one flat bf16 buffer) and its backward returns all
fp32 gradients the same way; the modules look their copy up with ``cw(param, dtype)``.

    with ComputeWeights(model.compute_weight_specs(), torch.bfloat16):
        losses = model(...)            # modules call cw(p, dt) / folded convs call cw(w)

Gradients reach the fp32 parameters through the Function, so optimizers, clipping and
gradient hooks are unchanged.  Under data parallelism the specs are cut into ``groups``
contiguous node groups (model order): a group's fp32 gradients -- and so its DDP / Horovod
bucket hooks -- become ready as soon as backward has passed the first module that uses
it, instead of all at the very end of backward, so the gradient all-reduce overlaps the
rest of backward again.  Frozen parameters (requires_grad False) are not
included: their modules keep caching their own copies (resnet.ConvNorm._folded).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

_ACTIVE: Dict[int, torch.Tensor] = {}


def cw(p: torch.Tensor, dt: torch.dtype) -> torch.Tensor:
    """The active compute copy of parameter ``p`` (already scaled when it was registered
    with a fold scale), else a plain cast."""
    t = _ACTIVE.get(id(p))
    if t is not None:
        return t
    return p.to(dt)


def has(p: torch.Tensor) -> bool:
    return id(p) in _ACTIVE


class _CastAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dt, scales, scaled_idx, *params):
        ctx.scales, ctx.scaled_idx = scales, scaled_idx
        src = list(params)
        if scaled_idx:
            prod = torch._foreach_mul([params[i] for i in scaled_idx], [scales[i] for i in scaled_idx])
            for i, t in zip(scaled_idx, prod):
                src[i] = t
        sizes = [p.numel() for p in params]
        flat = torch.empty(sum(sizes), dtype=dt, device=params[0].device)
        outs = []
        for v, p in zip(flat.split(sizes), params):
            if p.dim() == 4:
                # conv weights in channels_last, the layout MIOpen's NHWC kernels take,
                # so the conv does not transpose the weight on every call
                o, i, kh, kw = p.shape
                outs.append(v.view(o, kh, kw, i).permute(0, 3, 1, 2))
            else:
                outs.append(v.view(p.shape))
        torch._foreach_copy_(outs, src)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        idx = [i for i, g in enumerate(grads) if g is not None]
        out: List[Optional[torch.Tensor]] = [None] * len(grads)
        if idx:
            g32 = [torch.empty(grads[i].shape, dtype=torch.float32, device=grads[i].device) for i in idx]
            torch._foreach_copy_(g32, [grads[i] for i in idx])
            pos = {i: j for j, i in enumerate(idx)}
            sc = [i for i in ctx.scaled_idx if i in pos]
            if sc:
                # d(w * s)/dw = s
                torch._foreach_mul_([g32[pos[i]] for i in sc], [ctx.scales[i] for i in sc])
            for i, g in zip(idx, g32):
                out[i] = g
        return (None, None, None, *out)


class ComputeWeights:
    """Context manager: builds the compute copies of ``specs`` = [(param, fold_scale or
    None)] once on entry (one autograd node) and makes them visible to cw()."""

    def __init__(self, specs: Sequence[Tuple[torch.Tensor, Optional[torch.Tensor]]], dt: torch.dtype,
                 groups: int = 1):
        self.specs = [(p, s) for p, s in specs if p.requires_grad]
        self.dt = dt
        self.groups = max(1, int(groups))

    @staticmethod
    def split(specs, groups: int):
        """Contiguous chunks of ~equal parameter count (model order kept)."""
        if groups <= 1 or len(specs) <= 1:
            return [list(specs)]
        total = sum(p.numel() for p, _ in specs)
        out, cur, acc = [], [], 0
        for p, s in specs:
            cur.append((p, s))
            acc += p.numel()
            if acc >= total * (len(out) + 1) / groups and len(out) < groups - 1:
                out.append(cur)
                cur = []
        if cur:
            out.append(cur)
        return out

    def __enter__(self):
        if self.specs and torch.is_grad_enabled():
            for chunk in self.split(self.specs, self.groups):
                params = [p for p, _ in chunk]
                scales = [s for _, s in chunk]
                scaled = [i for i, s in enumerate(scales) if s is not None]
                outs = _CastAll.apply(self.dt, scales, scaled, *params)
                for p, o in zip(params, outs):
                    _ACTIVE[id(p)] = o
        return self

    def __exit__(self, *exc):
        for p, _ in self.specs:
            _ACTIVE.pop(id(p), None)
        return False
