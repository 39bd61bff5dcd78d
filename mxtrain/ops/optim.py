"""Fused AdamW + gradient L2-norm on flat shards (``csrc/optim.hip``), with reference."""
from __future__ import annotations

import torch

from . import _lib

# hyper[] layout shared with csrc/optim.hip
H_LR, H_B1, H_B2, H_EPS, H_WD, H_BC1, H_BC2, H_GS, H_CLIP, H_N = range(10)


def sumsq_bf16(g, scale=1.0, out=None, accumulate=False, flags=None):
    """out[0] (+)= sum((g*scale)^2) as fp32 on g's device (no host sync).  ``flags``: one
    uint8 per 64-element chunk, chunks flagged 0 are excluded."""
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=g.device)
    if not _lib.use_hip(g):
        x = g.float() * scale
        if flags is not None:
            x = x * flags.to(torch.float32).repeat_interleave(64)[: x.numel()]
        v = x.pow(2).sum()
        if accumulate:
            out += v
        else:
            out.fill_(float(v))
        return out
    nparts = _lib.query("mx_sumsq_nparts")
    partial = torch.empty(nparts, dtype=torch.float32, device=g.device)
    _lib.call("mx_sumsq_bf16", _lib.ptr(g), g.numel(), float(scale), _lib.ptr(flags),
              _lib.ptr(partial), _lib.ptr(out), int(accumulate), _lib.stream())
    return out


def adamw_step(master, exp_avg, exp_avg_sq, grad, param_out, hyper, normsq=None, wd_flags=None):
    """One fused AdamW step over flat fp32 ``master`` with bf16 ``grad``; writes bf16
    ``param_out``.  ``hyper`` is the fp32 device array documented in csrc/optim.hip;
    ``wd_flags`` a uint8 flag per 64-element chunk (None = decay everything)."""
    n = master.numel()
    if not _lib.use_hip(master):
        h = hyper.float().tolist()
        ns = float(normsq.item()) if normsq is not None else 0.0
        if normsq is not None and not (ns == ns and ns != float("inf")):
            return False
        gs = h[H_GS]
        if h[H_CLIP] > 0 and normsq is not None:
            coef = h[H_CLIP] / (ns ** 0.5 + 1e-6)
            if coef < 1:
                gs *= coef
        g = grad.float() * gs
        exp_avg.mul_(h[H_B1]).add_(g, alpha=1 - h[H_B1])
        exp_avg_sq.mul_(h[H_B2]).addcmul_(g, g, value=1 - h[H_B2])
        denom = exp_avg_sq.sqrt() / (h[H_BC2] ** 0.5) + h[H_EPS]
        if wd_flags is None:
            decay = torch.full_like(master, h[H_WD])
        else:
            decay = wd_flags.to(torch.float32).repeat_interleave(64)[:n] * h[H_WD]
        master.mul_(1 - h[H_LR] * decay)
        master.addcdiv_(exp_avg, denom, value=-h[H_LR] / h[H_BC1])
        param_out.copy_(master.to(param_out.dtype))
        return True
    assert n % 4 == 0
    _lib.call("mx_adamw_step", _lib.ptr(master), _lib.ptr(exp_avg), _lib.ptr(exp_avg_sq),
              _lib.ptr(grad), _lib.ptr(param_out), _lib.ptr(wd_flags), n, _lib.ptr(hyper),
              _lib.ptr(normsq), _lib.stream())
    return True
