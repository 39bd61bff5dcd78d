"""Flash attention op (``csrc/attention.hip``) + fp32 reference.

Tensors are token-major: ``q``, ``k``, ``v`` are 2-D views [B*S, H*D] with an arbitrary
row stride (so the packed QKV projection output is consumed in place); the output is
[B*S, Hq*D].  ``lse`` is the base-2 log-sum-exp [B, Hq, S] the backward needs.
"""
from __future__ import annotations

import math

import torch

from . import _lib

LOG2E = 1.4426950408889634


def _ref_fwd(q, k, v, B, S, Hq, Hkv, D, causal, klen, scale):
    qf = q.float().reshape(B, S, Hq, D).transpose(1, 2)
    kf = k.float().reshape(B, S, Hkv, D).transpose(1, 2)
    vf = v.float().reshape(B, S, Hkv, D).transpose(1, 2)
    if Hq != Hkv:
        kf = kf.repeat_interleave(Hq // Hkv, 1)
        vf = vf.repeat_interleave(Hq // Hkv, 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    mask = torch.zeros(B, 1, S, S, dtype=torch.bool, device=q.device)
    if causal:
        mask |= torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
    if klen is not None:
        kidx = torch.arange(S, device=q.device)
        mask |= (kidx[None, :] >= klen[:, None].to(q.device)).view(B, 1, 1, S)
    s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, -1)  # natural
    p = torch.exp(s - lse[..., None])
    o = torch.matmul(p, vf).transpose(1, 2).reshape(B * S, Hq * D)
    return o, lse * LOG2E


def attn_fwd(q, k, v, B, S, Hq, Hkv, D, causal=True, klen=None, scale=None):
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not _lib.use_hip(q):
        o, lse = _ref_fwd(q, k, v, B, S, Hq, Hkv, D, causal, klen, scale)
        return o.to(q.dtype), lse
    assert q.dtype == torch.bfloat16 and D in (64, 128)
    assert q.stride(1) == 1 and k.stride(1) == 1 and v.stride(1) == 1
    o = torch.empty(B * S, Hq * D, dtype=q.dtype, device=q.device)
    lse = torch.empty(B, Hq, S, dtype=torch.float32, device=q.device)
    kl = klen.to(torch.int32).contiguous() if klen is not None else None
    _lib.call("mx_attn_fwd", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), q.stride(0), k.stride(0),
              v.stride(0), _lib.ptr(o), o.stride(0), _lib.ptr(lse), B, S, Hq, Hkv, D, int(causal),
              _lib.ptr(kl), float(scale), _lib.stream())
    return o, lse


def attn_bwd(dout, q, k, v, o, lse, B, S, Hq, Hkv, D, causal=True, klen=None, scale=None,
             dq=None, dk=None, dv=None):
    """Returns (dq, dk, dv); if views dq/dk/dv (e.g. slices of a packed dqkv) are given
    they are written in place."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not _lib.use_hip(q):
        with torch.enable_grad():
            qq = q.detach().float().requires_grad_(True)
            kk = k.detach().float().requires_grad_(True)
            vv = v.detach().float().requires_grad_(True)
            oo, _ = _ref_fwd(qq, kk, vv, B, S, Hq, Hkv, D, causal, klen, scale)
            gq, gk, gv = torch.autograd.grad(oo, (qq, kk, vv), dout.float())
        outs = []
        for g, buf in ((gq, dq), (gk, dk), (gv, dv)):
            if buf is not None:
                buf.copy_(g.to(buf.dtype))
                outs.append(buf)
            else:
                outs.append(g.to(q.dtype))
        return tuple(outs)
    if dq is None:
        dq = torch.empty(B * S, Hq * D, dtype=q.dtype, device=q.device)
    if dk is None:
        dk = torch.empty(B * S, Hkv * D, dtype=q.dtype, device=q.device)
    if dv is None:
        dv = torch.empty(B * S, Hkv * D, dtype=q.dtype, device=q.device)
    delta = torch.empty(B, Hq, S, dtype=torch.float32, device=q.device)
    # zeroed by the delta pre-pass inside mx_attn_bwd
    dq_acc = torch.empty(B * S, Hq * D, dtype=torch.float32, device=q.device)
    kl = klen.to(torch.int32).contiguous() if klen is not None else None
    _lib.call("mx_attn_bwd", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), q.stride(0), k.stride(0),
              v.stride(0), _lib.ptr(o), o.stride(0), _lib.ptr(dout), dout.stride(0), _lib.ptr(lse),
              _lib.ptr(delta), _lib.ptr(dq_acc), _lib.ptr(dq), dq.stride(0), _lib.ptr(dk),
              _lib.ptr(dv), dk.stride(0), dv.stride(0), B, S, Hq, Hkv, D, int(causal), _lib.ptr(kl),
              float(scale), _lib.stream())
    return dq, dk, dv


class FlashAttnFn(torch.autograd.Function):
    """Autograd wrapper over [B, S, H, D]-style inputs flattened to [B*S, H*D]."""

    @staticmethod
    def forward(ctx, q, k, v, B, S, Hq, Hkv, D, causal, klen, scale):
        o, lse = attn_fwd(q, k, v, B, S, Hq, Hkv, D, causal, klen, scale)
        ctx.save_for_backward(q, k, v, o, lse, klen if klen is not None else torch.empty(0))
        ctx.meta = (B, S, Hq, Hkv, D, causal, scale, klen is not None)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kl = ctx.saved_tensors
        B, S, Hq, Hkv, D, causal, scale, has_kl = ctx.meta
        dq, dk, dv = attn_bwd(do.contiguous(), q, k, v, o, lse, B, S, Hq, Hkv, D, causal,
                              kl if has_kl else None, scale)
        return dq, dk, dv, None, None, None, None, None, None, None, None


def flash_attention(q, k, v, B, S, Hq, Hkv, D, causal=True, klen=None, scale=None):
    return FlashAttnFn.apply(q, k, v, B, S, Hq, Hkv, D, causal, klen, scale)
