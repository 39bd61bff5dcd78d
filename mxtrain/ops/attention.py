"""Flash attention op (``csrc/attention.hip``) + fp32 reference.

Tensors are token-major: ``q``, ``k``, ``v`` are 2-D views [B*S, H*D] with an arbitrary
row stride (so the packed QKV projection output is consumed in place); the output is
[B*S, Hq*D].  ``lse`` is the base-2 log-sum-exp [B, Hq, S] the backward needs.

Attention dropout (Megatron ``--attention-dropout``, default 0.1 in the reference's GPT
configs: examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-zero1.yaml:39-53 sets no
override; HF BERT ``attention_probs_dropout_prob`` 0.1) is applied to the softmax
probabilities inside the kernels.  The keep-mask is a pure function of (seed, salt, batch,
GLOBAL head, query, key) -- :func:`dropout_keep_mask` is the definition, bit-identical to
``attn_dropmask_kernel`` -- so tensor- and context-parallel shards (``head_offset``) draw
exactly the single-GPU mask, and backward reuses the forward's key-on-lane image.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from .rng import M32, hash32

LOG2E = 1.4426950408889634


def dropout_threshold(p: float) -> int:
    """16-bit keep threshold (an element is kept when its 16-bit hash >= thr)."""
    return int(p * 65536.0 + 0.5)


def effective_keep_scale(p: float) -> float:
    """1 / (1 - p_eff), p_eff = thr/65536 (the probability the kernels actually drop)."""
    thr = dropout_threshold(p)
    return 65536.0 / (65536.0 - thr)


def dropout_keep_mask(B, S, Hq, seed: int, salt: int, p: float, head_offset: int = 0,
                      total_heads=None, device="cpu") -> torch.Tensor:
    """Dense boolean keep-mask [B, Hq, S(q), S(k)] -- the definition the kernels implement
    (flash.hip drop_stream_bits).  For query row q of head h (row = (b*Hg + h_global)*S + q)
    and key k = 32 kb + kk: the lane half hh = (kk >> 2) & 1 and pair j = ((kk & 3) + 4 (kk >> 3))
    >> 1 select the j-th output of an xorshift32 stream seeded by hash32(row*0x85EBCA6B +
    2 kb + hh, seed + salt) | 1; its low (k even) or high (k odd) 16 bits are the draw, and the
    element is kept when draw >= round(p * 65536)."""
    Hg = total_heads or Hq
    seed = (int(seed) + int(salt)) & M32
    NB = (S + 31) // 32
    b = torch.arange(B, dtype=torch.int64, device=device).view(B, 1, 1, 1, 1)
    h = torch.arange(Hq, dtype=torch.int64, device=device).view(1, Hq, 1, 1, 1) + head_offset
    q = torch.arange(S, dtype=torch.int64, device=device).view(1, 1, S, 1, 1)
    kb = torch.arange(NB, dtype=torch.int64, device=device).view(1, 1, 1, NB, 1)
    hh = torch.arange(2, dtype=torch.int64, device=device).view(1, 1, 1, 1, 2)
    row = ((b * Hg + h) * S + q) & M32
    x = hash32((row * 0x85EBCA6B + 2 * kb + hh) & M32, seed) | 1
    xs = [x]
    for _ in range(7):
        x = x ^ ((x << 13) & M32)
        x = x ^ (x >> 17)
        x = x ^ ((x << 5) & M32)
        xs.append(x)
    X = torch.stack(xs, -1)                                   # [B, Hq, S, NB, 2, 8]
    k = torch.arange(S, dtype=torch.int64, device=device)
    kk = k % 32
    sel_kb, sel_hh = k // 32, (kk >> 2) & 1
    sel_j = ((kk & 3) + 4 * (kk >> 3)) >> 1
    draws = X[:, :, :, sel_kb, sel_hh, sel_j]                 # [B, Hq, S, S]
    draws = (draws >> (16 * (kk & 1))) & 0xFFFF
    return draws >= dropout_threshold(p)


def _ref_fwd(q, k, v, B, S, Hq, Hkv, D, causal, klen, scale, keep=None, keep_scale=1.0):
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
    if keep is not None:
        p = p * keep.to(p.device, p.dtype) * keep_scale
    o = torch.matmul(p, vf).transpose(1, 2).reshape(B * S, Hq * D)
    return o, lse * LOG2E


class DropMask:
    """Attention-dropout state of one forward, kept for its backward: the kernels' two bit
    images (query-on-lane for the forward / dQ kernels, key-on-lane for dK/dV) on the GPU,
    the dense keep-mask on the CPU path; ``event`` marks the side-stream generation."""

    __slots__ = ("fbits", "bbits", "keep", "p", "event")

    def __init__(self, p, fbits=None, bbits=None, keep=None, event=None):
        self.p, self.fbits, self.bbits, self.keep, self.event = p, fbits, bbits, keep, event

    @property
    def keep_scale(self):
        return effective_keep_scale(self.p)

    def ready(self):
        if self.event is not None:
            torch.cuda.current_stream().wait_event(self.event)
            self.event = None


def dropmask(B, S, Hq, p, seed_t, salt=0, head_offset=0, total_heads=None, causal=True,
             device=None) -> DropMask:
    """Generate the keep-mask images of one attention call."""
    device = device if device is not None else seed_t.device
    if device.type != "cuda" or not _lib.use_hip(seed_t):
        keep = dropout_keep_mask(B, S, Hq, int(seed_t.reshape(-1)[0]), salt, p, head_offset, total_heads, device)
        return DropMask(p, keep=keep)
    NB, NKT, NQT = (S + 31) // 32, (S + 127) // 128, (S + 63) // 64
    fbits = torch.empty(B * Hq * NB * NKT * 64, dtype=torch.int64, device=device)
    bbits = torch.empty(B * Hq * NB * NQT * 64, dtype=torch.int32, device=device)
    _lib.call("mx_flash_dropmask", _lib.ptr(seed_t), int(salt) & M32, float(p), B, S, Hq, int(head_offset),
              int(total_heads or Hq), int(causal), _lib.ptr(fbits), _lib.ptr(bbits), _lib.stream())
    return DropMask(p, fbits, bbits)


def dropmask_layers(B, S, Hq, p, seed_t, salt, L, head_offset=0, total_heads=None, causal=True,
                    device=None):
    """The keep-mask images of L consecutive layers (salts salt .. salt + L - 1) in ONE
    launch -- identical to L dropmask() calls; a step's masks depend only on its seed, so
    the model generates them all before the first layer (one launch instead of one per
    layer, and the single large grid keeps the chip full).  Returns [DropMask] * L."""
    device = device if device is not None else seed_t.device
    if device.type != "cuda" or not _lib.use_hip(seed_t):
        return [dropmask(B, S, Hq, p, seed_t, salt + l, head_offset, total_heads, causal, device) for l in range(L)]
    NB, NKT, NQT = (S + 31) // 32, (S + 127) // 128, (S + 63) // 64
    nf, nb = B * Hq * NB * NKT * 64, B * Hq * NB * NQT * 64
    fbits = torch.empty(L, nf, dtype=torch.int64, device=device)
    bbits = torch.empty(L, nb, dtype=torch.int32, device=device)
    _lib.call("mx_flash_dropmask_layers", _lib.ptr(seed_t), int(salt) & M32, float(p), B, S, Hq,
              int(head_offset), int(total_heads or Hq), int(causal), L, _lib.ptr(fbits[0]), _lib.ptr(bbits[0]),
              2 * nf, nb, _lib.stream())
    return [DropMask(p, fbits[l], bbits[l]) for l in range(L)]


def attn_fwd(q, k, v, B, S, Hq, Hkv, D, causal=True, klen=None, scale=None, dropout_p=0.0,
             seed_t=None, salt=0, head_offset=0, total_heads=None, dmask=None):
    """Returns (o, lse, dmask): dmask is the DropMask backward needs (None without dropout).
    A pre-generated ``dmask`` (dropmask / dropmask_layers) is used as is."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    drop = dropout_p > 0.0 or dmask is not None
    if drop and dmask is None:
        assert seed_t is not None, "attention dropout needs the device seed tensor"
        dmask = dropmask(B, S, Hq, dropout_p, seed_t, salt, head_offset, total_heads, causal, device=q.device)
    if not _lib.use_hip(q):
        o, lse = _ref_fwd(q, k, v, B, S, Hq, Hkv, D, causal, klen, scale,
                          dmask.keep if drop else None, dmask.keep_scale if drop else 1.0)
        return o.to(q.dtype), lse, dmask
    assert q.dtype == torch.bfloat16 and D in (64, 128)
    assert q.stride(1) == 1 and k.stride(1) == 1 and v.stride(1) == 1
    o = torch.empty(B * S, Hq * D, dtype=q.dtype, device=q.device)
    lse = torch.empty(B, Hq, S, dtype=torch.float32, device=q.device)
    kl = klen.to(torch.int32).contiguous() if klen is not None else None
    if drop:
        dmask.ready()
    _lib.call("mx_flash_fwd", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), q.stride(0), k.stride(0),
              v.stride(0), _lib.ptr(o), o.stride(0), _lib.ptr(lse), B, S, Hq, Hkv, D, int(causal),
              _lib.ptr(kl), float(scale), _lib.ptr(dmask.fbits) if drop else None,
              float(dmask.keep_scale) if drop else 1.0, _lib.stream())
    return o, lse, dmask


def attn_bwd(dout, q, k, v, o, lse, B, S, Hq, Hkv, D, causal=True, klen=None, scale=None,
             dq=None, dk=None, dv=None, dmask=None, dropout_p=0.0, bias_partial=None):
    """Returns (dq, dk, dv); if views dq/dk/dv (e.g. slices of a packed dqkv) are given
    they are written in place.  ``dmask`` is the third output of :func:`attn_fwd`.

    ``bias_partial`` (GPU, S % 32 == 0): fp32 [B*S/32, (Hq + 2 Hkv) * D] that receives the
    column sums of every 32-row group of [dq | dk | dv] (the QKV bias gradient's partials,
    reduced later by the deferred column reduction) -- computed from the kernels'
    accumulators, so dq / dk / dv are not read again."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not _lib.use_hip(q):
        assert bias_partial is None, "bias_partial is a GPU-kernel output"
        keep = dmask.keep if dmask is not None else None
        with torch.enable_grad():
            qq = q.detach().float().requires_grad_(True)
            kk = k.detach().float().requires_grad_(True)
            vv = v.detach().float().requires_grad_(True)
            oo, _ = _ref_fwd(qq, kk, vv, B, S, Hq, Hkv, D, causal, klen, scale, keep,
                             dmask.keep_scale if keep is not None else 1.0)
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
    kl = klen.to(torch.int32).contiguous() if klen is not None else None
    _lib.call("mx_flash_bwd", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), q.stride(0), k.stride(0),
              v.stride(0), _lib.ptr(o), o.stride(0), _lib.ptr(dout), dout.stride(0), _lib.ptr(lse),
              _lib.ptr(delta), _lib.ptr(dq), dq.stride(0), _lib.ptr(dk), _lib.ptr(dv), dk.stride(0),
              dv.stride(0), B, S, Hq, Hkv, D, int(causal), _lib.ptr(kl), float(scale),
              _lib.ptr(dmask.fbits) if dmask is not None else None,
              _lib.ptr(dmask.bbits) if dmask is not None else None,
              float(dmask.keep_scale) if dmask is not None else 1.0, _lib.ptr(bias_partial),
              bias_partial.stride(0) if bias_partial is not None else 0, _lib.stream())
    return dq, dk, dv


class FlashAttnFn(torch.autograd.Function):
    """Autograd wrapper over [B, S, H, D]-style inputs flattened to [B*S, H*D]."""

    @staticmethod
    def forward(ctx, q, k, v, B, S, Hq, Hkv, D, causal, klen, scale, dropout_p, seed_t, salt):
        o, lse, dmask = attn_fwd(q, k, v, B, S, Hq, Hkv, D, causal, klen, scale, dropout_p, seed_t, salt)
        ctx.save_for_backward(q, k, v, o, lse, klen if klen is not None else torch.empty(0))
        ctx.dmask = dmask
        ctx.meta = (B, S, Hq, Hkv, D, causal, scale, klen is not None, dropout_p)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kl = ctx.saved_tensors
        B, S, Hq, Hkv, D, causal, scale, has_kl, p = ctx.meta
        dq, dk, dv = attn_bwd(do.contiguous(), q, k, v, o, lse, B, S, Hq, Hkv, D, causal,
                              kl if has_kl else None, scale, dmask=ctx.dmask, dropout_p=p)
        ctx.dmask = None
        return dq, dk, dv, None, None, None, None, None, None, None, None, None, None, None


def flash_attention(q, k, v, B, S, Hq, Hkv, D, causal=True, klen=None, scale=None, dropout_p=0.0,
                    seed_t=None, salt=0):
    return FlashAttnFn.apply(q, k, v, B, S, Hq, Hkv, D, causal, klen, scale, dropout_p, seed_t, salt)
