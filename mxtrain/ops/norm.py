"""LayerNorm / RMSNorm and the fused bias-dropout-add + norm (BDA-norm) ops.

GPU tensors run the HIP kernels of ``csrc/norm.hip``; CPU tensors run the fp32 PyTorch
reference below (also the numerics oracle of ``tests/test_kernels_gpu.py``).
"""
from __future__ import annotations

import torch

from . import _lib
from .rng import keep_mask


def _seed_val(seed_t, salt):
    if seed_t is None:
        return 0
    return (int(seed_t.reshape(-1)[0].item()) + salt) & 0xFFFFFFFF


# ------------------------------------------------------------------ reference (CPU)
def _ref_norm(h32, gamma, beta, eps, rms):
    if rms:
        rstd = torch.rsqrt(h32.pow(2).mean(-1) + eps)
        mean = torch.zeros_like(rstd)
        y = h32 * rstd[:, None] * gamma.float()
    else:
        mean = h32.mean(-1)
        var = (h32 - mean[:, None]).pow(2).mean(-1)
        rstd = torch.rsqrt(var + eps)
        y = (h32 - mean[:, None]) * rstd[:, None] * gamma.float()
        if beta is not None:
            y = y + beta.float()
    return y, mean, rstd


def _ref_bda(x, bias, residual, p, seed_t, salt):
    t = x.float()
    if bias is not None:
        t = t + bias.float()
    if p > 0:
        m = keep_mask(t.numel(), _seed_val(seed_t, salt), p).view_as(t)
        t = torch.where(m, t / (1 - p), torch.zeros_like(t))
    if residual is not None:
        t = t + residual.float()
    return t


# ------------------------------------------------------------------ forward
def layernorm_fwd(x, gamma, beta, eps=1e-5, rms=False):
    """x [rows, cols] -> (y, mean, rstd)."""
    rows, cols = x.shape
    if not _lib.use_hip(x):
        y, mean, rstd = _ref_norm(x.float(), gamma, beta, eps, rms)
        return y.to(x.dtype), mean, rstd
    y = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    if rms:
        _lib.call("mx_rmsnorm_fwd", _lib.ptr(x), _lib.ptr(gamma), _lib.ptr(y), _lib.ptr(rstd),
                  rows, cols, eps, _lib.stream())
    else:
        _lib.call("mx_layernorm_fwd", _lib.ptr(x), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(y),
                  _lib.ptr(mean), _lib.ptr(rstd), rows, cols, eps, _lib.stream())
    return y, mean, rstd


def bda_norm_fwd(x, bias, residual, gamma, beta, eps=1e-5, p=0.0, seed_t=None, salt=0,
                 rms=False):
    """h = residual + dropout(x + bias); y = norm(h).  Returns (h, y, mean, rstd)."""
    rows, cols = x.shape
    if not _lib.use_hip(x):
        h32 = _ref_bda(x, bias, residual, p, seed_t, salt)
        h = h32.to(x.dtype)
        y, mean, rstd = _ref_norm(h.float(), gamma, beta, eps, rms)
        return h, y.to(x.dtype), mean, rstd
    h = torch.empty_like(x)
    y = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    _lib.call("mx_bda_norm_fwd", _lib.ptr(x), _lib.ptr(bias), _lib.ptr(residual), _lib.ptr(gamma),
              _lib.ptr(beta), _lib.ptr(h), _lib.ptr(y), _lib.ptr(mean), _lib.ptr(rstd), rows, cols,
              eps, float(p), _lib.ptr(seed_t), salt, int(rms), _lib.stream())
    return h, y, mean, rstd


# ------------------------------------------------------------------ backward
def norm_bwd(dy, dres, h, mean, rstd, gamma, want_dx=False, p=0.0, seed_t=None, salt=0,
             rms=False, dgamma=None, dbeta=None, dbias=None, accumulate=False):
    """Backward of (bda_)norm.

    dh = dres + dnorm/dh;  dx = dh * dropout-mask * 1/(1-p) (if want_dx).
    Column reductions are written (or added when ``accumulate``) into the bf16 buffers
    ``dgamma``, ``dbeta``, ``dbias`` when given.  Returns (dh, dx or None).
    """
    rows, cols = dy.shape
    if not _lib.use_hip(dy):
        h32 = h.float()
        xh = (h32 - mean[:, None]) * rstd[:, None] if not rms else h32 * rstd[:, None]
        d32 = dy.float()
        gy = d32 * gamma.float()
        m1 = gy.mean(-1, keepdim=True) if not rms else 0.0
        m2 = (gy * xh).mean(-1, keepdim=True)
        dh32 = rstd[:, None] * (gy - m1 - xh * m2)
        if dres is not None:
            dh32 = dh32 + dres.float()
        dh = dh32.to(dy.dtype)
        dx = None
        if want_dx:
            t = dh.float()
            if p > 0:
                m = keep_mask(t.numel(), _seed_val(seed_t, salt), p).view_as(t)
                t = torch.where(m, t / (1 - p), torch.zeros_like(t))
            dx = t.to(dy.dtype)
        for buf, val in ((dgamma, (d32 * xh).sum(0)), (dbeta, d32.sum(0)),
                         (dbias, dx.float().sum(0) if dx is not None else None)):
            if buf is not None and val is not None:
                if accumulate:
                    buf.copy_((buf.float() + val).to(buf.dtype))
                else:
                    buf.copy_(val.to(buf.dtype))
        return dh, dx
    nparts = _lib.query("mx_norm_bwd_nparts2", rows, cols)
    scratch_n = _lib.query64("mx_colreduce_scratch", nparts, 3 * cols)
    partial = torch.empty(nparts * 3 * cols + scratch_n, dtype=torch.float32, device=dy.device)
    dh = torch.empty_like(dy)
    dx = torch.empty_like(dy) if want_dx else None
    _lib.call("mx_norm_bwd", _lib.ptr(dy), _lib.ptr(dres), _lib.ptr(h), _lib.ptr(mean),
              _lib.ptr(rstd), _lib.ptr(gamma), _lib.ptr(dh), _lib.ptr(dx), _lib.ptr(partial),
              rows, cols, float(p), _lib.ptr(seed_t), salt, int(rms), _lib.stream())
    if dgamma is not None or dbeta is not None or dbias is not None:
        scratch = partial[nparts * 3 * cols:]
        _lib.call("mx_colsum_finalize", _lib.ptr(partial), nparts, cols, 3, _lib.ptr(dgamma),
                  _lib.ptr(dbeta), _lib.ptr(dbias if want_dx else None), int(accumulate),
                  _lib.ptr(scratch), _lib.stream())
    return dh, dx


def colsum(x, out, accumulate=False):
    """out (bf16 [cols]) (+)= x.sum(0) for x [rows, cols] bf16."""
    rows, cols = x.shape
    if not _lib.use_hip(x):
        v = x.float().sum(0)
        if accumulate:
            v = v + out.float()
        out.copy_(v.to(out.dtype))
        return out
    nparts = (rows + 15) // 16
    scratch_n = _lib.query64("mx_colreduce_scratch", nparts, cols)
    partial = torch.empty(nparts * cols + scratch_n, dtype=torch.float32, device=x.device)
    _lib.call("mx_colsum_bf16", _lib.ptr(x), rows, cols, _lib.ptr(partial), _lib.ptr(out),
              int(accumulate), _lib.stream())
    return out


# ------------------------------------------------------------------ autograd wrappers
class LayerNormFn(torch.autograd.Function):
    """Plain (Rms/Layer)Norm with autograd; parameter grads go to autograd .grad."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, rms):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd = layernorm_fwd(x2, gamma, beta, eps, rms)
        ctx.save_for_backward(x2, mean, rstd, gamma)
        ctx.rms = rms
        ctx.has_beta = beta is not None
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, mean, rstd, gamma = ctx.saved_tensors
        dg = torch.empty_like(gamma)
        db = torch.empty_like(gamma) if ctx.has_beta else None
        dh, _ = norm_bwd(dy.reshape(x2.shape).contiguous(), None, x2, mean, rstd, gamma,
                         rms=ctx.rms, dgamma=dg, dbeta=db)
        return dh.view(ctx.shape), dg, db, None, None


def layer_norm(x, gamma, beta=None, eps=1e-5):
    return LayerNormFn.apply(x, gamma, beta, eps, False)


def rms_norm(x, gamma, eps=1e-6):
    return LayerNormFn.apply(x, gamma, None, eps, True)


class BDANormFn(torch.autograd.Function):
    """y = norm(residual + dropout(x + bias)) with autograd (post-LN transformer blocks,
    e.g. BERT): one fused HIP pass forward, one fused pass backward producing
    d(residual), d(x) (dropout mask regenerated from the seed) and the dgamma/dbeta/dbias
    column sums."""

    @staticmethod
    def forward(ctx, x, bias, residual, gamma, beta, eps, p, seed_t, salt, rms):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        r2 = residual.reshape(-1, shape[-1]).contiguous() if residual is not None else None
        h, y, mean, rstd = bda_norm_fwd(x2, bias, r2, gamma, beta, eps, p, seed_t, salt, rms)
        ctx.save_for_backward(h, mean, rstd, gamma)
        ctx.meta = (p, seed_t, salt, rms, bias is not None, beta is not None, residual is not None, shape)
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        h, mean, rstd, gamma = ctx.saved_tensors
        p, seed_t, salt, rms, has_bias, has_beta, has_res, shape = ctx.meta
        dg = torch.empty_like(gamma)
        db = torch.empty_like(gamma) if has_beta else None
        dbias = torch.empty_like(gamma) if has_bias else None
        dh, dx = norm_bwd(dy.reshape(h.shape).contiguous(), None, h, mean, rstd, gamma, want_dx=True, p=p,
                          seed_t=seed_t, salt=salt, rms=rms, dgamma=dg, dbeta=db, dbias=dbias)
        return (dx.view(shape), dbias, dh.view(shape) if has_res else None, dg, db,
                None, None, None, None, None)


def bda_norm(x, bias, residual, gamma, beta, eps=1e-5, p=0.0, seed_t=None, salt=0, rms=False):
    return BDANormFn.apply(x, bias, residual, gamma, beta, eps, p, seed_t, salt, rms)
