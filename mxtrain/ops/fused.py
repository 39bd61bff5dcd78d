"""Bias-GeLU, embedding and softmax-cross-entropy ops (``csrc/fused.hip``) with fp32
PyTorch references for CPU tensors."""
from __future__ import annotations

import math

import torch

from . import _lib


def _gelu_tanh(x):
    return 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * x * (1.0 + 0.044715 * x * x)))


def _gelu_tanh_grad(x):
    k0, k1 = 0.7978845608028654, 0.044715
    t = torch.tanh(k0 * x * (1 + k1 * x * x))
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)


# ------------------------------------------------------------------ bias + GeLU
def bias_gelu_fwd(x, bias):
    rows, cols = x.shape
    if not _lib.use_hip(x):
        return _gelu_tanh(x.float() + bias.float()).to(x.dtype)
    y = torch.empty_like(x)
    _lib.call("mx_bias_gelu_fwd", _lib.ptr(x), _lib.ptr(bias), _lib.ptr(y), rows, cols,
              _lib.stream())
    return y


def bias_gelu_bwd(dy, x, bias, dbias=None, accumulate=False, inplace=False, defer=None):
    """dx = dy * gelu'(x + b); dbias (+)= dx.sum(0).  ``inplace`` writes dx over dy."""
    rows, cols = dy.shape
    if not _lib.use_hip(dy):
        dx = (dy.float() * _gelu_tanh_grad(x.float() + bias.float())).to(dy.dtype)
        if dbias is not None:
            v = dx.float().sum(0)
            if accumulate:
                v = v + dbias.float()
            dbias.copy_(v.to(dbias.dtype))
        if inplace:
            dy.copy_(dx)
            return dy
        return dx
    dx = dy if inplace else torch.empty_like(dy)
    rpb = _lib.query("mx_bias_gelu_bwd_rows_per_block")
    nparts = (rows + rpb - 1) // rpb
    partial = None
    if defer is not None and dbias is not None:
        partial = defer.partial((dbias.data_ptr(),), (dbias, None, None), nparts, cols, 1, cols, accumulate)
    if partial is not None:   # partials now, the dbias reduction in the step's batched flush
        _lib.call("mx_bias_gelu_bwd", _lib.ptr(dy), _lib.ptr(x), _lib.ptr(bias), _lib.ptr(dx),
                  None, int(accumulate), _lib.ptr(partial), rows, cols, _lib.stream())
        return dx
    scratch_n = _lib.query64("mx_colreduce_scratch", nparts, cols)
    partial = torch.empty(nparts * cols + scratch_n, dtype=torch.float32, device=dy.device)
    _lib.call("mx_bias_gelu_bwd", _lib.ptr(dy), _lib.ptr(x), _lib.ptr(bias), _lib.ptr(dx),
              _lib.ptr(dbias), int(accumulate), _lib.ptr(partial), rows, cols, _lib.stream())
    return dx


class BiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        ctx.save_for_backward(x2, bias)
        ctx.shape = shape
        return bias_gelu_fwd(x2, bias).view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, bias = ctx.saved_tensors
        db = torch.empty_like(bias)
        dx = bias_gelu_bwd(dy.reshape(x2.shape).contiguous(), x2, bias, dbias=db)
        return dx.view(ctx.shape), db


def bias_gelu(x, bias):
    return BiasGeluFn.apply(x, bias)


# ------------------------------------------------------------------ bias + SwiGLU
def _silu(x):
    return x * torch.sigmoid(x)


def bias_swiglu_fwd(pre, bias=None):
    """pre [rows, 2f] = [a | b] -> silu(a + ba) * (b + bb) [rows, f] (Megatron --swiglu)."""
    rows, f2 = pre.shape
    f = f2 // 2
    if not _lib.use_hip(pre):
        x = pre.float() + (bias.float() if bias is not None else 0.0)
        return (_silu(x[:, :f]) * x[:, f:]).to(pre.dtype)
    y = torch.empty(rows, f, dtype=pre.dtype, device=pre.device)
    _lib.call("mx_bias_swiglu_fwd", _lib.ptr(pre), _lib.ptr(bias), _lib.ptr(y), rows, f,
              _lib.stream())
    return y


def bias_swiglu_bwd(dy, pre, bias=None, dbias=None, accumulate=False):
    """dpre [rows, 2f] from dy [rows, f]; dbias (+)= dpre.sum(0)."""
    rows, f = dy.shape
    if not _lib.use_hip(dy):
        x = pre.float() + (bias.float() if bias is not None else 0.0)
        a, b = x[:, :f], x[:, f:]
        sg = torch.sigmoid(a)
        g = dy.float()
        dpre = torch.cat([g * b * (sg + a * sg * (1 - sg)), g * a * sg], 1).to(dy.dtype)
        if dbias is not None:
            v = dpre.float().sum(0)
            if accumulate:
                v = v + dbias.float()
            dbias.copy_(v.to(dbias.dtype))
        return dpre
    dpre = torch.empty_like(pre)
    nparts = (rows + 15) // 16
    scratch_n = _lib.query64("mx_colreduce_scratch", nparts, 2 * f)
    partial = torch.empty(nparts * 2 * f + scratch_n, dtype=torch.float32, device=dy.device)
    _lib.call("mx_bias_swiglu_bwd", _lib.ptr(dy), _lib.ptr(pre), _lib.ptr(bias), _lib.ptr(dpre),
              _lib.ptr(dbias), int(accumulate), _lib.ptr(partial), rows, f, _lib.stream())
    return dpre


# ------------------------------------------------------------------ embedding
def embed_fwd(ids, wte, wpe=None, seq=None, vocab_start=0, pos_offset=0):
    """ids [ntok] int64 -> wte[ids - vocab_start] (+ wpe[t % seq + pos_offset]).
    Rows whose id is outside [vocab_start, vocab_start + wte.shape[0]) are zero."""
    ntok = ids.numel()
    V, H = wte.shape
    seq = seq or ntok
    if not _lib.use_hip(wte):
        loc = ids - vocab_start
        inside = (loc >= 0) & (loc < V)
        out = wte.float()[loc.clamp(0, V - 1)] * inside[:, None]
        if wpe is not None:
            pos = (torch.arange(ntok, device=ids.device) % seq) + pos_offset
            out = out + wpe.float()[pos]
        return out.to(wte.dtype)
    out = torch.empty(ntok, H, dtype=wte.dtype, device=wte.device)
    _lib.call("mx_embed_fwd", _lib.ptr(ids), _lib.ptr(wte), _lib.ptr(wpe), _lib.ptr(out), ntok, H,
              seq, vocab_start, vocab_start + V, pos_offset, _lib.stream())
    return out


def embed_bwd(ids, dout, dwte, vocab_start=0):
    """dwte[ids] += dout (deterministic; dwte already holds any other contribution)."""
    ntok, H = dout.shape
    V = dwte.shape[0]
    if not _lib.use_hip(dout):
        loc = ids - vocab_start
        inside = (loc >= 0) & (loc < V)
        acc = dwte.float()
        acc.index_add_(0, loc[inside], dout.float()[inside])
        dwte.copy_(acc.to(dwte.dtype))
        return dwte
    if (ids.dtype == torch.int64 and ids.is_contiguous() and dout.is_contiguous() and dwte.is_contiguous()
            and ids.numel() * 8 <= 64 * 1024 and H in (512, 1024, 2048, 4096)):
        # one launch, no sort (csrc/fused.hip embed_bwd_scan_kernel)
        _lib.call("mx_embed_bwd_scan", _lib.ptr(ids), _lib.ptr(dout), _lib.ptr(dwte), ntok, H, vocab_start,
                  vocab_start + V, _lib.stream())
        return dwte
    sorted_ids, perm = torch.sort(ids)
    _lib.call("mx_embed_bwd", _lib.ptr(sorted_ids), _lib.ptr(perm), _lib.ptr(dout), _lib.ptr(dwte),
              ntok, H, vocab_start, vocab_start + V, _lib.stream())
    return dwte


def pos_embed_bwd(dout, dwpe, batch, seq):
    """dwpe[:seq] += sum over batch of dout.view(batch, seq, H)."""
    H = dout.shape[-1]
    if not _lib.use_hip(dout):
        v = dout.float().view(batch, seq, H).sum(0)
        dwpe[:seq].copy_((dwpe[:seq].float() + v).to(dwpe.dtype))
        return dwpe
    _lib.call("mx_pos_embed_bwd", _lib.ptr(dout), _lib.ptr(dwpe), batch, seq, H, _lib.stream())
    return dwpe


# ------------------------------------------------------------------ cross entropy
def ce_stats(logits, labels, vocab_start=0):
    """Per-row (max, sum exp(x - max), x[label] if label in this vocab shard)."""
    rows, V = logits.shape
    if not _lib.use_hip(logits):
        x = logits.float()
        m = x.max(-1).values
        s = torch.exp(x - m[:, None]).sum(-1)
        loc = labels - vocab_start
        inside = (loc >= 0) & (loc < V)
        tgt = torch.where(inside, x.gather(1, loc.clamp(0, V - 1)[:, None])[:, 0],
                          torch.zeros_like(m))
        return m, s, tgt
    m = torch.empty(rows, dtype=torch.float32, device=logits.device)
    s = torch.empty_like(m)
    tgt = torch.empty_like(m)
    _lib.call("mx_ce_stats", _lib.ptr(logits), _lib.ptr(labels), rows, V, vocab_start, _lib.ptr(m),
              _lib.ptr(s), _lib.ptr(tgt), _lib.stream())
    return m, s, tgt


def ce_grad_inplace(logits, labels, lse, tgt, scale, vocab_start=0, ignore_index=-100):
    """logits <- (softmax - onehot) * scale (per valid row); returns per-row loss."""
    rows, V = logits.shape
    if not _lib.use_hip(logits):
        x = logits.float()
        p = torch.exp(x - lse[:, None])
        loc = labels - vocab_start
        inside = (loc >= 0) & (loc < V)
        rows_idx = torch.arange(rows, device=logits.device)
        p[rows_idx[inside], loc[inside]] -= 1.0
        valid = (labels != ignore_index).float()
        sc = scale.float().reshape(()) if torch.is_tensor(scale) else float(scale)
        p = p * valid[:, None] * sc
        logits.copy_(p.to(logits.dtype))
        return torch.where(labels != ignore_index, lse - tgt, torch.zeros_like(lse))
    loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
    if torch.is_tensor(scale):
        sp, sv = _lib.ptr(scale), 0.0
    else:
        sp, sv = None, float(scale)
    _lib.call("mx_ce_grad", _lib.ptr(logits), _lib.ptr(labels), rows, V, vocab_start, _lib.ptr(lse),
              _lib.ptr(tgt), _lib.ptr(loss), sp, sv, ignore_index, _lib.stream())
    return loss


def lse_from_stats(m, s):
    if not _lib.use_hip(m):
        return m + torch.log(s)
    lse = torch.empty_like(m)
    _lib.call("mx_ce_lse", _lib.ptr(m), _lib.ptr(s), _lib.ptr(lse), m.numel(), _lib.stream())
    return lse


# one-pass CE kernel when the whole vocabulary is local (module switch for A/B runs)
SINGLE_PASS_CE = True


def cross_entropy_fwd_bwd(logits, labels, grad_scale, ignore_index=-100, tp_group=None,
                          vocab_start=0):
    """Fused CE: returns per-row losses and overwrites ``logits`` with d(loss*grad_scale)/dlogits.

    With ``tp_group`` the logits are the local vocab shard [vocab_start, vocab_start+V) and
    the row statistics are combined across the tensor-parallel group (vocab-parallel CE,
    three tiny all-reduces: max, rescaled sum, target logit).
    """
    rows, V = logits.shape
    if (SINGLE_PASS_CE and tp_group is None and vocab_start == 0 and _lib.use_hip(logits) and V % 8 == 0
            and V <= 64 * 256 * 8):
        # one pass, the row held in registers (csrc/fused.hip ce_fused_kernel)
        loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
        if torch.is_tensor(grad_scale):
            sp, sv = _lib.ptr(grad_scale), 0.0
        else:
            sp, sv = None, float(grad_scale)
        _lib.call("mx_ce_fused", _lib.ptr(logits), _lib.ptr(labels), rows, V, _lib.ptr(loss), sp, sv,
                  ignore_index, _lib.stream())
        return loss
    m, s, tgt = ce_stats(logits, labels, vocab_start)
    if tp_group is not None:
        # the row max as an all-gather + local max and (sum, target logit) as ONE sum
        # all-reduce: both are collectives the xGMI kernels run, so a captured TP step keeps
        # the CE inside the graph (a MAX reduction would need RCCL / gloo)
        from ..parallel import collectives as C
        gm = C.all_gather_dim0(m.float().reshape(1, -1).contiguous(), tp_group).amax(0)
        st = torch.stack([s.float() * torch.exp(m - gm), tgt.float()])
        C.all_reduce_(st, tp_group)
        s, tgt, m = st[0], st[1], gm
    lse = lse_from_stats(m, s)
    return ce_grad_inplace(logits, labels, lse, tgt, grad_scale, vocab_start, ignore_index)


class CrossEntropyFn(torch.autograd.Function):
    """Mean softmax CE over rows with label != ignore_index; gradient computed in forward."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        x = logits.reshape(-1, logits.shape[-1]).contiguous().clone()
        lab = labels.reshape(-1).contiguous()
        n = max(int((lab != ignore_index).sum().item()), 1)
        losses = cross_entropy_fwd_bwd(x, lab, 1.0 / n, ignore_index)
        ctx.save_for_backward(x)
        ctx.shape = logits.shape
        return losses.sum() / n

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return (x.float() * g).to(x.dtype).view(ctx.shape), None, None


def cross_entropy(logits, labels, ignore_index=-100):
    return CrossEntropyFn.apply(logits, labels, ignore_index)


def softmax_scale(head_dim):
    return 1.0 / math.sqrt(head_dim)
