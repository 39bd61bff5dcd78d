"""Hand-written MFMA GEMMs (csrc/gemm.hip).

``wgrad_group([(gbuf, dy, x), ...], accumulate)`` computes ``gbuf (+)= dy^T x`` for up to
four Linear layers in ONE launch -- the weight gradients of a transformer layer that become
ready together (fc1 + fc2, qkv + proj).  dy [T, out] and x [T, in] are read in place (row
strides allowed); gbuf [out, in] is the bf16 gradient view.  ``accumulate=False`` writes
the gradient (so the gradient buffer needs no zero-fill), True adds to it.

Shapes the kernel does not tile (out or in not a multiple of 128, T not a multiple of 64,
misaligned strides) go through ``torch.addmm`` -- that path is part of the contract, not an
error fallback; CPU tensors always use it.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

import torch

from . import _lib

_DESC_T = ctypes.c_int64 * 32


def _tileable(gbuf: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> bool:
    if gbuf.dtype != torch.bfloat16 or dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16:
        return False
    if dy.dim() != 2 or x.dim() != 2 or gbuf.dim() != 2:
        return False
    T, M = dy.shape
    N = x.shape[1]
    if x.shape[0] != T or tuple(gbuf.shape) != (M, N):
        return False
    if M % 128 or N % 128 or T % 64:
        return False
    if dy.stride(1) != 1 or x.stride(1) != 1 or gbuf.stride(1) != 1:
        return False
    if dy.stride(0) % 8 or x.stride(0) % 8:
        return False
    if dy.data_ptr() % 16 or x.data_ptr() % 16:
        return False
    return True


def wgrad_group(items: Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]], accumulate: bool = True,
                variant: int = -1, splits: int = 0):
    items = list(items)
    if not items:
        return
    if not _lib.use_hip(items[0][0]):
        for gbuf, dy, x in items:
            _torch_wgrad(gbuf, dy, x, accumulate)
        return
    T = items[0][1].shape[0]
    fast: List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = []
    for it in items:
        if _tileable(*it) and it[1].shape[0] == T and len(fast) < 4:
            fast.append(it)
        else:
            _torch_wgrad(*it, accumulate)
    if not fast:
        return
    if variant < 0:
        pl = plan(fast, T)
        if pl is None:
            for it in fast:
                _torch_wgrad(*it, accumulate)
            return
        variant, splits = pl
    elif splits <= 0:
        splits = 1
    desc = _DESC_T()
    for q, (gbuf, dy, x) in enumerate(fast):
        desc[8 * q:8 * q + 8] = [dy.data_ptr(), x.data_ptr(), gbuf.data_ptr(), dy.stride(0), x.stride(0),
                                 gbuf.stride(0), dy.shape[1], x.shape[1]]
    slab = ticket = None
    if splits > 1:
        bm, bn = _tile(variant)
        tiles = sum((dy.shape[1] // bm) * (x.shape[1] // bn) for _, dy, x in fast)
        slab, ticket = _workspace(fast[0][0].device, tiles * splits * bm * bn, tiles)
    _lib.call("mx_gemm_kk", len(fast), desc, T, 1.0 if accumulate else 0.0, variant, splits,
              _lib.ptr(slab), _lib.ptr(ticket), _lib.stream())


_TILE = {}


def _tile(variant):
    t = _TILE.get(variant)
    if t is None:
        t = _TILE[variant] = (_lib.query("mx_gemm_kk_tile", variant, 0), _lib.query("mx_gemm_kk_tile", variant, 1))
    return t


NUM_CU = 256
_FORCE = None      # "variant[:splits]": benchmarking scripts pin the wgrad plan


def plan(items, T: int):
    """(variant, splits) for a group, from measurements on one MI355X (scripts/gemm_bench.py,
    T = 4096): one tile per CU -> 8 waves of 64 x 32 (variant 6: 48.6 us for qkv+proj vs
    75.4 us hipBLASLt); two per CU -> 4-wave 128 x 128 workgroups, two per CU (variant 0:
    75 us for fc1+fc2 vs 95 us).  Split-K loses (the fp32 slab round trip), so it is not
    planned.  Returns None when hipBLASLt is the better choice: under 128 tiles (idle CUs)
    or over 1024 (large outputs, e.g. the LM head, where its 256-wide tiles win)."""
    if _FORCE:
        v, s = (_FORCE.split(":") + ["1"])[:2]
        return int(v), int(s)
    tiles = sum((dy.shape[1] // 128) * (x.shape[1] // 128) for _, dy, x in items)
    if tiles < 128 or tiles > 1024:
        return None
    return (6, 1) if tiles <= 320 else (0, 1)


_WS = {}


def _workspace(device, slab_elems, tiles):
    key = device
    ws = _WS.get(key)
    if ws is None or ws[0].numel() < slab_elems or ws[1].numel() < tiles:
        s = max(slab_elems, ws[0].numel() if ws else 0)
        t = max(tiles, ws[1].numel() if ws else 0)
        ws = _WS[key] = (torch.empty(s, device=device, dtype=torch.float32),
                         torch.zeros(t, device=device, dtype=torch.int32))
    return ws


def _torch_wgrad(gbuf, dy, x, accumulate):
    if accumulate:
        gbuf.addmm_(dy.t(), x)
    else:
        torch.mm(dy.t(), x, out=gbuf)


def wgrad(gbuf, dy, x, accumulate: bool = True):
    wgrad_group([(gbuf, dy, x)], accumulate)


# ============================================================================== forward / dgrad
# csrc/gemm_nt.hip: C = A W^T (forward) or C = A W (dgrad) with the Linear layer's
# elementwise tail fused into the epilogue (bias; bias + GeLU saving the pre-activation;
# GeLU' + bias-gradient column partials).  Shapes the kernel does not tile go through
# torch (part of the contract, like wgrad above); CPU tensors always do.
_NT_TILE = {}
_NT_FORCE = None   # benchmarking scripts pin the gemm_nt variant
# preference order: big tiles first (less L2 traffic per FLOP), as long as one launch still
# has >= ~one tile per CU
_NT_ORDER = (0, 1, 4, 5, 3, 2)


def _nt_tile(variant):
    t = _NT_TILE.get(variant)
    if t is None:
        t = _NT_TILE[variant] = tuple(_lib.query("mx_gemm_nt_tile", variant, w) for w in range(4))
    return t


# Above this many multiply-adds hipBLASLt wins even against the fused epilogues: at the
# GPT-3 6.7B layer shapes (T 4096, hidden 4096: M*N*K 6.9e10 .. 2.7e11) it ran the layer's
# forward + dgrad GEMMs in 2408 us vs 2771 us for the planned variants (1.3-1.6 vs 1.0-1.3
# PF/s; profiles/r3_s4/gemm_gpt3_shapes.txt) and the one-GPU GPT-3 bench 22.10k vs 21.06k
# tokens/s, while at the GPT-2 345M shapes (<= 1.7e10) the hand-written kernels take the
# layer from 291 to 232 us (profiles/r3_s1/gemm_nt_vs_hipblaslt.txt).
# The model asks nt_fits() before routing a Linear through these kernels (models/gpt.py);
# above the limit it takes its hipBLASLt + separate-epilogue path.
NT_MAX_MNK = 1 << 35


def nt_fits(M: int, N: int, K: int) -> bool:
    """True when the hand-written fused-epilogue GEMM is the faster choice for this size."""
    return M * N * K <= NT_MAX_MNK


def nt_plan(M: int, N: int, K: int, kmajor: bool) -> int:
    """Variant of csrc/gemm_nt.hip for an [M, K] x [K, N] problem, or -1 (not tileable)."""
    if K % 64:
        return -1
    if _NT_FORCE:
        v = int(_NT_FORCE)
        bm, bn, _, kok = _nt_tile(v)
        return v if (M % bm == 0 and N % bn == 0 and (kok or not kmajor)) else -1
    fallback = -1
    for v in _NT_ORDER:
        bm, bn, _, kok = _nt_tile(v)
        if M % bm or N % bn or (kmajor and not kok):
            continue
        if (M // bm) * (N // bn) >= 224:
            return v
        if fallback < 0 or (M // bm) * (N // bn) > (M // _nt_tile(fallback)[0]) * (N // _nt_tile(fallback)[1]):
            fallback = v
    return fallback


def _nt_ok(t: torch.Tensor) -> bool:
    return (t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and t.data_ptr() % 16 == 0)


def _gelu_ref(h):
    return 0.5 * h * (1.0 + torch.tanh(0.7978845608028654 * (h + 0.044715 * h * h * h)))


def _gelu_grad_ref(h):
    t = torch.tanh(0.7978845608028654 * (h + 0.044715 * h * h * h))
    return 0.5 * (1.0 + t) + 0.5 * h * (1.0 - t * t) * 0.7978845608028654 * (1.0 + 3 * 0.044715 * h * h)


def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias=None, gelu: bool = False, out=None, variant: int = -1):
    """y = x @ w^T (+ bias), x [M, K], w [N, K].  With ``gelu``: returns (gelu(h), h) where
    h = x w^T + bias is the bf16 pre-activation kept for backward (Megatron bias_gelu)."""
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K, (x.shape, w.shape)
    assert bias is not None or not gelu
    v = variant
    hip = _lib.use_hip(x)
    if hip and v < 0 and _nt_ok(x) and _nt_ok(w) and (bias is None or bias.is_contiguous()) \
            and (out is None or _nt_ok(out)):
        v = nt_plan(M, N, K, False)
    if not hip or v < 0:
        if gelu:
            h = torch.addmm(bias, x, w.t()) if hip else (x.float() @ w.float().t() + bias.float())
            y = _gelu_ref(h.float()).to(x.dtype)
            h = h.to(x.dtype)
            if out is not None:
                out.copy_(y)
                y = out
            return y, h
        if hip:
            y = torch.addmm(bias, x, w.t()) if bias is not None else torch.mm(x, w.t())
        else:
            y32 = x.float() @ w.float().t()
            if bias is not None:
                y32 = y32 + bias.float()
            y = y32.to(x.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    y = out if out is not None else torch.empty((M, N), dtype=x.dtype, device=x.device)
    h = torch.empty((M, N), dtype=x.dtype, device=x.device) if gelu else None
    epi = 2 if gelu else (1 if bias is not None else 0)
    _lib.call("mx_gemm_nt", x.data_ptr(), w.data_ptr(), y.data_ptr(), _lib.ptr(h), _lib.ptr(bias), None,
              x.stride(0), w.stride(0), y.stride(0), N, M, N, K, 0, epi, v, _lib.stream())
    return (y, h) if gelu else y


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, gelu_aux=None, dbias=None, accumulate: bool = True,
                 defer=None, variant: int = -1, out=None):
    """dx = dy @ w, dy [M, N_out], w [N_out, K_in] -> dx [M, K_in].  With ``gelu_aux`` (the
    pre-activation h of the layer that produced dy's input... i.e. the fc1 output): returns
    dx * gelu'(h), and ``dbias`` (bf16 [K_in]) (+)= its column sums -- the fc1 bias gradient
    (``defer``: ops/norm.py ColReduceQueue, reduced in the step's batched flush)."""
    M, Kd = dy.shape
    N = w.shape[1]
    assert w.shape[0] == Kd, (dy.shape, w.shape)
    hip = _lib.use_hip(dy)
    v = variant
    if hip and v < 0 and _nt_ok(dy) and _nt_ok(w) and (gelu_aux is None or _nt_ok(gelu_aux)) \
            and (out is None or _nt_ok(out)):
        v = nt_plan(M, N, Kd, True)
    if not hip or v < 0:
        if hip and gelu_aux is None:
            return torch.mm(dy, w, out=out) if out is not None else torch.mm(dy, w)
        d32 = torch.mm(dy, w).float() if hip else dy.float() @ w.float()
        if gelu_aux is None:
            if out is not None:
                out.copy_(d32)
                return out
            return d32.to(dy.dtype)
        d32 = d32 * _gelu_grad_ref(gelu_aux.float())
        if dbias is not None:
            s = d32.sum(0)
            if accumulate:
                s = s + dbias.float()
            dbias.copy_(s.to(dbias.dtype))
        if out is not None:
            out.copy_(d32)
            return out
        return d32.to(dy.dtype)
    dx = out if out is not None else torch.empty((M, N), dtype=dy.dtype, device=dy.device)
    if gelu_aux is None:
        _lib.call("mx_gemm_nt", dy.data_ptr(), w.data_ptr(), dx.data_ptr(), None, None, None,
                  dy.stride(0), w.stride(0), dx.stride(0), 0, M, N, Kd, 1, 0, v, _lib.stream())
        return dx
    prow = _nt_tile(v)[2]
    nparts = M // prow
    part = None
    if defer is not None and dbias is not None:
        part = defer.partial((dbias.data_ptr(),), (dbias, None, None), nparts, N, 1, N, accumulate)
    deferred = part is not None
    if part is None:
        scratch_n = _lib.query64("mx_colreduce_scratch", nparts, N)
        part = torch.empty(nparts * N + scratch_n, dtype=torch.float32, device=dy.device)
    _lib.call("mx_gemm_nt", dy.data_ptr(), w.data_ptr(), dx.data_ptr(), gelu_aux.data_ptr(), None,
              part.data_ptr(), dy.stride(0), w.stride(0), dx.stride(0), gelu_aux.stride(0), M, N, Kd, 1, 3, v,
              _lib.stream())
    if dbias is not None and not deferred:
        _lib.call("mx_colsum_finalize", part.data_ptr(), nparts, N, 1, dbias.data_ptr(), None, None,
                  int(accumulate), part[nparts * N:].data_ptr(), _lib.stream())
    return dx
