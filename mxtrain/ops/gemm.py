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
import os
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
_FORCE = os.environ.get("MXTRAIN_GEMM_VARIANT")


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
