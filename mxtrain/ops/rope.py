"""Rotary position embedding (``csrc/rope.hip``, K5 in SURVEY §2.8) + fp32 reference.

Applied in place to the Q and K column blocks of the packed QKV activation
[tokens, (Hq + 2*Hkv) * D] right after the QKV GEMM (forward), and the transpose
rotation is applied in place to dQ / dK before the QKV weight-gradient GEMM (backward).
Rotate-half convention (Megatron-DeepSpeed ``apply_rotary_pos_emb`` / GPT-NeoX / LLaMA)
with ``rotary_percent`` support (rd = D * percent).

The cos/sin tables are fp32 [max_pos, rd/2], built in fp64 once per (device, rd, base,
max_pos) and cached.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from . import _lib

_TABLES: Dict[Tuple, Tuple[torch.Tensor, torch.Tensor]] = {}


def rope_tables(max_pos: int, rd: int, base: float = 10000.0, device="cpu"):
    key = (str(device), max_pos, rd, float(base))
    t = _TABLES.get(key)
    if t is None:
        inv = 1.0 / (base ** (torch.arange(0, rd, 2, dtype=torch.float64) / rd))
        ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
        t = (ang.cos().float().contiguous().to(device), ang.sin().float().contiguous().to(device))
        _TABLES[key] = t
    return t


def _ref_rope_(x, col0, heads, D, rd, S, pos_offset, pos_ids, cos, sin, inverse):
    T = x.shape[0]
    half = rd // 2
    pos = pos_ids if pos_ids is not None else (torch.arange(T, device=x.device) % S) + pos_offset
    c = cos[pos].float()[:, None, :]   # [T, 1, half]
    s = sin[pos].float()[:, None, :]
    if inverse:
        s = -s
    blk = x[:, col0:col0 + heads * D].float().reshape(T, heads, D)
    x1 = blk[..., :half].clone()
    x2 = blk[..., half:rd].clone()
    blk[..., :half] = x1 * c - x2 * s
    blk[..., half:rd] = x2 * c + x1 * s
    x[:, col0:col0 + heads * D] = blk.reshape(T, heads * D).to(x.dtype)
    return x


def apply_rope_(x: torch.Tensor, col0: int, heads: int, head_dim: int, seq: int,
                rotary_dim: Optional[int] = None, base: float = 10000.0, pos_offset: int = 0,
                pos_ids: Optional[torch.Tensor] = None, max_pos: Optional[int] = None,
                inverse: bool = False) -> torch.Tensor:
    """Rotate ``heads`` head blocks of ``x`` [tokens, ld] starting at column ``col0`` in
    place.  ``x`` may be a column slice with row stride ``ld`` (e.g. the q or k view of a
    packed QKV buffer)."""
    rd = rotary_dim or head_dim
    T = x.shape[0]
    mp = max_pos or (int(pos_ids.max().item()) + 1 if pos_ids is not None else seq + pos_offset)
    cos, sin = rope_tables(mp, rd, base, x.device)
    if not _lib.use_hip(x):
        return _ref_rope_(x, col0, heads, head_dim, rd, seq, pos_offset, pos_ids, cos, sin, inverse)
    assert x.dtype == torch.bfloat16 and x.stride(1) == 1
    assert rd % 8 == 0 and rd <= head_dim and head_dim % 4 == 0
    pid = pos_ids.to(torch.int64).contiguous() if pos_ids is not None else None
    _lib.call("mx_rope", _lib.ptr(x), x.stride(0), col0, heads, head_dim, rd, T, seq, pos_offset,
              _lib.ptr(pid), _lib.ptr(cos), _lib.ptr(sin), int(inverse), _lib.stream())
    return x


class RopeFn(torch.autograd.Function):
    """Out-of-place autograd wrapper over a [T, H*D] tensor (tests / generic models)."""

    @staticmethod
    def forward(ctx, x, heads, head_dim, seq, rotary_dim, base, pos_offset):
        y = x.contiguous().clone()
        apply_rope_(y, 0, heads, head_dim, seq, rotary_dim, base, pos_offset)
        ctx.meta = (heads, head_dim, seq, rotary_dim, base, pos_offset)
        return y

    @staticmethod
    def backward(ctx, g):
        heads, head_dim, seq, rotary_dim, base, pos_offset = ctx.meta
        d = g.contiguous().clone()
        apply_rope_(d, 0, heads, head_dim, seq, rotary_dim, base, pos_offset, inverse=True)
        return d, None, None, None, None, None, None


def rope(x, heads, head_dim, seq, rotary_dim=None, base=10000.0, pos_offset=0):
    return RopeFn.apply(x, heads, head_dim, seq, rotary_dim, base, pos_offset)
