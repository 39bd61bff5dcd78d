"""Counter-based dropout RNG shared by the HIP kernels and the CPU reference.

Elements come in aligned groups of 8: group g = idx >> 3 seeds an xorshift32 stream with
``x0 = hash32(lo(g) ^ hi(g)*0x85ebca6b, seed) | 1``; word j of the stream holds the 16-bit
draws of elements 8g + 2j (low half) and 8g + 2j + 1 (high half), kept when
>= round(p * 2^16).  Bit-identical to ``mx::dropout_keep8`` in ``csrc/common.h``.  Masks are
never stored: backward regenerates them from the same (seed, element index).

The seed lives in a 1-element int32 device tensor so a hipGraph-captured step sees a
fresh value on every replay (``DropoutSeed.advance`` is itself captured).
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF


def _u32(x: torch.Tensor) -> torch.Tensor:
    return x & M32


def hash32(x: torch.Tensor, seed: int) -> torch.Tensor:
    x = _u32(x ^ _u32(torch.tensor(seed, dtype=torch.int64) * 0x9E3779B9))
    x = x ^ (x >> 16)
    x = _u32(x * 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _u32(x * 0x846CA68B)
    x = x ^ (x >> 16)
    return x


def _xorshift(x: torch.Tensor) -> torch.Tensor:
    x = x ^ _u32(x << 13)
    x = x ^ (x >> 17)
    return x ^ _u32(x << 5)


def keep_threshold16(p: float) -> int:
    """16-bit keep threshold from p, exactly as the kernels derive it from p * 2^32."""
    t32 = int(p * 4294967296.0) if p > 0 else 0
    return (t32 + 0x8000) >> 16


def keep_mask(numel: int, seed: int, p: float, device="cpu", base: int = 0) -> torch.Tensor:
    """Boolean keep-mask for flat element indices base..base+numel-1."""
    if p <= 0:
        return torch.ones(numel, dtype=torch.bool, device=device)
    g0, g1 = base >> 3, (base + numel + 7) >> 3
    g = torch.arange(g0, g1, dtype=torch.int64, device=device)
    x = (g & M32) ^ _u32(((g >> 32) & M32) * 0x85EBCA6B)
    x = hash32(x, seed) | 1
    words = [x]
    for _ in range(3):
        x = _xorshift(x)
        words.append(x)
    w = torch.stack(words, 1)                                   # [G, 4]
    draws = torch.stack([w & 0xFFFF, w >> 16], 2).reshape(-1)   # element order 2j, 2j + 1
    keep = draws >= keep_threshold16(p)
    off = base - 8 * g0
    return keep[off:off + numel]


class DropoutSeed:
    """Device-resident dropout seeds, advanced once per training step.

    Element 0 seeds the token-local dropouts (hidden / residual; it differs across data-
    and context-parallel ranks, which hold different tokens); element 1 (``attn_t``, when
    ``attn_seed`` is given) seeds attention dropout, whose mask is keyed on the global
    (batch, head, query, key) and so must be the SAME on every context-parallel rank."""

    def __init__(self, device, seed: int = 1234, attn_seed=None):
        vals = [seed & 0x7FFFFFFF] + ([attn_seed & 0x7FFFFFFF] if attn_seed is not None else [])
        self.t = torch.tensor(vals, dtype=torch.int32, device=device)
        self.attn_t = self.t[1:2] if attn_seed is not None else self.t[0:1]

    def value(self) -> int:
        return int(self.t[0].item())

    INC = 0x61C88647 & 0x7FFFFFFF

    def advance(self):
        # stays on-device (captured into hipGraphs); wraps harmlessly
        self.t.add_(self.INC)
        self.t.bitwise_and_(0x7FFFFFFF)

    def set_step(self, seed: int, steps: int, attn_seed=None):
        """State after `steps` advances from `seed` (checkpoint resume)."""
        self.t[0] = ((seed & 0x7FFFFFFF) + steps * self.INC) % (1 << 31)
        if attn_seed is not None and self.t.numel() > 1:
            self.t[1] = ((attn_seed & 0x7FFFFFFF) + steps * self.INC) % (1 << 31)
