"""Counter-based dropout RNG shared by the HIP kernels and the CPU reference.

``keep(idx)`` = hash32(lo(idx) ^ hi(idx)*0x85ebca6b, seed) >= p*2^32, bit-identical to
``mx::dropout_keep`` in ``csrc/common.h``.  Masks are never stored: backward
regenerates them from the same (seed, element index).

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


def keep_mask(numel: int, seed: int, p: float, device="cpu", base: int = 0) -> torch.Tensor:
    """Boolean keep-mask for flat element indices base..base+numel-1."""
    idx = torch.arange(base, base + numel, dtype=torch.int64, device=device)
    lo = idx & M32
    hi = (idx >> 32) & M32
    x = lo ^ _u32(hi * 0x85EBCA6B)
    h = hash32(x, seed)
    thresh = int(p * 4294967296.0) if p > 0 else 0
    return h >= thresh


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
