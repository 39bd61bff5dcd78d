"""Flat, bucketed parameter / gradient storage.

Every parameter of a model stage is a view into ONE contiguous bf16 buffer, and its
gradient (`main_grad`) a view into a parallel bf16 buffer.  The layout is chosen for
the MI355X collectives:

* each parameter starts on a 64-element (128-B) boundary -> 16-B vector loads in the
  fused optimizer, and a weight-decay flag per 64-element chunk;
* parameters are grouped into buckets in *backward completion order*, each bucket
  padded to a multiple of 64 * dp_world so a reduce-scatter of a bucket gives every
  DP rank an equally sized, 64-aligned shard (ZeRO-1);
* bucket sizes default to ~100 MB of bf16 -- big enough that RCCL reaches its
  per-link bandwidth on xGMI, small enough to start the first reduce-scatter early
  in backward.

Replaces DeepSpeed's ZeRO-1 flat fp16 groups and Horovod's 64 MB fusion buffer (K18).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

ALIGN = 64


@dataclass
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    init: str = "normal"          # normal | zeros | ones | scaled_normal
    std: float = 0.02
    weight_decay: bool = True
    unit: int = 0                 # backward-completion unit (bucketing key)
    tp_duplicated: bool = True    # identical on every TP rank (count once in grad norm)
    sp_reduce: bool = False       # grad needs TP all-reduce under sequence parallelism
    shared: Optional[str] = None  # tied-weight group name (e.g. "word_embeddings")

    @property
    def numel(self):
        n = 1
        for s in self.shape:
            n *= s
        return n


@dataclass
class Bucket:
    index: int
    start: int
    end: int
    units: List[int] = field(default_factory=list)
    names: List[str] = field(default_factory=list)

    @property
    def size(self):
        return self.end - self.start


def _round_up(x, m):
    return (x + m - 1) // m * m


class FlatParams:
    """Owns the flat param/grad buffers and the per-parameter views."""

    def __init__(self, specs: Sequence[ParamSpec], device, dtype=torch.bfloat16, dp_world: int = 1,
                 bucket_numel: int = 50_000_000, unit_order: Optional[List[int]] = None):
        self.specs = list(specs)
        self.dtype = dtype
        self.device = torch.device(device)
        self.dp_world = dp_world
        units = sorted({s.unit for s in self.specs})
        if unit_order is None:
            unit_order = list(reversed(units))  # last unit finishes backward first
        by_unit: Dict[int, List[ParamSpec]] = {u: [] for u in units}
        for s in self.specs:
            by_unit[s.unit].append(s)
        self.offsets: Dict[str, int] = {}
        self.buckets: List[Bucket] = []
        pad_to = ALIGN * dp_world
        off = 0
        cur = Bucket(0, 0, 0)
        for u in unit_order:
            for s in by_unit[u]:
                self.offsets[s.name] = off
                off += _round_up(s.numel, ALIGN)
                cur.names.append(s.name)
            cur.units.append(u)
            if off - cur.start >= bucket_numel:
                off = _round_up(off, pad_to)
                cur.end = off
                self.buckets.append(cur)
                cur = Bucket(len(self.buckets), off, off)
        if cur.units:
            off = _round_up(max(off, cur.start + 1), pad_to)
            cur.end = off
            self.buckets.append(cur)
        self.numel = off
        self.unit_to_bucket = {u: b.index for b in self.buckets for u in b.units}
        self.data = torch.zeros(self.numel, dtype=dtype, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=dtype, device=self.device)
        self.params: Dict[str, torch.Tensor] = {}
        self.grads: Dict[str, torch.Tensor] = {}
        self.spec_by_name = {s.name: s for s in self.specs}
        for s in self.specs:
            o = self.offsets[s.name]
            self.params[s.name] = self.data[o:o + s.numel].view(s.shape)
            self.grads[s.name] = self.grad[o:o + s.numel].view(s.shape)
        # one weight-decay flag per 64-element chunk of the flat buffer
        flags = torch.zeros(self.numel // ALIGN, dtype=torch.uint8)
        for s in self.specs:
            if s.weight_decay:
                o = self.offsets[s.name] // ALIGN
                flags[o:o + _round_up(s.numel, ALIGN) // ALIGN] = 1
        self.wd_flags = flags.to(self.device)

    def bucket_of_grad_ptr(self, ptr: int) -> Optional[int]:
        """Index of the bucket whose slice of the flat gradient buffer holds address
        ``ptr`` (None: not in the buffer)."""
        base = self.grad.data_ptr()
        e = (ptr - base) // self.grad.element_size()
        if e < 0 or e >= self.numel:
            return None
        for b in self.buckets:
            if b.start <= e < b.end:
                return b.index
        return None

    # ----------------------------------------------------------------- init
    def initialize(self, generator: Optional[torch.Generator] = None, num_layers: int = 1):
        for s in self.specs:
            p = self.params[s.name]
            if s.init == "zeros":
                p.zero_()
            elif s.init == "ones":
                p.fill_(1.0)
            else:
                std = s.std
                if s.init == "scaled_normal":
                    std = s.std / (2.0 * num_layers) ** 0.5
                t = torch.empty(s.shape, dtype=torch.float32)
                t.normal_(0.0, std, generator=generator)
                p.copy_(t.to(self.dtype))

    def set_overwritten(self, names) -> None:
        """Gradients in ``names`` are written whole (beta = 0 GEMMs) by the first
        micro-batch of every step: zero_grad() / zero_grad_range() then clear only the other
        elements (norm / bias / embedding gradients, ~1 % of the buffer) with one
        index_fill instead of a fill of the whole flat buffer."""
        keep = torch.ones(self.numel, dtype=torch.bool)
        for n in names:
            o = self.offsets[n]
            keep[o:o + self.spec_by_name[n].numel] = False
        idx = keep.nonzero().flatten()
        self._zero_idx = idx.to(self.device)
        self._zero_idx_cpu = idx

    def zero_grad(self):
        idx = getattr(self, "_zero_idx", None)
        if idx is None:
            self.grad.zero_()
        else:
            self.grad.index_fill_(0, idx, 0)

    def zero_grad_range(self, start: int, end: int):
        """zero_grad() restricted to grad[start:end] (one bucket)."""
        idx = getattr(self, "_zero_idx", None)
        if idx is None:
            self.grad[start:end].zero_()
            return
        cache = self.__dict__.setdefault("_zero_idx_ranges", {})
        sub = cache.get((start, end))
        if sub is None:
            cpu = self._zero_idx_cpu
            lo = int(torch.searchsorted(cpu, start))
            hi = int(torch.searchsorted(cpu, end))
            sub = cache[(start, end)] = idx[lo:hi]
        if sub.numel():
            self.grad.index_fill_(0, sub, 0)

    def state_dict(self):
        return {n: p.detach().clone().cpu() for n, p in self.params.items()}

    def load_state_dict(self, sd, strict=True):
        for n, p in self.params.items():
            if n in sd:
                p.copy_(sd[n].to(p.dtype))
            elif strict:
                raise KeyError(n)
