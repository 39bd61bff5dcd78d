"""Thin collective helpers used by TP / SP / PP / DP code (RCCL on GPU, gloo on CPU).

All tensors are token-major ([tokens, hidden]); sequence parallelism shards the token
dimension, so SP all-gather / reduce-scatter work on dim 0 and are single contiguous
RCCL calls (no transposes, one kernel per call).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.distributed as dist

from . import xgmi as _xgmi


def world(group) -> int:
    return dist.get_world_size(group) if group is not None else 1


def all_reduce_(t: torch.Tensor, group, op=None):
    if group is None or world(group) == 1:
        return t
    if (op is None or op == dist.ReduceOp.SUM) and t.is_contiguous():
        c = _xgmi.route(group, t, "all_reduce", t.numel() * t.element_size())
        if c is not None:
            return c.all_reduce_(t)
    dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=group)
    return t


def all_gather_dim0(t: torch.Tensor, group) -> torch.Tensor:
    n = world(group)
    if n == 1:
        return t
    out = torch.empty((t.shape[0] * n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    c = _xgmi.route(group, t, "all_gather", out.numel() * out.element_size())
    if c is not None:
        return c.all_gather(out, t.contiguous())
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def reduce_scatter_dim0(t: torch.Tensor, group) -> torch.Tensor:
    n = world(group)
    if n == 1:
        return t
    assert t.shape[0] % n == 0
    out = torch.empty((t.shape[0] // n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    c = _xgmi.route(group, t, "reduce_scatter", t.numel() * t.element_size())
    if c is not None:
        return c.reduce_scatter(out, t.contiguous())
    dist.reduce_scatter_tensor(out, t.contiguous(), group=group)
    return out


def split_dim0(t: torch.Tensor, group) -> torch.Tensor:
    n = world(group)
    if n == 1:
        return t
    r = dist.get_rank(group)
    c = t.shape[0] // n
    return t[r * c:(r + 1) * c].contiguous()


# --------------------------------------------------------------------------- async (TP overlap)
_SIDE: Dict[int, object] = {}


def _side_stream(device) -> "torch.cuda.Stream":
    i = torch.device(device).index or 0
    s = _SIDE.get(i)
    if s is None:
        s = _SIDE[i] = torch.cuda.Stream(device=device)
    return s


class Pending:
    """A collective in flight: ``wait()`` orders the caller's stream after it (never a host
    block on the GPU: RCCL's work.wait() and the side-stream join are stream dependencies)
    and returns the result tensor."""
    __slots__ = ("out", "work", "stream")

    def __init__(self, out: torch.Tensor, work=None, stream=None):
        self.out, self.work, self.stream = out, work, stream

    def wait(self) -> torch.Tensor:
        if self.work is not None:
            self.work.wait()
            self.work = None
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.out.device)
            cur.wait_stream(self.stream)
            self.out.record_stream(cur)
            self.stream = None
        return self.out


def _on_side(x: torch.Tensor, fn) -> Pending:
    """Run an xGMI kernel collective on the side stream, after the producer of ``x``."""
    cur = torch.cuda.current_stream(x.device)
    s = _side_stream(x.device)
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        out = fn()
    x.record_stream(s)
    return Pending(out, stream=s)


def all_reduce_async(t: torch.Tensor, group) -> Pending:
    """Start a SUM all-reduce of ``t`` (in place) without ordering the caller after it."""
    if group is None or world(group) == 1:
        return Pending(t)
    c = _xgmi.route(group, t, "all_reduce", t.numel() * t.element_size()) if t.is_contiguous() else None
    if c is not None:
        return _on_side(t, lambda: c.all_reduce_(t))
    return Pending(t, work=dist.all_reduce(t, group=group, async_op=True))


def reduce_scatter_dim0_async(t: torch.Tensor, group) -> Pending:
    n = world(group)
    if n == 1:
        return Pending(t)
    assert t.shape[0] % n == 0
    t = t.contiguous()
    c = _xgmi.route(group, t, "reduce_scatter", t.numel() * t.element_size())
    if c is not None:
        def go():
            o = torch.empty((t.shape[0] // n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            return c.reduce_scatter(o, t)
        return _on_side(t, go)
    out = torch.empty((t.shape[0] // n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    return Pending(out, work=dist.reduce_scatter_tensor(out, t, group=group, async_op=True))


def all_gather_dim0_async(t: torch.Tensor, group) -> Pending:
    n = world(group)
    if n == 1:
        return Pending(t)
    t = t.contiguous()
    out = torch.empty((t.shape[0] * n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    c = _xgmi.route(group, t, "all_gather", out.numel() * out.element_size())
    if c is not None:
        return _on_side(t, lambda: c.all_gather(out, t))
    return Pending(out, work=dist.all_gather_into_tensor(out, t, group=group, async_op=True))
