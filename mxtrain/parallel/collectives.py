"""Thin collective helpers used by TP / SP / PP / DP code (RCCL on GPU, gloo on CPU).

All tensors are token-major ([tokens, hidden]); sequence parallelism shards the token
dimension, so SP all-gather / reduce-scatter work on dim 0 and are single contiguous
RCCL calls (no transposes, one kernel per call).
"""
from __future__ import annotations

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
