"""Mixture-of-Experts MLP with expert parallelism (Megatron-DeepSpeed MoE: ``--num-experts``,
``--moe-expert-parallel-size``, ``--topk``, ``--moe-train-capacity-factor``,
``--moe-min-capacity``, ``--moe-loss-coeff``, ``--expert-interval``).

Capacity-based routing, so every tensor has a static shape (the step stays capturable
in a hipGraph and the expert-parallel exchange is ONE equal-split all-to-all):

    logits = m Wg^T (fp32) -> softmax -> top-k experts per token
    capacity C = max(min_capacity, ceil(k * T / E * capacity_factor)); a token's k-th
        choice takes slot position cumsum-order in its expert (all first choices before
        second choices); positions >= C are dropped (the token keeps its residual)
    dispatch  [E, C, h] <- tokens            (index scatter)
    all-to-all over the EP group: [ep, E/ep, C, h]  (rank j gets every rank's slots of
        its E/ep experts)
    experts: batched GEMMs over the local experts: gelu(x W1^T + b1) W2^T + b2
    all-to-all back, combine: y[t] = sum_k gate[t, k] * out[slot(t, k)]
    l_aux = E * sum_e mean_t(probs[:, e]) * mean_t(top1_mask[:, e])   (load balancing)

Gating gates for k = 2 are renormalised over the kept choices (DeepSpeed top2gating).
The MoE MLP runs under torch autograd inside the GPT layer's hand-written Function (the
inner graph is built in forward, replayed in backward: no recompute); the aux-loss
gradient (coeff / micro-batches) is injected there, so the main loss needs no extra term
and pipeline stages need no extra output.

Expert parameters live in their own flat buffer: each rank holds E/ep experts, which
are replicated only across the expert-data-parallel group (grad_world / ep ranks), so
they have their own ZeRO-1 optimizer over that group; gradient clipping uses the joint
norm of dense + expert gradients (parallel/zero.py::joint_step).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..parallel.buffers import ParamSpec


def is_moe_layer(cfg, i: int) -> bool:
    return cfg.num_experts > 1 and (i + 1) % max(1, cfg.expert_interval) == 0


def moe_param_specs(cfg, l0: int, l1: int, ep: int) -> List[ParamSpec]:
    """Expert parameters of layers [l0, l1) for one EP rank (E/ep experts).  The router
    (replicated) stays in the dense buffer (see gpt_param_specs)."""
    h, f = cfg.hidden_size, cfg.ffn_hidden_size
    El = cfg.num_experts // ep
    std = cfg.init_method_std
    specs = []
    for i in range(l0, l1):
        if not is_moe_layer(cfg, i):
            continue
        p = f"layers.{i}.experts."
        u = i + 1
        specs += [ParamSpec(p + "fc1_w", (El, f, h), std=std, unit=u),
                  ParamSpec(p + "fc1_b", (El, f), "zeros", weight_decay=False, unit=u),
                  ParamSpec(p + "fc2_w", (El, h, f), "scaled_normal", std=std, unit=u),
                  ParamSpec(p + "fc2_b", (El, h), "zeros", weight_decay=False, unit=u)]
    return specs


class _AllToAll(torch.autograd.Function):
    """Equal-split all-to-all along dim 0 (its own transpose: backward = all-to-all)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        out = torch.empty_like(x)
        dist.all_to_all_single(out, x.contiguous(), group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        out = torch.empty_like(g)
        dist.all_to_all_single(out, g.contiguous(), group=ctx.group)
        return out, None


def all_to_all(x, group):
    if group is None or dist.get_world_size(group) == 1:
        return x
    return _AllToAll.apply(x, group)


def _gelu(x):
    return 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x * x * x)))


def route(logits: torch.Tensor, k: int, capacity: int):
    """Returns (slot [T,k] long in [0, E*C) or -1 if dropped, gate [T,k] fp32, l_aux,
    top1 expert fraction [E])."""
    T, E = logits.shape
    probs = torch.softmax(logits.float(), dim=-1)
    topv, topi = probs.topk(k, dim=-1)                              # [T, k]
    onehot = F.one_hot(topi, E)                                      # [T, k, E] int
    # slot positions: choice-major order (all first choices, then second choices)
    order = onehot.permute(1, 0, 2).reshape(k * T, E)
    loc = (torch.cumsum(order, 0) - 1).reshape(k, T, E).permute(1, 0, 2)  # [T, k, E]
    pos = (loc * onehot).sum(-1)                                     # [T, k]
    kept = pos < capacity
    slot = torch.where(kept, topi * capacity + pos, torch.full_like(pos, -1))
    gate = topv * kept
    if k > 1:
        gate = gate / gate.sum(-1, keepdim=True).clamp_min(torch.finfo(torch.float32).eps)
    me = probs.mean(0)
    ce = onehot[:, 0, :].float().mean(0)
    l_aux = E * (me * ce).sum()
    return slot, gate, l_aux, ce


def capacity(cfg, T: int, training: bool) -> int:
    cf = cfg.moe_train_capacity_factor if training else cfg.moe_eval_capacity_factor
    return max(int(cfg.moe_min_capacity), int(math.ceil(cfg.moe_topk * T / cfg.num_experts * cf)))


def moe_mlp(x: torch.Tensor, router_w: torch.Tensor, w1, b1, w2, b2, cfg, ep_group,
            training: bool = True) -> Tuple[torch.Tensor, torch.Tensor, Dict]:
    """x [T, h] -> y [T, h] (differentiable w.r.t. x, router and expert weights)."""
    T, h = x.shape
    E, k = cfg.num_experts, cfg.moe_topk
    ep = dist.get_world_size(ep_group) if ep_group is not None else 1
    El = E // ep
    C = capacity(cfg, T, training)
    logits = torch.mm(x.float(), router_w.float().t())             # router in fp32
    slot, gate, l_aux, frac = route(logits, k, C)
    # dispatch: [E*C + 1, h] with a trash row for dropped choices
    flat_slot = torch.where(slot >= 0, slot, torch.full_like(slot, E * C)).reshape(-1)   # [T*k]
    src = x.unsqueeze(1).expand(T, k, h).reshape(T * k, h)
    disp = torch.zeros(E * C + 1, h, dtype=x.dtype, device=x.device).index_copy(0, flat_slot, src)
    disp = disp[: E * C].view(ep, El * C, h)
    recv = all_to_all(disp, ep_group)                                # [ep(src), El*C, h]
    inp = recv.view(ep, El, C, h).permute(1, 0, 2, 3).reshape(El, ep * C, h)
    hid = _gelu(torch.baddbmm(b1.unsqueeze(1), inp, w1.transpose(1, 2)).float()).to(x.dtype)
    out = torch.baddbmm(b2.unsqueeze(1), hid, w2.transpose(1, 2))     # [El, ep*C, h]
    back = out.view(El, ep, C, h).permute(1, 0, 2, 3).reshape(ep, El * C, h)
    res = all_to_all(back, ep_group).reshape(E * C, h)
    res = torch.cat([res, torch.zeros(1, h, dtype=res.dtype, device=res.device)], 0)
    picked = res.index_select(0, flat_slot).view(T, k, h)
    y = (picked.float() * gate.unsqueeze(-1)).sum(1).to(x.dtype)
    # device tensors only (no host sync inside the step)
    stats = {"dropped_fraction": (slot < 0).float().mean().detach(), "expert_fraction": frac.detach()}
    return y, l_aux, stats
