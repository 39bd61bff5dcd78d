"""Megatron-style GPT (GPT-2 345M / GPT-3 6.7B configs) built on mxtrain's HIP kernels.

Workload parity: Megatron-DeepSpeed `pretrain_gpt.py` GPT model as configured by
examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-zero1.yaml:39-53 (24 layers, hidden
1024, 16 heads, seq 1024, learned positions, pre-LN, tied embeddings, GeLU MLP, hidden
dropout 0.1) and the TP2/PP2 variant (pretrain-ddp-tp-pp-zero1.yaml:39-40).

MI355X-first structure: each transformer layer is ONE autograd Function with a
hand-scheduled forward and backward:

  fwd: qkv = a Wqkv^T + b (hipBLASLt, bias epilogue) -> flash-attn (HIP, MFMA)
       -> o = ctx Wo^T -> [h1, m] = BDA-LN(o, bo, h) (HIP: bias+dropout+residual+LN
       in one pass) -> pre = m W1^T -> f = bias-GeLU(pre) (HIP) -> g = f W2^T
       -> [h2, a_next] = BDA-LN(g, b2, h1) with the NEXT layer's LN1 (or the final LN)
  bwd: the mirror image; weight gradients are written straight into the flat bf16
       gradient buffer with beta=1 GEMMs (Megatron "gradient accumulation fusion"),
       bias/LN gradients come out of the fused backward kernels' column reductions,
       and the layer reports completion so its gradient bucket's reduce-scatter can
       start while earlier layers are still in backward.

Tensor parallelism (Megatron column/row split: QKV+fc1 column-parallel, proj+fc2
row-parallel, vocab-parallel embedding/CE) and sequence parallelism (LN/dropout on
token shards with all-gather / reduce-scatter instead of all-reduce) are built in.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch

from .. import ops
from ..ops import attention as attn_ops
from ..ops.norm import bda_norm_fwd, colsum, colsum_finalize, colsum_partials_buffer, layernorm_fwd, norm_bwd
from ..ops.gemm import linear_dgrad, linear_fwd, nt_fits, wgrad_group
from ..ops.rope import apply_rope_
from ..ops.fused import (bias_gelu_bwd, bias_gelu_fwd, bias_swiglu_bwd, bias_swiglu_fwd,
                         cross_entropy_fwd_bwd, embed_bwd, embed_fwd, pos_embed_bwd)
from ..parallel import collectives as C
from ..parallel.buffers import ParamSpec
from ..parallel.ulysses import head_to_seq, seq_to_head
from .moe import is_moe_layer, moe_mlp


# QKV bias gradient from the attention backward kernels' column partials (module switch for
# A/B runs: scripts/bisect_deferred.py)
FUSED_QKV_BIAS_GRAD = True


@dataclass
class GPTConfig:
    num_layers: int = 24
    hidden_size: int = 1024
    num_attention_heads: int = 16
    num_kv_heads: Optional[int] = None
    ffn_hidden_size: Optional[int] = None
    vocab_size: int = 50257
    make_vocab_size_divisible_by: int = 128
    seq_length: int = 1024
    max_position_embeddings: int = 1024
    hidden_dropout: float = 0.1
    attention_dropout: float = 0.1         # Megatron default (--attention-dropout 0.1)
    layernorm_epsilon: float = 1e-5
    init_method_std: float = 0.02
    normalization: str = "layernorm"       # layernorm | rmsnorm
    position_embedding: str = "learned"    # learned | rope
    rotary_percent: float = 1.0
    swiglu: bool = False                   # fc1 -> [a | b], silu(a) * b (Megatron --swiglu)
    # Mixture of Experts (Megatron-DeepSpeed MoE flags; models/moe.py)
    num_experts: int = 0                   # <= 1: dense MLP everywhere
    expert_interval: int = 2               # MoE MLP in every expert_interval-th layer
    moe_topk: int = 1
    moe_train_capacity_factor: float = 1.0
    moe_eval_capacity_factor: float = 1.0
    moe_min_capacity: int = 4
    moe_loss_coeff: float = 0.01
    rotary_base: float = 10000.0
    tie_embeddings: bool = True
    # Megatron --recompute-activations / --checkpoint-activations (granularity "full"): each
    # layer keeps only its inputs and re-runs its forward inside its backward
    recompute: bool = False

    def __post_init__(self):
        if self.ffn_hidden_size is None:
            self.ffn_hidden_size = 4 * self.hidden_size
        if self.num_kv_heads is None:
            self.num_kv_heads = self.num_attention_heads

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    def padded_vocab(self, tp: int = 1) -> int:
        m = self.make_vocab_size_divisible_by * tp
        return (self.vocab_size + m - 1) // m * m

    def num_params(self, tp: int = 1) -> int:
        h, f, L = self.hidden_size, self.ffn_hidden_size, self.num_layers
        V = self.padded_vocab(tp)
        kvh = self.num_kv_heads * self.head_dim
        f1 = 2 * f if self.swiglu else f
        per_layer = (2 * h + (h * (h + 2 * kvh) + h + 2 * kvh) + (h * h + h) + 2 * h
                     + (h * f1 + f1) + (f * h + h))
        if self.normalization == "rmsnorm":
            per_layer -= 2 * h
        n = V * h + L * per_layer + 2 * h
        if self.position_embedding == "learned":
            n += self.max_position_embeddings * h
        if not self.tie_embeddings:
            n += V * h
        return n

    def flops_per_token(self) -> float:
        """Megatron/MFU convention: 6N + 12*L*h*s (fwd+bwd, no recompute)."""
        return 6.0 * self.num_params() + 12.0 * self.num_layers * self.hidden_size * self.seq_length


GPT_CONFIGS = {
    "gpt2-345m": dict(num_layers=24, hidden_size=1024, num_attention_heads=16, seq_length=1024,
                      max_position_embeddings=1024),
    "gpt3-6.7b": dict(num_layers=32, hidden_size=4096, num_attention_heads=32, seq_length=2048,
                      max_position_embeddings=2048),
    "gpt-tiny": dict(num_layers=2, hidden_size=128, num_attention_heads=2, seq_length=64,
                     max_position_embeddings=64, vocab_size=1000),
}

SALT_EMB = 7
SALT_ATTN = 50000   # + layer index; the attention mask is keyed on GLOBAL heads, so no TP term
# + GLOBAL micro-batch index x MICRO_SALT: every micro-batch of a step draws fresh dropout
# masks (Megatron draws a new mask on every call).  The index is global over data-parallel
# ranks (dp_rank x micro-batches per step + m) and hidden-dropout masks are keyed on global
# element indices (sequence-parallel shards offset by their rows), so the masks -- and the
# whole training trajectory -- do not depend on the DP / TP / SP / PP layout: a DP2 x TP2 x
# PP2 run draws the bits of the one-GPU run with the same micro-batches
MICRO_SALT = 0x2545F491
M32 = 0xFFFFFFFF
_NORM_PARAMS = ("ln1_w", "ln1_b")


# ============================================================================== specs
def stage_layer_range(cfg: GPTConfig, pp: int, pp_rank: int):
    per = cfg.num_layers // pp
    extra = cfg.num_layers % pp
    start = pp_rank * per + min(pp_rank, extra)
    n = per + (1 if pp_rank < extra else 0)
    return start, start + n


def gpt_param_specs(cfg: GPTConfig, tp: int = 1, pp: int = 1, pp_rank: int = 0,
                    sequence_parallel: bool = False) -> List[ParamSpec]:
    """Parameter specs for one (tp, pp) stage.  unit = backward-completion unit:
    0 = embedding (+ layer0.ln1), i+1 = layer i (+ the next layer's ln1 / final LN)."""
    h = cfg.hidden_size
    D = cfg.head_dim
    hl = cfg.num_attention_heads // tp
    kvl = cfg.num_kv_heads // tp
    fl = cfg.ffn_hidden_size // tp
    f1l = 2 * fl if cfg.swiglu else fl
    V = cfg.padded_vocab(tp) // tp
    std = cfg.init_method_std
    rms = cfg.normalization == "rmsnorm"
    sp = sequence_parallel and tp > 1
    l0, l1 = stage_layer_range(cfg, pp, pp_rank)
    first, last = pp_rank == 0, pp_rank == pp - 1
    specs: List[ParamSpec] = []

    def norm(prefix, unit):
        specs.append(ParamSpec(f"{prefix}_w", (h,), "ones", weight_decay=False, unit=unit,
                               sp_reduce=sp))
        if not rms:
            specs.append(ParamSpec(f"{prefix}_b", (h,), "zeros", weight_decay=False, unit=unit,
                                   sp_reduce=sp))

    if first:
        specs.append(ParamSpec("wte", (V, h), std=std, unit=0, tp_duplicated=False,
                               shared="word_embeddings"))
        if cfg.position_embedding == "learned":
            specs.append(ParamSpec("wpe", (cfg.max_position_embeddings, h), std=std, unit=0))
    for i in range(l0, l1):
        u = i + 1
        if i == l0:
            # the stage's first layer owns its LN1 (computed by embedding or its own Fn)
            # LN1 of the stage's first layer: computed by EmbedFn (first stage) or NormFn,
            # finishes backward last on this stage -> unit l0 (== 0 on the first stage)
            norm(f"layers.{i}.ln1", l0)
        p = f"layers.{i}."
        nd = False
        specs += [
            ParamSpec(p + "qkv_w", ((hl + 2 * kvl) * D, h), std=std, unit=u, tp_duplicated=nd),
            ParamSpec(p + "qkv_b", ((hl + 2 * kvl) * D,), "zeros", weight_decay=False, unit=u,
                      tp_duplicated=nd),
            ParamSpec(p + "proj_w", (h, hl * D), "scaled_normal", std=std, unit=u,
                      tp_duplicated=nd),
            ParamSpec(p + "proj_b", (h,), "zeros", weight_decay=False, unit=u, sp_reduce=sp),
        ]
        norm(p + "ln2", u)
        if is_moe_layer(cfg, i):
            specs.append(ParamSpec(p + "router_w", (cfg.num_experts, h), std=std, unit=u))
        else:
            specs += [
                ParamSpec(p + "fc1_w", (f1l, h), std=std, unit=u, tp_duplicated=nd),
                ParamSpec(p + "fc1_b", (f1l,), "zeros", weight_decay=False, unit=u, tp_duplicated=nd),
                ParamSpec(p + "fc2_w", (h, fl), "scaled_normal", std=std, unit=u, tp_duplicated=nd),
                ParamSpec(p + "fc2_b", (h,), "zeros", weight_decay=False, unit=u, sp_reduce=sp),
            ]
        if i + 1 < l1:
            norm(f"layers.{i + 1}.ln1", u)
        elif last:
            norm("final_ln", u)
    if last and (not first or not cfg.tie_embeddings):
        name = "wte_head" if cfg.tie_embeddings else "lm_head"
        specs.append(ParamSpec(name, (V, h), std=std, unit=l1, tp_duplicated=False,
                               shared="word_embeddings" if cfg.tie_embeddings else None))
    return specs


def shard_gpt_state(global_sd: Dict[str, torch.Tensor], cfg: GPTConfig, tp: int = 1,
                    tp_rank: int = 0, pp: int = 1, pp_rank: int = 0) -> Dict[str, torch.Tensor]:
    """Map an unsharded (tp=1, pp=1) GPT state dict onto one (tp_rank, pp_rank) stage:
    column-parallel weights (qkv, fc1, vocab) split on dim 0, row-parallel weights (proj,
    fc2) on dim 1, everything else replicated; the tied LM head of a later pipeline stage
    is a copy of the word embedding.  Used for TP/PP parity tests and checkpoint
    re-partitioning."""
    D = cfg.head_dim
    H, KV = cfg.num_attention_heads, cfg.num_kv_heads
    hl, kvl = H // tp, KV // tp
    r = tp_rank
    out = {}
    for spec in gpt_param_specs(cfg, tp, pp, pp_rank):
        name = spec.name
        src = "wte" if name in ("wte_head",) else name
        t = global_sd[src]
        base = name.split(".")[-1]
        if base in ("wte", "wte_head", "lm_head") or name in ("wte", "wte_head", "lm_head"):
            V = spec.shape[0]
            tt = torch.zeros(V * tp, t.shape[1], dtype=t.dtype)
            tt[: t.shape[0]] = t[: V * tp]
            t = tt[r * V:(r + 1) * V]
        elif base in ("qkv_w", "qkv_b"):
            q = t[: H * D]
            k = t[H * D:(H + KV) * D]
            v = t[(H + KV) * D:]
            t = torch.cat([q[r * hl * D:(r + 1) * hl * D], k[r * kvl * D:(r + 1) * kvl * D],
                           v[r * kvl * D:(r + 1) * kvl * D]], 0)
        elif base in ("fc1_w", "fc1_b") and cfg.swiglu:
            # column-parallel [a | b]: every rank keeps matching slices of both halves
            fh = t.shape[0] // 2
            n = fh // tp
            t = torch.cat([t[r * n:(r + 1) * n], t[fh + r * n:fh + (r + 1) * n]], 0)
        elif base in ("fc1_w", "fc1_b"):
            n = t.shape[0] // tp
            t = t[r * n:(r + 1) * n]
        elif base in ("proj_w", "fc2_w"):
            n = t.shape[1] // tp
            t = t[:, r * n:(r + 1) * n]
        out[name] = t.clone()
        assert tuple(out[name].shape) == tuple(spec.shape), (name, out[name].shape, spec.shape)
    return out


# ============================================================================== runtime
@dataclass
class StepRuntime:
    """Per-model runtime handed to the autograd Functions (non-tensor state)."""
    cfg: GPTConfig
    params: Dict[str, torch.Tensor]
    grads: Dict[str, torch.Tensor]
    B: int = 1
    S: int = 1
    tp_group: Optional[object] = None
    tp: int = 1
    tp_rank: int = 0
    sp: bool = False
    cp: int = 1                   # Ulysses context parallel: tokens here are S/cp of each sequence
    cp_rank: int = 0
    cp_group: Optional[object] = None
    seed_t: Optional[torch.Tensor] = None
    attn_seed_t: Optional[torch.Tensor] = None   # attention-dropout seed (shared across CP ranks)
    training: bool = True
    vocab_start: int = 0
    unit_done: Optional[Callable[[int], None]] = None
    before_unit: Optional[Callable[[int], None]] = None   # wait for the unit's params (AG overlap)
    grad_scale: float = 1.0       # loss gradient scale (1 / tokens / microbatches)
    # the first micro-batch of a step WRITES the weight gradients (GEMM beta = 0) instead of
    # accumulating into a zero-filled buffer (set by the trainer, which then zeroes only the
    # other gradients)
    wgrad_overwrite: bool = False
    # MoE: this rank's experts (separate flat buffer), the EP group, aux-loss gradient
    eparams: Optional[Dict[str, torch.Tensor]] = None
    egrads: Optional[Dict[str, torch.Tensor]] = None
    ep_group: Optional[object] = None
    aux_scale: float = 0.0        # d(total loss)/d(l_aux of one layer) = coeff / micro-batches
    aux_log: Optional[List] = None
    # TP communication overlap (MXTRAIN_TP_OVERLAP, default on): the row-parallel dgrad's
    # all-reduce / reduce-scatter runs asynchronously while the layer's weight-gradient
    # GEMMs run; under SP the all-gather feeding a column-parallel GEMM overlaps the GEMM
    # of this rank's own token chunk (the other chunks' GEMMs follow the gather)
    tp_overlap: bool = True
    sp_gemm_overlap: bool = True
    # deferred column reductions (ops/norm.py ColReduceQueue: LN / bias gradients folded in one
    # launch at the end of backward); set by the trainer when no per-bucket gradient
    # reduction runs during backward (one DP rank, no TP / PP)
    colq: Optional[object] = None
    # attention-dropout masks of every layer of the stage for the current step (generated in
    # one launch before the first layer; reset by the trainer at each step start)
    dmasks: Optional[List] = None
    dmask_l0: int = 0
    dmask_key: Optional[tuple] = None
    batch_dmasks: bool = False    # GPTTrainer turns it on (it resets dmasks when the seed advances)
    micro: int = 0                # micro-batch index within the step (dropout-mask key)
    micro_base: int = 0           # global index of this rank's first micro-batch of the step
    # forward / dgrad GEMMs of the layer through csrc/gemm_nt.hip with the bias, bias-GeLU
    # and GeLU' + bias-gradient epilogues fused (ops/gemm.py linear_fwd / linear_dgrad);
    # False: hipBLASLt + the separate bias-GeLU kernels (the LM head always uses hipBLASLt)
    fused_linear: bool = True

    @property
    def p_drop(self):
        return self.cfg.hidden_dropout if self.training else 0.0

    @property
    def p_attn(self):
        return self.cfg.attention_dropout if self.training else 0.0

    @property
    def rms(self):
        return self.cfg.normalization == "rmsnorm"

    def rope_(self, x, hl, kvl, inverse=False):
        """RoPE (K5) in place on the Q and K blocks of a packed [T, (hl+2kvl)*D] buffer
        holding whole sequences (under context parallelism: after the Ulysses exchange)."""
        cfg = self.cfg
        if cfg.position_embedding != "rope":
            return
        D = cfg.head_dim
        rd = int(D * cfg.rotary_percent) // 8 * 8
        for col0, nh in ((0, hl), (hl * D, kvl)):
            apply_rope_(x, col0, nh, D, self.S * self.cp, rd, cfg.rotary_base,
                        max_pos=cfg.max_position_embeddings, inverse=inverse)

    def norm_params(self, prefix):
        w = self.params[prefix + "_w"]
        b = self.params.get(prefix + "_b")
        return w, b

    def norm_grads(self, prefix):
        return self.grads[prefix + "_w"], self.grads.get(prefix + "_b")

    def wgrad(self, *items):
        """gbuf (+)= dy^T x for every (gbuf, dy, x) -- one grouped MFMA launch
        (ops/gemm.py: the layer's weight gradients that become ready together).  Written
        (beta = 0) on the first micro-batch when ``wgrad_overwrite``."""
        wgrad_group(items, accumulate=not self.wgrad_overwrite)

    def done(self, unit):
        if self.unit_done is not None:
            self.unit_done(unit)

    def need(self, unit):
        if self.before_unit is not None:
            self.before_unit(unit)

    def salt(self, base, micro=None):
        m = self.micro if micro is None else micro
        return (base + MICRO_SALT * (self.micro_base + m)) & M32

    def attn_salt(self, layer, micro=None):
        m = self.micro if micro is None else micro
        return (SALT_ATTN + layer + MICRO_SALT * (self.micro_base + m)) & M32

    def elem0(self, rows: int) -> int:
        """Global flat index of element [0, 0] of this rank's [rows, hidden] activation
        shard: under sequence parallelism rank r holds rows r*rows.. of the TP group's
        tokens, so its hidden-dropout mask is that part of the unsharded mask."""
        return self.tp_rank * rows * self.cfg.hidden_size if self.sp else 0


def _gather(x, rt):
    return C.all_gather_dim0(x, rt.tp_group) if rt.sp else x


def _reduce(x, rt):
    """Row-parallel output combine: reduce-scatter under SP, all-reduce under TP."""
    if rt.tp == 1:
        return x
    if rt.sp:
        return C.reduce_scatter_dim0(x, rt.tp_group)
    return C.all_reduce_(x, rt.tp_group)


def _reduce_start(x, rt):
    """Start the row-parallel combine of ``x`` (a dgrad partial sum); ``.wait()`` gives the
    result.  Synchronous (done on return) unless ``rt.tp_overlap``."""
    if rt.tp == 1:
        return C.Pending(x)
    if not rt.tp_overlap:
        return C.Pending(_reduce(x, rt))
    if rt.sp:
        return C.reduce_scatter_dim0_async(x, rt.tp_group)
    return C.all_reduce_async(x, rt.tp_group)


def _mm(a, w, trans=True, bias=None, out=None, fused=False):
    """a @ W^T (+ bias) (``trans=False``: a @ W, the dgrad of a Linear): through the
    hand-written MFMA GEMM with the bias in its epilogue when ``fused`` and the size is one
    where it wins (ops/gemm.py nt_fits), else hipBLASLt."""
    if fused and a.is_cuda and not nt_fits(a.shape[0], w.shape[0] if trans else w.shape[1], a.shape[1]):
        fused = False
    if fused:
        if trans:
            return linear_fwd(a, w, bias, out=out)
        assert bias is None
        return linear_dgrad(a, w, out=out)
    b = w.t() if trans else w
    if out is None:
        return torch.addmm(bias, a, b) if bias is not None else torch.mm(a, b)
    if bias is None:
        return torch.mm(a, b, out=out)
    return torch.addmm(bias, a, b, out=out)


def _mm_into(out, a, w, trans, bias=None, fused=False):
    _mm(a, w, trans, bias, out=out, fused=fused)


def _gather_mm(x, w, rt, trans=True, bias=None, fused=None):
    """(x_full, x_full @ W^T [+ bias]) (``trans=False``: @ W) for a column-parallel GEMM
    whose input is sequence-parallel: with ``rt.sp_gemm_overlap`` the token-chunk GEMM of
    this rank runs while the all-gather brings the other chunks, then the rest."""
    fused = rt.fused_linear if fused is None else fused
    if not rt.sp:
        return x, _mm(x, w, trans, bias, fused=fused)
    if not rt.sp_gemm_overlap:
        x_full = _gather(x, rt)
        return x_full, _mm(x_full, w, trans, bias, fused=fused)
    pend = C.all_gather_dim0_async(x, rt.tp_group)
    c, r, n = x.shape[0], rt.tp_rank, rt.tp
    y = torch.empty((c * n, w.shape[0] if trans else w.shape[1]), dtype=x.dtype, device=x.device)
    _mm_into(y[r * c:(r + 1) * c], x, w, trans, bias, fused)
    x_full = pend.wait()
    if r > 0:
        _mm_into(y[:r * c], x_full[:r * c], w, trans, bias, fused)
    if r < n - 1:
        _mm_into(y[(r + 1) * c:], x_full[(r + 1) * c:], w, trans, bias, fused)
    return x_full, y


def _wgrad(gbuf, dy, x):
    """gbuf += dy^T x (beta=1 GEMM straight into the flat gradient buffer)."""
    wgrad_group([(gbuf, dy, x)], accumulate=True)


# ============================================================================== Functions
class EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, ids, rt: StepRuntime, first_layer: int):
        P = rt.params
        # vocab-parallel: every TP rank gathers its vocab shard and the shards are summed
        # by the all-reduce, so the (replicated) position table is added by rank 0 only
        wpe = P.get("wpe") if rt.tp_rank == 0 else None
        e = embed_fwd(ids, P["wte"], wpe, seq=rt.S, vocab_start=rt.vocab_start,
                      pos_offset=rt.cp_rank * rt.S)
        if rt.tp > 1:
            C.all_reduce_(e, rt.tp_group)
            if rt.sp:
                e = C.split_dim0(e, rt.tp_group)
        w, b = rt.norm_params(f"layers.{first_layer}.ln1")
        h, a, mean, rstd = bda_norm_fwd(e, None, None, w, b, rt.cfg.layernorm_epsilon, rt.p_drop,
                                        rt.seed_t, rt.salt(SALT_EMB), rt.rms, elem0=rt.elem0(e.shape[0]))
        ctx.saved = (ids, h, mean, rstd)
        ctx.rt = rt
        ctx.micro = rt.micro
        ctx.first_layer = first_layer
        return h, a

    @staticmethod
    def backward(ctx, dh, da):
        rt = ctx.rt
        ids, h, mean, rstd = ctx.saved
        w, _ = rt.norm_params(f"layers.{ctx.first_layer}.ln1")
        gw, gb = rt.norm_grads(f"layers.{ctx.first_layer}.ln1")
        _, de = norm_bwd(da.contiguous(), dh.contiguous(), h, mean, rstd, w, want_dx=True,
                         p=rt.p_drop, seed_t=rt.seed_t, salt=rt.salt(SALT_EMB, ctx.micro), rms=rt.rms,
                         dgamma=gw, dbeta=gb, accumulate=True, defer=rt.colq, elem0=rt.elem0(da.shape[0]))
        if rt.sp:
            de = C.all_gather_dim0(de, rt.tp_group)
        embed_bwd(ids, de, rt.grads["wte"], rt.vocab_start)
        if "wpe" in rt.grads:
            off = rt.cp_rank * rt.S
            pos_embed_bwd(de, rt.grads["wpe"][off:off + rt.S], rt.B, rt.S)
        rt.done(0)
        ctx.saved = None
        return None, None, None, None


class NormFn(torch.autograd.Function):
    """Stand-alone LN1 for the first layer of a non-first pipeline stage."""

    @staticmethod
    def forward(ctx, h, rt: StepRuntime, prefix: str, unit: int):
        w, b = rt.norm_params(prefix)
        a, mean, rstd = layernorm_fwd(h, w, b, rt.cfg.layernorm_epsilon, rt.rms)
        ctx.saved = (h, mean, rstd)
        ctx.rt, ctx.prefix, ctx.unit = rt, prefix, unit
        return a

    @staticmethod
    def backward(ctx, da):
        rt = ctx.rt
        h, mean, rstd = ctx.saved
        w, _ = rt.norm_params(ctx.prefix)
        gw, gb = rt.norm_grads(ctx.prefix)
        dh, _ = norm_bwd(da.contiguous(), None, h, mean, rstd, w, rms=rt.rms, defer=rt.colq, dgamma=gw,
                         dbeta=gb, accumulate=True)
        ctx.saved = None
        rt.done(ctx.unit)
        return dh, None, None, None


class GPTLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, a, rt: StepRuntime, i: int, next_norm: Optional[str]):
        h2, a2, saved, dmask, moe = GPTLayerFn._forward_body(rt, i, next_norm, h, a, micro=rt.micro)
        ctx.rt, ctx.i, ctx.next_norm, ctx.micro = rt, i, next_norm, rt.micro
        if rt.cfg.recompute and rt.training:
            # activation recompute: keep the layer inputs only (the dropout masks are pure
            # functions of the step's seed, so the re-run forward is bit-identical)
            ctx.saved, ctx.dmask, ctx.moe = None, None, None
            ctx.inputs = (h.detach(), a.detach())
        else:
            ctx.saved, ctx.dmask, ctx.moe = saved, dmask, moe
            ctx.inputs = None
        if next_norm is None:
            return h2, torch.empty(0, device=h2.device, dtype=h2.dtype)
        return h2, a2

    @staticmethod
    def _forward_body(rt: StepRuntime, i: int, next_norm: Optional[str], h, a, recomputing=False, micro=0):
        cfg = rt.cfg
        P = rt.params
        p = f"layers.{i}."
        D = cfg.head_dim
        hl = cfg.num_attention_heads // rt.tp
        kvl = cfg.num_kv_heads // rt.tp
        eps = cfg.layernorm_epsilon
        dmask = None
        if rt.p_attn > 0 and rt.dmasks is not None and rt.dmask_key == (rt.B, rt.S, micro):
            # this micro-batch's masks, all layers at once
            dmask = rt.dmasks[i - rt.dmask_l0]
        elif rt.p_attn > 0:
            # (unbatched: this layer's keep-mask alone)
            ha_ = hl // rt.cp
            dmask = attn_ops.dropmask(rt.B, rt.S * rt.cp, ha_, rt.p_attn,
                                      rt.attn_seed_t if rt.attn_seed_t is not None else rt.seed_t,
                                      salt=rt.attn_salt(i, micro), head_offset=rt.tp_rank * hl + rt.cp_rank * ha_,
                                      total_heads=cfg.num_attention_heads, causal=True, device=a.device)
        a_full, qkv = _gather_mm(a, P[p + "qkv_w"], rt, bias=P[p + "qkv_b"])
        if rt.cp > 1:   # Ulysses: whole sequences, 1/cp of the heads
            qkv_a = seq_to_head(qkv, (hl * D, kvl * D, kvl * D), rt.B, rt.S, rt.cp_group)
            ha, kva = hl // rt.cp, kvl // rt.cp
        else:
            qkv_a, ha, kva = qkv, hl, kvl
        rt.rope_(qkv_a, ha, kva)
        q = qkv_a[:, : ha * D]
        k = qkv_a[:, ha * D:(ha + kva) * D]
        v = qkv_a[:, (ha + kva) * D:]
        ctx_a, lse, dmask = attn_ops.attn_fwd(q, k, v, rt.B, rt.S * rt.cp, ha, kva, D, causal=True,
                                              dmask=dmask)
        ctx_ = head_to_seq(ctx_a, (hl * D,), rt.B, rt.S, rt.cp_group) if rt.cp > 1 else ctx_a
        o = _reduce(_mm(ctx_, P[p + "proj_w"], fused=rt.fused_linear), rt)
        w2, b2 = rt.norm_params(p + "ln2")
        h1, m, mean2, rstd2 = bda_norm_fwd(o, P[p + "proj_b"], h, w2, b2, eps, rt.p_drop, rt.seed_t,
                                           rt.salt(1000 + 2 * i, micro), rt.rms, elem0=rt.elem0(o.shape[0]))
        moe = None
        if is_moe_layer(cfg, i):
            m_full = _gather(m, rt)
            # MoE MLP under autograd: the inner graph is kept for backward (models/moe.py)
            e = p + "experts."
            leaves = [P[p + "router_w"]] + [rt.eparams[e + n] for n in ("fc1_w", "fc1_b", "fc2_w", "fc2_b")]
            leaves = [t.detach().requires_grad_(True) for t in leaves]
            m_leaf = m_full.detach().requires_grad_(True)
            with torch.enable_grad():
                g_moe, l_aux, _ = moe_mlp(m_leaf, *leaves, cfg, rt.ep_group, training=rt.training)
            if rt.aux_log is not None and not recomputing:
                rt.aux_log.append(l_aux.detach())
            moe = (m_leaf, leaves, g_moe, l_aux)
            g = g_moe.detach()
            pre = f = None
            b_fc2 = None
        else:
            if (rt.fused_linear and not rt.sp and not cfg.swiglu
                    and (not m.is_cuda or nt_fits(m.shape[0], P[p + "fc1_w"].shape[0], m.shape[1]))):
                # fc1 GEMM + bias + GeLU in one kernel; pre = the biased pre-activation
                m_full = m
                f, pre = linear_fwd(m, P[p + "fc1_w"], P[p + "fc1_b"], gelu=True)
            else:
                m_full, pre = _gather_mm(m, P[p + "fc1_w"], rt)
                if cfg.swiglu:
                    f = bias_swiglu_fwd(pre, P[p + "fc1_b"])
                else:
                    f = bias_gelu_fwd(pre, P[p + "fc1_b"])
                    pre = (pre,)   # (un-biased pre-activation: backward adds the bias)
            g = _reduce(_mm(f, P[p + "fc2_w"], fused=rt.fused_linear), rt)
            b_fc2 = P[p + "fc2_b"]
        if next_norm is not None:
            wn, bn = rt.norm_params(next_norm)
        else:  # stage boundary: plain bias-dropout-add; normalise into a throwaway
            wn, bn = P[p + "ln2_w"], P.get(p + "ln2_b")
        h2, a2, mean_n, rstd_n = bda_norm_fwd(g, b_fc2, h1, wn, bn, eps, rt.p_drop,
                                              rt.seed_t, rt.salt(1001 + 2 * i, micro), rt.rms,
                                              elem0=rt.elem0(g.shape[0]))
        saved = (a_full, qkv_a, ctx_, ctx_a, lse, h1, mean2, rstd2, m_full, pre, f, h2, mean_n, rstd_n)
        return h2, a2, saved, dmask, moe

    @staticmethod
    def backward(ctx, dh2, da2):
        rt, i = ctx.rt, ctx.i
        cfg = rt.cfg
        P, G = rt.params, rt.grads
        p = f"layers.{i}."
        D = cfg.head_dim
        hl = cfg.num_attention_heads // rt.tp
        kvl = cfg.num_kv_heads // rt.tp
        if ctx.inputs is not None:   # activation recompute
            h_in, a_in = ctx.inputs
            ctx.inputs = None
            with torch.no_grad():
                _, _, ctx.saved, ctx.dmask, ctx.moe = GPTLayerFn._forward_body(rt, i, ctx.next_norm, h_in, a_in,
                                                                              recomputing=True, micro=ctx.micro)
        (a_full, qkv_a, ctx_, ctx_a, lse, h1, mean2, rstd2, m_full, pre, f, h2, mean_n, rstd_n) = ctx.saved
        ctx.saved = None
        dh2 = dh2.contiguous()
        # ---- BDA-LN(next) backward
        if ctx.next_norm is not None:
            wn, _ = rt.norm_params(ctx.next_norm)
            gwn, gbn = rt.norm_grads(ctx.next_norm)
            dh1, dg = norm_bwd(da2.contiguous(), dh2, h2, mean_n, rstd_n, wn, want_dx=True,
                               p=rt.p_drop, seed_t=rt.seed_t, salt=rt.salt(1001 + 2 * i, ctx.micro),
                               rms=rt.rms, dgamma=gwn, dbeta=gbn, dbias=G.get(p + "fc2_b"),
                               accumulate=True, defer=rt.colq, elem0=rt.elem0(dh2.shape[0]))
        else:
            wn = P[p + "ln2_w"]
            zero = torch.zeros_like(dh2)
            dh1, dg = norm_bwd(zero, dh2, h2, mean_n, rstd_n, wn, want_dx=True, p=rt.p_drop,
                               seed_t=rt.seed_t, salt=rt.salt(1001 + 2 * i, ctx.micro), rms=rt.rms,
                               dbias=G.get(p + "fc2_b"), accumulate=True, defer=rt.colq,
                               elem0=rt.elem0(dh2.shape[0]))
        # ---- MLP backward
        if ctx.moe is not None:
            m_leaf, leaves, g_moe, l_aux = ctx.moe
            ctx.moe = None
            outs, gos = [g_moe], [dg]
            if rt.aux_scale:
                outs.append(l_aux)
                gos.append(torch.full_like(l_aux, rt.aux_scale))
            grads = torch.autograd.grad(outs, [m_leaf] + leaves, gos)
            e = p + "experts."
            for gbuf, gr in zip([G[p + "router_w"]] + [rt.egrads[e + n] for n in ("fc1_w", "fc1_b", "fc2_w", "fc2_b")],
                                grads[1:]):
                gbuf.add_(gr.to(gbuf.dtype))
            dm = grads[0].to(dg.dtype)
            return GPTLayerFn._attn_backward(ctx, dm, dh1, a_full, qkv_a, ctx_, ctx_a, lse, h1, mean2, rstd2)
        if cfg.swiglu:
            dg_full, df = _gather_mm(dg, P[p + "fc2_w"], rt, trans=False)
            dpre = bias_swiglu_bwd(df, pre, P[p + "fc1_b"], dbias=G[p + "fc1_b"], accumulate=True)
        elif isinstance(pre, tuple):
            dg_full, df = _gather_mm(dg, P[p + "fc2_w"], rt, trans=False)
            dpre = bias_gelu_bwd(df, pre[0], P[p + "fc1_b"], dbias=G[p + "fc1_b"], accumulate=True,
                                 inplace=True, defer=rt.colq)
        else:
            # fc2 dgrad GEMM x GeLU'(pre) with the fc1 bias-gradient column sums in its epilogue
            dg_full = dg
            dpre = linear_dgrad(dg, P[p + "fc2_w"], gelu_aux=pre, dbias=G[p + "fc1_b"], accumulate=True,
                                defer=rt.colq)
        # dgrad first: its TP combine overlaps the fc2 + fc1 weight-gradient GEMMs (one
        # grouped launch, both operands read in place)
        pend = _reduce_start(_mm(dpre, P[p + "fc1_w"], trans=False, fused=rt.fused_linear), rt)
        rt.wgrad((G[p + "fc2_w"], dg_full, f), (G[p + "fc1_w"], dpre, m_full))
        dm = pend.wait()
        return GPTLayerFn._attn_backward(ctx, dm, dh1, a_full, qkv_a, ctx_, ctx_a, lse, h1, mean2, rstd2)

    @staticmethod
    def _attn_backward(ctx, dm, dh1, a_full, qkv_a, ctx_, ctx_a, lse, h1, mean2, rstd2):
        rt, i = ctx.rt, ctx.i
        cfg = rt.cfg
        P, G = rt.params, rt.grads
        p = f"layers.{i}."
        D = cfg.head_dim
        hl = cfg.num_attention_heads // rt.tp
        kvl = cfg.num_kv_heads // rt.tp
        # ---- BDA-LN2 backward
        w2, _ = rt.norm_params(p + "ln2")
        gw2, gb2 = rt.norm_grads(p + "ln2")
        dh, do_ = norm_bwd(dm, dh1, h1, mean2, rstd2, w2, want_dx=True, p=rt.p_drop,
                           seed_t=rt.seed_t, salt=rt.salt(1000 + 2 * i, ctx.micro), rms=rt.rms, dgamma=gw2,
                           dbeta=gb2, dbias=G[p + "proj_b"], accumulate=True, defer=rt.colq,
                           elem0=rt.elem0(dm.shape[0]))
        # ---- attention backward
        do_full, dctx = _gather_mm(do_, P[p + "proj_w"], rt, trans=False)
        if rt.cp > 1:
            dctx = seq_to_head(dctx, (hl * D,), rt.B, rt.S, rt.cp_group)
            ha, kva = hl // rt.cp, kvl // rt.cp
        else:
            ha, kva = hl, kvl
        dqkv = torch.empty_like(qkv_a)
        q = qkv_a[:, : ha * D]
        k = qkv_a[:, ha * D:(ha + kva) * D]
        v = qkv_a[:, (ha + kva) * D:]
        # QKV bias gradient: column partials straight from the attention backward kernels
        # when dqkv is final as they write it (no RoPE / context-parallel reshuffle after),
        # reduced by the deferred batched flush, or right away when there is no queue /
        # on its recording step -- the same partials and reduction either way
        gb = G[p + "qkv_b"]
        fused_bias = (FUSED_QKV_BIAS_GRAD and cfg.position_embedding != "rope" and rt.cp == 1
                      and rt.S % 32 == 0 and dqkv.is_cuda)
        bpart = pbuf = None
        if fused_bias:
            nparts, ncols = rt.B * rt.S // 32, dqkv.shape[1]
            if rt.colq is not None:
                bpart = rt.colq.partial((gb.data_ptr(),), (gb, None, None), nparts, ncols, 1, ncols, True)
            if bpart is not None:
                bpart = bpart.view(nparts, ncols)
            else:
                bpart, pbuf = colsum_partials_buffer(nparts, ncols, dqkv.device)
        attn_ops.attn_bwd(dctx, q, k, v, ctx_a, lse, rt.B, rt.S * rt.cp, ha, kva, D, causal=True,
                          dq=dqkv[:, : ha * D], dk=dqkv[:, ha * D:(ha + kva) * D],
                          dv=dqkv[:, (ha + kva) * D:], dmask=ctx.dmask, bias_partial=bpart)
        if pbuf is not None:
            colsum_finalize(pbuf, nparts, ncols, gb, accumulate=True)
        ctx.dmask = None
        rt.rope_(dqkv, ha, kva, inverse=True)
        if rt.cp > 1:
            dqkv = head_to_seq(dqkv, (hl * D, kvl * D, kvl * D), rt.B, rt.S, rt.cp_group)
        pend = _reduce_start(_mm(dqkv, P[p + "qkv_w"], trans=False, fused=rt.fused_linear), rt)
        if not fused_bias:
            colsum(dqkv, gb, accumulate=True, defer=rt.colq)
        rt.wgrad((G[p + "proj_w"], do_full, ctx_), (G[p + "qkv_w"], dqkv, a_full))
        da = pend.wait()
        rt.done(i + 1)
        return dh, da, None, None, None


class LMHeadLossFn(torch.autograd.Function):
    """logits = x W^T (vocab-parallel under TP) -> fused softmax-CE; the gradient is
    produced in the forward pass (in place over the logits)."""

    @staticmethod
    def forward(ctx, x, labels, rt: StepRuntime, wname: str):
        W = rt.params[wname]
        x_full, logits = _gather_mm(x, W, rt, fused=False)   # (hipBLASLt: 256-wide tiles win at V = 50k)
        losses = cross_entropy_fwd_bwd(logits, labels, rt.grad_scale,
                                       tp_group=rt.tp_group if rt.tp > 1 else None,
                                       vocab_start=rt.vocab_start)
        ctx.saved = (x_full, logits)
        ctx.rt, ctx.wname = rt, wname
        return losses.sum() * rt.grad_scale

    @staticmethod
    def backward(ctx, g):
        rt = ctx.rt
        x_full, dlogits = ctx.saved
        ctx.saved = None
        W = rt.params[ctx.wname]
        gv = g.reshape(1).to(x_full.dtype)
        pend = _reduce_start(torch.mm(dlogits, W) * gv, rt)
        wgrad_group([(rt.grads[ctx.wname], dlogits, x_full * gv)], accumulate=not rt.wgrad_overwrite)
        dx = pend.wait()
        return dx, None, None, None


# ============================================================================== model
class GPTStage:
    """The layers of one pipeline stage (all layers when pp == 1)."""

    def __init__(self, cfg: GPTConfig, params, grads, tp=1, tp_rank=0, tp_group=None, pp=1,
                 pp_rank=0, sequence_parallel=False, seed_t=None, cp=1, cp_rank=0, cp_group=None,
                 eparams=None, egrads=None, ep_group=None, attn_seed_t=None):
        self.cfg = cfg
        self.l0, self.l1 = stage_layer_range(cfg, pp, pp_rank)
        self.first, self.last = pp_rank == 0, pp_rank == pp - 1
        V = cfg.padded_vocab(tp) // tp
        self.rt = StepRuntime(cfg=cfg, params=params, grads=grads, tp_group=tp_group, tp=tp,
                              tp_rank=tp_rank, sp=sequence_parallel and tp > 1, seed_t=seed_t,
                              vocab_start=tp_rank * V, cp=cp, cp_rank=cp_rank, cp_group=cp_group,
                              eparams=eparams, egrads=egrads, ep_group=ep_group,
                              attn_seed_t=attn_seed_t)
        ov = os.environ.get("MXTRAIN_TP_OVERLAP", "1") == "1"
        self.rt.tp_overlap = self.rt.sp_gemm_overlap = ov
        if cfg.num_experts > 1:
            assert tp == 1, "MoE layers run with tensor-parallel size 1 (expert parallelism instead)"
        if cp > 1:
            assert (cfg.num_attention_heads // tp) % cp == 0 and (cfg.num_kv_heads // tp) % cp == 0, \
                "Ulysses needs the (per-TP-rank) query and KV head counts divisible by the cp size"
        self.anchor = torch.zeros(1, requires_grad=True)
        if self.last:
            if cfg.tie_embeddings:
                self.head_name = "wte" if self.first else "wte_head"
            else:
                self.head_name = "lm_head"


    def gemm_grad_names(self) -> List[str]:
        """Gradients written whole by the backward's weight-gradient GEMMs (GPTLayerFn /
        LMHeadLossFn): with ``rt.wgrad_overwrite`` the first micro-batch writes them with
        beta = 0, so the trainer's per-step zero-fill can skip them."""
        cfg = self.cfg
        names = []
        for i in range(self.l0, self.l1):
            if is_moe_layer(cfg, i):
                names.append(f"layers.{i}.proj_w")
                names.append(f"layers.{i}.qkv_w")
                continue
            names += [f"layers.{i}.{n}" for n in ("qkv_w", "proj_w", "fc1_w", "fc2_w")]
        if self.last:
            names.append(self.head_name)
        return names
    def forward(self, ids=None, hidden=None, labels=None, B=1, S=None, micro: int = 0):
        """First stage takes token ids [B*S]; later stages take the hidden state
        [tokens, h] (requires_grad).  Last stage returns the scalar loss, other stages
        the hidden state to send downstream."""
        rt = self.rt
        rt.B, rt.S = B, S or self.cfg.seq_length
        rt.micro = micro
        if self.first:
            rt.need(0)
            h, a = EmbedFn.apply(self.anchor, ids, rt, self.l0)
        else:
            h = hidden
            rt.need(self.l0)
            a = NormFn.apply(h, rt, f"layers.{self.l0}.ln1", self.l0)
        if rt.dmasks is not None and rt.dmask_key != (rt.B, rt.S, micro):
            rt.dmasks = None
        if (rt.p_attn > 0 and rt.batch_dmasks and rt.dmasks is None and self.l1 > self.l0
                and rt.seed_t is not None and rt.seed_t.is_cuda):
            rt.dmask_key = (rt.B, rt.S, micro)
            cfg = self.cfg
            hl = cfg.num_attention_heads // rt.tp
            ha_ = hl // rt.cp
            rt.dmask_l0 = self.l0
            rt.dmasks = attn_ops.dropmask_layers(rt.B, rt.S * rt.cp, ha_, rt.p_attn,
                                                 rt.attn_seed_t if rt.attn_seed_t is not None else rt.seed_t,
                                                 rt.attn_salt(self.l0, micro), self.l1 - self.l0,
                                                 head_offset=rt.tp_rank * hl + rt.cp_rank * ha_,
                                                 total_heads=cfg.num_attention_heads, causal=True)
        for i in range(self.l0, self.l1):
            if i + 1 < self.l1:
                nxt = f"layers.{i + 1}.ln1"
            elif self.last:
                nxt = "final_ln"
            else:
                nxt = None
            rt.need(i + 1)
            h, a = GPTLayerFn.apply(h, a, rt, i, nxt)
        if not self.last:
            return h
        return LMHeadLossFn.apply(a, labels, rt, self.head_name)
