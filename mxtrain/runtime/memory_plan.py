"""Per-rank HBM footprint of a GPT training configuration ("288 GB HBM
sizing"; BASELINE.json config 4: GPT-3 6.7B at TP=2 PP=2 DP=2 over xGMI, the reference's
examples/megatron-deepspeed/gpt3_6.7b/ pretrain-tp2-pp2-dp2 layout).

The numbers follow what THIS framework allocates, not a textbook formula:

* parameters / gradients: the exact numel of the rank's flat buffers (models/gpt.py
  ``gpt_param_specs`` for every pipeline stage; the largest stage is reported), both in the
  compute dtype (parallel/buffers.py keeps bf16 gradients);
* ZeRO-1 state: fp32 master + exp_avg + exp_avg_sq of a 1/(dp*cp) shard
  (parallel/zero.py ``DistributedOptimizer``);
* activations: the tensors ``GPTLayerFn._forward_body`` keeps for backward (its ``saved``
  tuple; the CPU test counts them on a real forward), the batched attention-dropout bit
  images, and the fp32 logits of the last stage, times the micro-batches a 1F1B stage
  holds at once (stage 0 holds ``pp`` of them).

``rank_memory`` returns a breakdown in bytes; ``fits`` compares it with the MI355X's
288 GB (minus a reserve for the allocator, RCCL buffers and workspaces)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

from ..models.gpt import GPTConfig, gpt_param_specs, stage_layer_range

HBM_BYTES = 288 * 10 ** 9
RESERVE_BYTES = 16 * 2 ** 30    # caching-allocator slack, RCCL / hipBLASLt workspaces, graph pools


@dataclass
class MemoryPlan:
    params: int
    grads: int
    optimizer: int
    activations: int
    logits: int
    dropout_masks: int
    detail: Dict[str, int] = field(default_factory=dict)

    @property
    def total(self) -> int:
        return self.params + self.grads + self.optimizer + self.activations + self.logits + self.dropout_masks

    def fits(self, hbm: int = HBM_BYTES, reserve: int = RESERVE_BYTES) -> bool:
        return self.total + reserve <= hbm

    def summary(self) -> Dict[str, float]:
        g = 1e9
        return {k: round(v / g, 3) for k, v in (("params_GB", self.params), ("grads_GB", self.grads),
                                               ("optimizer_GB", self.optimizer),
                                               ("activations_GB", self.activations), ("logits_GB", self.logits),
                                               ("dropout_masks_GB", self.dropout_masks),
                                               ("total_GB", self.total))}


def stage_numel(cfg: GPTConfig, tp: int, pp: int, pp_rank: int, sequence_parallel: bool = False) -> int:
    return sum(_numel(s.shape) for s in gpt_param_specs(cfg, tp, pp, pp_rank, sequence_parallel))


def _numel(shape) -> int:
    n = 1
    for d in shape:
        n *= int(d)
    return n


def layer_saved_bytes(cfg: GPTConfig, tokens: int, tp: int = 1, sequence_parallel: bool = False,
                      elt: int = 2) -> int:
    """Bytes ``GPTLayerFn`` keeps for backward for one dense layer and one micro-batch of
    ``tokens`` tokens (B * S): the saved tuple (a_full, qkv, ctx, lse, h1, mean2, rstd2,
    m_full, pre, f, h2, mean_n, rstd_n).  With sequence parallelism the residual stream
    and LN statistics are sequence-sharded; the gathered LN outputs are kept whole."""
    h = cfg.hidden_size
    D = cfg.head_dim
    hl = cfg.num_attention_heads // tp
    kvl = cfg.num_kv_heads // tp
    fl = cfg.ffn_hidden_size // tp
    f1l = 2 * fl if cfg.swiglu else fl
    s = tp if (sequence_parallel and tp > 1) else 1
    rms = cfg.normalization == "rmsnorm"
    per_tok = 0
    per_tok += h * elt                       # a_full: LN1 output as the QKV GEMM read it
    per_tok += (hl + 2 * kvl) * D * elt      # qkv (after RoPE)
    per_tok += hl * D * elt                  # attention context
    per_tok += hl * 4                        # softmax log-sum-exp (fp32)
    per_tok_sharded = 2 * h * elt            # h1, h2: residual stream
    per_tok_sharded += (1 if rms else 2) * 4 * 2   # (mean,) rstd of LN2 and the next norm (fp32)
    per_tok += h * elt                       # m_full: LN2 output as the fc1 GEMM read it
    per_tok += f1l * elt                     # pre-activation (fused GEMM aux / swiglu input)
    per_tok += fl * elt                      # activation output f (fc2's input)
    return tokens * per_tok + (tokens // s) * per_tok_sharded


def dropout_mask_bytes(cfg: GPTConfig, B: int, S: int, tp: int = 1) -> int:
    """Keep-mask images of one layer and micro-batch (ops/attention.py dropmask: a forward
    and a backward bit image, ~S*S/8 bytes each per (sequence, local head))."""
    if cfg.attention_dropout <= 0:
        return 0
    return B * (cfg.num_attention_heads // tp) * S * S // 4


def rank_memory(cfg: GPTConfig, tp: int = 1, pp: int = 1, dp: int = 1, micro_batch: int = 1,
                num_micro: Optional[int] = None, sequence_parallel: bool = False, cp: int = 1,
                elt: int = 2) -> MemoryPlan:
    """Largest per-rank footprint over the pipeline stages (bytes)."""
    S = cfg.seq_length
    tokens = micro_batch * S // cp
    best: Optional[MemoryPlan] = None
    nm = num_micro if num_micro is not None else pp
    for r in range(pp):
        n = stage_numel(cfg, tp, pp, r, sequence_parallel)
        l0, l1 = stage_layer_range(cfg, pp, r)
        inflight = min(nm, pp - r)           # 1F1B: stage r holds pp - r micro-batches
        act = (l1 - l0) * layer_saved_bytes(cfg, tokens, tp, sequence_parallel, elt) * inflight
        masks = (l1 - l0) * dropout_mask_bytes(cfg, micro_batch, S // cp, tp) * inflight
        # embedding output + first LN input of the stage boundary activation
        act += tokens * cfg.hidden_size * elt * inflight
        logits = 0
        if r == pp - 1:   # fp32 logits of one micro-batch (vocab-parallel CE keeps them for backward)
            logits = tokens * (cfg.padded_vocab(tp) // tp) * 4
        plan = MemoryPlan(params=n * elt, grads=n * elt, optimizer=(n * 12 + dp * cp - 1) // (dp * cp),
                          activations=act, logits=logits, dropout_masks=masks,
                          detail={"stage": r, "numel": n, "layers": l1 - l0, "inflight_micro": inflight})
        if best is None or plan.total > best.total:
            best = plan
    return best
