"""BERT encoder + sequence-classification head on mxtrain's HIP kernels.

Workload parity: the reference fine-tunes `bert-base-cased` with
`AutoModelForSequenceClassification` on GLUE MRPC through Accelerate
(examples/accelerate/bert-glue-mrpc/pretrain.yaml:42-51) and the Ray
Lightning sample does the same (examples/ray/lightning-bert/fine-tune.yaml:49).

MI355X-first structure (post-LN BERT layer, token-major [B*S, h] activations):

  qkv = x Wqkv^T + b            one fused QKV GEMM (hipBLASLt)
  ctx = flash-attn(q, k, v)      HIP kernel, non-causal, key-padding mask as per-sequence
                                 valid length (K2)
  x1  = LN(x + drop(ctx Wo^T + bo))      fused bias-dropout-add-LN (HIP, K3/K7)
  f   = gelu(x1 W1^T + b1)               fused bias-GeLU (HIP, K6)
  x2  = LN(x1 + drop(f W2^T + b2))       fused BDA-LN

Parameters are fp32 masters (AMP style: compute in bf16 on the GPU, autograd returns
fp32 grads), named like Hugging Face's BertForSequenceClassification except for the
fused query/key/value weight; ``load_hf_state_dict`` / ``hf_state_dict`` convert.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import _lib
from ..ops.attention import flash_attention
from ..ops.fused import bias_gelu
from ..ops.norm import bda_norm, layer_norm
from ..ops.rng import DropoutSeed


@dataclass
class BertConfig:
    vocab_size: int = 28996          # bert-base-cased
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1   # applied to P inside the flash kernels
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02
    num_labels: int = 2
    pad_token_id: int = 0

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads


BERT_CONFIGS = {
    "bert-base-cased": dict(),
    "bert-base-uncased": dict(vocab_size=30522),
    "bert-large-cased": dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                             intermediate_size=4096),
    "bert-tiny": dict(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=512,
                      vocab_size=1024, max_position_embeddings=128),
}


def _c(t: torch.Tensor, dt) -> torch.Tensor:
    return t if t.dtype == dt else t.to(dt)


class BertLayer(nn.Module):
    def __init__(self, cfg: BertConfig, index: int):
        super().__init__()
        h, f = cfg.hidden_size, cfg.intermediate_size
        self.cfg, self.index = cfg, index
        self.qkv_weight = nn.Parameter(torch.empty(3 * h, h))
        self.qkv_bias = nn.Parameter(torch.zeros(3 * h))
        self.attn_out_weight = nn.Parameter(torch.empty(h, h))
        self.attn_out_bias = nn.Parameter(torch.zeros(h))
        self.ln1_weight = nn.Parameter(torch.ones(h))
        self.ln1_bias = nn.Parameter(torch.zeros(h))
        self.fc1_weight = nn.Parameter(torch.empty(f, h))
        self.fc1_bias = nn.Parameter(torch.zeros(f))
        self.fc2_weight = nn.Parameter(torch.empty(h, f))
        self.fc2_bias = nn.Parameter(torch.zeros(h))
        self.ln2_weight = nn.Parameter(torch.ones(h))
        self.ln2_bias = nn.Parameter(torch.zeros(h))

    def forward(self, x, B, S, klen, p, seed_t, dt, pa=0.0):
        cfg = self.cfg
        H, D = cfg.num_attention_heads, cfg.head_dim
        h = cfg.hidden_size
        qkv = F.linear(x, _c(self.qkv_weight, dt), _c(self.qkv_bias, dt))
        q, k, v = qkv[:, :h], qkv[:, h:2 * h], qkv[:, 2 * h:]
        ctx = flash_attention(q, k, v, B, S, H, H, D, causal=False, klen=klen, scale=1.0 / math.sqrt(D),
                              dropout_p=pa, seed_t=seed_t, salt=30011 + self.index)
        a = F.linear(ctx, _c(self.attn_out_weight, dt))
        salt = 101 + 2 * self.index
        x1 = bda_norm(a, _c(self.attn_out_bias, dt), x, _c(self.ln1_weight, dt), _c(self.ln1_bias, dt),
                      cfg.layer_norm_eps, p, seed_t, salt)
        u = F.linear(x1, _c(self.fc1_weight, dt))
        g = bias_gelu(u, _c(self.fc1_bias, dt))
        o = F.linear(g, _c(self.fc2_weight, dt))
        return bda_norm(o, _c(self.fc2_bias, dt), x1, _c(self.ln2_weight, dt), _c(self.ln2_bias, dt),
                        cfg.layer_norm_eps, p, seed_t, salt + 1)


class BertForSequenceClassification(nn.Module):
    def __init__(self, cfg: BertConfig, seed: int = 1234):
        super().__init__()
        self.cfg = cfg
        h = cfg.hidden_size
        self.word_embeddings = nn.Parameter(torch.empty(cfg.vocab_size, h))
        self.position_embeddings = nn.Parameter(torch.empty(cfg.max_position_embeddings, h))
        self.token_type_embeddings = nn.Parameter(torch.empty(cfg.type_vocab_size, h))
        self.emb_ln_weight = nn.Parameter(torch.ones(h))
        self.emb_ln_bias = nn.Parameter(torch.zeros(h))
        self.layers = nn.ModuleList([BertLayer(cfg, i) for i in range(cfg.num_hidden_layers)])
        self.pooler_weight = nn.Parameter(torch.empty(h, h))
        self.pooler_bias = nn.Parameter(torch.zeros(h))
        self.classifier_weight = nn.Parameter(torch.empty(cfg.num_labels, h))
        self.classifier_bias = nn.Parameter(torch.zeros(cfg.num_labels))
        self._seed0 = seed
        self.dropout_seed: Optional[DropoutSeed] = None
        self.reset_parameters(seed)

    def reset_parameters(self, seed: int = 1234):
        g = torch.Generator().manual_seed(seed)
        std = self.cfg.initializer_range
        for name, p in self.named_parameters():
            if name.endswith("bias"):
                continue
            if "ln" in name.split(".")[-1]:
                continue
            with torch.no_grad():
                p.copy_(torch.randn(p.shape, generator=g) * std)
        with torch.no_grad():
            self.word_embeddings[self.cfg.pad_token_id].zero_()

    def _seed(self, device):
        if self.dropout_seed is None or self.dropout_seed.t.device != device:
            self.dropout_seed = DropoutSeed(device, self._seed0)
        return self.dropout_seed

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, labels=None):
        """input_ids [B, S] (right-padded); attention_mask [B, S] 1 = token, 0 = pad.
        Returns a dict with ``logits`` [B, num_labels] (fp32) and ``loss`` if labels."""
        cfg = self.cfg
        B, S = input_ids.shape
        dev = input_ids.device
        dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
        if dev.type == "cuda":
            _lib.lib()   # fail loudly if the HIP kernels are missing
        if attention_mask is None:
            klen = torch.full((B,), S, dtype=torch.int32, device=dev)
        else:
            klen = attention_mask.sum(-1).to(torch.int32)
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        pos = torch.arange(S, device=dev)
        e = (F.embedding(input_ids, self.word_embeddings) + self.position_embeddings[pos][None]
             + F.embedding(token_type_ids, self.token_type_embeddings))
        x = layer_norm(_c(e.reshape(B * S, -1), dt), _c(self.emb_ln_weight, dt), _c(self.emb_ln_bias, dt),
                       cfg.layer_norm_eps)
        p = cfg.hidden_dropout_prob if self.training else 0.0
        if p > 0:
            x = F.dropout(x, p, True)
        seed = self._seed(dev)
        if self.training:
            seed.advance()
        pa = cfg.attention_probs_dropout_prob if self.training else 0.0
        for layer in self.layers:
            x = layer(x, B, S, klen, p, seed.t, dt, pa)
        cls = x.view(B, S, -1)[:, 0]
        pooled = torch.tanh(F.linear(cls, _c(self.pooler_weight, dt), _c(self.pooler_bias, dt)))
        if p > 0:
            pooled = F.dropout(pooled, p, True)
        logits = F.linear(pooled, _c(self.classifier_weight, dt), _c(self.classifier_bias, dt)).float()
        out = {"logits": logits}
        if labels is not None:
            out["loss"] = F.cross_entropy(logits, labels)
        return out

    # ---------------------------------------------------------------- HF interop
    def hf_state_dict(self) -> Dict[str, torch.Tensor]:
        h = self.cfg.hidden_size
        sd = {"bert.embeddings.word_embeddings.weight": self.word_embeddings,
              "bert.embeddings.position_embeddings.weight": self.position_embeddings,
              "bert.embeddings.token_type_embeddings.weight": self.token_type_embeddings,
              "bert.embeddings.LayerNorm.weight": self.emb_ln_weight,
              "bert.embeddings.LayerNorm.bias": self.emb_ln_bias,
              "bert.pooler.dense.weight": self.pooler_weight, "bert.pooler.dense.bias": self.pooler_bias,
              "classifier.weight": self.classifier_weight, "classifier.bias": self.classifier_bias}
        for i, L in enumerate(self.layers):
            p = f"bert.encoder.layer.{i}."
            for j, n in enumerate(("query", "key", "value")):
                sd[p + f"attention.self.{n}.weight"] = L.qkv_weight[j * h:(j + 1) * h]
                sd[p + f"attention.self.{n}.bias"] = L.qkv_bias[j * h:(j + 1) * h]
            sd.update({p + "attention.output.dense.weight": L.attn_out_weight,
                       p + "attention.output.dense.bias": L.attn_out_bias,
                       p + "attention.output.LayerNorm.weight": L.ln1_weight,
                       p + "attention.output.LayerNorm.bias": L.ln1_bias,
                       p + "intermediate.dense.weight": L.fc1_weight, p + "intermediate.dense.bias": L.fc1_bias,
                       p + "output.dense.weight": L.fc2_weight, p + "output.dense.bias": L.fc2_bias,
                       p + "output.LayerNorm.weight": L.ln2_weight, p + "output.LayerNorm.bias": L.ln2_bias})
        return {k: v.detach().clone() for k, v in sd.items()}

    def load_hf_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        mine = self.hf_state_dict()
        missing = [k for k in mine if k not in sd]
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:5]}...")
        h = self.cfg.hidden_size
        with torch.no_grad():
            def put(dst, key, sl=None):
                if key in sd:
                    (dst if sl is None else dst[sl]).copy_(sd[key])
            put(self.word_embeddings, "bert.embeddings.word_embeddings.weight")
            put(self.position_embeddings, "bert.embeddings.position_embeddings.weight")
            put(self.token_type_embeddings, "bert.embeddings.token_type_embeddings.weight")
            put(self.emb_ln_weight, "bert.embeddings.LayerNorm.weight")
            put(self.emb_ln_bias, "bert.embeddings.LayerNorm.bias")
            put(self.pooler_weight, "bert.pooler.dense.weight")
            put(self.pooler_bias, "bert.pooler.dense.bias")
            put(self.classifier_weight, "classifier.weight")
            put(self.classifier_bias, "classifier.bias")
            for i, L in enumerate(self.layers):
                p = f"bert.encoder.layer.{i}."
                for j, n in enumerate(("query", "key", "value")):
                    put(L.qkv_weight, p + f"attention.self.{n}.weight", slice(j * h, (j + 1) * h))
                    put(L.qkv_bias, p + f"attention.self.{n}.bias", slice(j * h, (j + 1) * h))
                for attr, key in (("attn_out_weight", "attention.output.dense.weight"),
                                  ("attn_out_bias", "attention.output.dense.bias"),
                                  ("ln1_weight", "attention.output.LayerNorm.weight"),
                                  ("ln1_bias", "attention.output.LayerNorm.bias"),
                                  ("fc1_weight", "intermediate.dense.weight"), ("fc1_bias", "intermediate.dense.bias"),
                                  ("fc2_weight", "output.dense.weight"), ("fc2_bias", "output.dense.bias"),
                                  ("ln2_weight", "output.LayerNorm.weight"), ("ln2_bias", "output.LayerNorm.bias")):
                    put(getattr(L, attr), p + key)
