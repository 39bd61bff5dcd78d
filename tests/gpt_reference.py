"""Independent plain-PyTorch GPT used as the autograd oracle for mxtrain's hand-written
layer backward (fp32, no fusion, torch SDPA math)."""
import math

import torch
import torch.nn.functional as F


def gelu_tanh(x):
    return 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))


def rope_complex(x, rd, base):
    """Independent RoPE oracle: rotate-half as a complex multiply on (x[i], x[i+rd/2])."""
    B_, H_, S_, D_ = x.shape
    half = rd // 2
    inv = 1.0 / (base ** (torch.arange(0, rd, 2, dtype=torch.float64) / rd))
    ang = torch.arange(S_, dtype=torch.float64)[:, None] * inv[None, :]
    rot = torch.polar(torch.ones_like(ang), ang).to(torch.complex64)
    z = torch.complex(x[..., :half], x[..., half:rd]) * rot
    return torch.cat([z.real, z.imag, x[..., rd:]], -1)


def ref_loss(P, ids, labels, cfg, B, S, head="wte", mlp_hook=None, attn_keep=None):
    """attn_keep(i) -> (keep [B, H, S, S] bool, scale): attention-dropout mask of layer i."""
    h = cfg.hidden_size
    nh = cfg.num_attention_heads
    D = h // nh
    eps = cfg.layernorm_epsilon
    x = P["wte"][ids]
    if "wpe" in P:
        x = x + P["wpe"][torch.arange(B * S) % S]

    def ln(t, pre):
        if cfg.normalization == "rmsnorm":
            return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + eps) * P[pre + "_w"]
        return F.layer_norm(t, (h,), P[pre + "_w"], P[pre + "_b"], eps)

    for i in range(cfg.num_layers):
        p = f"layers.{i}."
        a = ln(x, p + "ln1")
        qkv = a @ P[p + "qkv_w"].t() + P[p + "qkv_b"]
        kvh = cfg.num_kv_heads
        q, k, v = qkv.split([h, kvh * D, kvh * D], dim=-1)
        q = q.view(B, S, nh, D).transpose(1, 2)
        k = k.view(B, S, kvh, D).transpose(1, 2)
        v = v.view(B, S, kvh, D).transpose(1, 2)
        if cfg.position_embedding == "rope":
            rd = int(D * cfg.rotary_percent) // 8 * 8
            q = rope_complex(q, rd, cfg.rotary_base)
            k = rope_complex(k, rd, cfg.rotary_base)
        if kvh != nh:
            k = k.repeat_interleave(nh // kvh, 1)
            v = v.repeat_interleave(nh // kvh, 1)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(D)
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float("-inf"))
        prob = torch.softmax(s, -1)
        if attn_keep is not None:
            keep, ks = attn_keep(i)
            prob = prob * keep.float() * ks
        ctx = (prob @ v).transpose(1, 2).reshape(B * S, h)
        x = x + ctx @ P[p + "proj_w"].t() + P[p + "proj_b"]
        m = ln(x, p + "ln2")
        if mlp_hook is not None and (p + "router_w") in P:
            x = x + mlp_hook(m, i)
            continue
        pre = m @ P[p + "fc1_w"].t() + P[p + "fc1_b"]
        if getattr(cfg, "swiglu", False):
            a_, b_ = pre.chunk(2, dim=-1)
            f = F.silu(a_) * b_
        else:
            f = gelu_tanh(pre)
        x = x + f @ P[p + "fc2_w"].t() + P[p + "fc2_b"]
    xf = ln(x, "final_ln")
    logits = xf @ P[head].t()
    return F.cross_entropy(logits, labels)
