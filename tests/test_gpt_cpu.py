"""The hand-written fused GPT layer backward must match PyTorch autograd exactly (fp32,
CPU reference path of every op, dropout off)."""
import torch

from mxtrain.models.gpt import GPTConfig, GPTStage, gpt_param_specs
from mxtrain.parallel.buffers import FlatParams
from gpt_reference import ref_loss


def _setup(cfg, B, S, seed=0):
    specs = gpt_param_specs(cfg)
    flat = FlatParams(specs, "cpu", torch.float32)
    flat.initialize(torch.Generator().manual_seed(seed), cfg.num_layers)
    # non-trivial LN/bias values
    g = torch.Generator().manual_seed(seed + 1)
    for s in specs:
        if s.init in ("ones", "zeros"):
            flat.params[s.name].add_(0.1 * torch.randn(s.shape, generator=g))
    ids = torch.randint(0, cfg.vocab_size, (B * S,), generator=g)
    labels = torch.randint(0, cfg.vocab_size, (B * S,), generator=g)
    return flat, ids, labels


def test_gpt_loss_and_grads_match_autograd():
    cfg = GPTConfig(num_layers=2, hidden_size=64, num_attention_heads=4, seq_length=16,
                    max_position_embeddings=16, vocab_size=100, hidden_dropout=0.0, attention_dropout=0.0)
    B, S = 2, 16
    flat, ids, labels = _setup(cfg, B, S)
    stage = GPTStage(cfg, flat.params, flat.grads)
    stage.rt.grad_scale = 1.0 / (B * S)
    loss = stage.forward(ids=ids, labels=labels, B=B, S=S)
    loss.backward()

    P = {n: p.detach().clone().requires_grad_(True) for n, p in flat.params.items()}
    ref = ref_loss(P, ids, labels, cfg, B, S)
    ref.backward()
    assert torch.allclose(loss, ref, atol=1e-5), (float(loss), float(ref))
    for n, p in P.items():
        g = flat.grads[n]
        assert torch.allclose(g, p.grad, atol=2e-5, rtol=1e-4), (n, (g - p.grad).abs().max())


def test_gpt_attention_dropout_matches_autograd():
    """Attention dropout 0.1 (Megatron default) through the CPU path of the flash op: the
    hand-written backward equals autograd of a plain softmax * keep / (1-p) attention."""
    from mxtrain.models.gpt import SALT_ATTN
    from mxtrain.ops.attention import dropout_keep_mask, effective_keep_scale
    cfg = GPTConfig(num_layers=2, hidden_size=64, num_attention_heads=4, seq_length=16,
                    max_position_embeddings=16, vocab_size=100, hidden_dropout=0.0, attention_dropout=0.1)
    B, S = 2, 16
    flat, ids, labels = _setup(cfg, B, S, seed=5)
    seed = torch.tensor([987], dtype=torch.int32)
    stage = GPTStage(cfg, flat.params, flat.grads, seed_t=seed, attn_seed_t=seed)
    stage.rt.grad_scale = 1.0 / (B * S)
    loss = stage.forward(ids=ids, labels=labels, B=B, S=S)
    loss.backward()
    P = {n: p.detach().clone().requires_grad_(True) for n, p in flat.params.items()}
    keep = lambda i: (dropout_keep_mask(B, S, 4, 987, SALT_ATTN + i, 0.1), effective_keep_scale(0.1))
    assert 0.05 < 1 - keep(0)[0].float().mean() < 0.15
    ref = ref_loss(P, ids, labels, cfg, B, S, attn_keep=keep)
    ref.backward()
    assert torch.allclose(loss, ref, atol=1e-5), (float(loss), float(ref))
    for n, p in P.items():
        assert torch.allclose(flat.grads[n], p.grad, atol=2e-5, rtol=1e-4), (n, (flat.grads[n] - p.grad).abs().max())


def test_gpt_rmsnorm_variant():
    cfg = GPTConfig(num_layers=2, hidden_size=64, num_attention_heads=4, seq_length=8,
                    max_position_embeddings=8, vocab_size=50, hidden_dropout=0.0, attention_dropout=0.0,
                    normalization="rmsnorm")
    B, S = 2, 8
    flat, ids, labels = _setup(cfg, B, S, seed=3)
    stage = GPTStage(cfg, flat.params, flat.grads)
    stage.rt.grad_scale = 1.0 / (B * S)
    loss = stage.forward(ids=ids, labels=labels, B=B, S=S)
    loss.backward()
    P = {n: p.detach().clone().requires_grad_(True) for n, p in flat.params.items()}
    ref = ref_loss(P, ids, labels, cfg, B, S)
    ref.backward()
    assert torch.allclose(loss, ref, atol=1e-5)
    for n, p in P.items():
        assert torch.allclose(flat.grads[n], p.grad, atol=2e-5, rtol=1e-4), n


def test_gpt_rope_gqa_variant():
    """RoPE (K5, partial rotary) + GQA + RMSNorm + SwiGLU (LLaMA-style)."""
    cfg = GPTConfig(num_layers=2, hidden_size=64, num_attention_heads=4, num_kv_heads=2,
                    seq_length=8, max_position_embeddings=8, vocab_size=50, hidden_dropout=0.0, attention_dropout=0.0,
                    normalization="rmsnorm", position_embedding="rope", rotary_percent=0.5,
                    swiglu=True, ffn_hidden_size=96)
    B, S = 2, 8
    flat, ids, labels = _setup(cfg, B, S, seed=5)
    assert "wpe" not in flat.params
    stage = GPTStage(cfg, flat.params, flat.grads)
    stage.rt.grad_scale = 1.0 / (B * S)
    loss = stage.forward(ids=ids, labels=labels, B=B, S=S)
    loss.backward()
    P = {n: p.detach().clone().requires_grad_(True) for n, p in flat.params.items()}
    ref = ref_loss(P, ids, labels, cfg, B, S)
    ref.backward()
    assert torch.allclose(loss, ref, atol=1e-5), (float(loss), float(ref))
    for n, p in P.items():
        assert torch.allclose(flat.grads[n], p.grad, atol=2e-5, rtol=1e-4), n


def test_rope_op_inverse_and_grad():
    from mxtrain.ops.rope import apply_rope_, rope
    T, H, D = 12, 3, 16
    x = torch.randn(T, H * D)
    y = x.clone()
    apply_rope_(y, 0, H, D, seq=6, rotary_dim=8)
    assert not torch.allclose(y, x)
    assert torch.allclose(y[:, 8:16], x[:, 8:16])     # un-rotated tail of head 0
    apply_rope_(y, 0, H, D, seq=6, rotary_dim=8, inverse=True)
    assert torch.allclose(y, x, atol=1e-6)
    xr = x.clone().requires_grad_(True)
    g = torch.randn(T, H * D)
    rope(xr, H, D, 6, 8).backward(g)
    xa = x.clone().requires_grad_(True)
    from gpt_reference import rope_complex
    ya = rope_complex(xa.view(2, 6, H, D).transpose(1, 2), 8, 10000.0).transpose(1, 2).reshape(T, H * D)
    ya.backward(g)
    assert torch.allclose(xr.grad, xa.grad, atol=1e-5)


def test_dropout_mask_reproducible():
    from mxtrain.ops.rng import keep_mask
    m1 = keep_mask(10000, 123, 0.1)
    m2 = keep_mask(10000, 123, 0.1)
    assert torch.equal(m1, m2)
    frac = 1 - m1.float().mean().item()
    assert 0.08 < frac < 0.12


def test_dropout_mask_stream_properties():
    """One hash per 8-element group + xorshift16 draws: drop rate within 0.5 % (relative)
    of p over 4M draws, any sub-range equals the slice of the full mask (the kernels index by
    absolute element), and neighbouring seeds / groups are uncorrelated."""
    from mxtrain.ops.rng import keep_mask, keep_threshold16
    n = 1 << 22
    for p in (0.1, 0.5):
        m = keep_mask(n, 99, p)
        rate = 1 - m.float().mean().item()
        assert abs(rate - p) < 0.005 * p, (p, rate)
        assert abs(keep_threshold16(p) / 65536 - p) < 2 ** -16
    full = keep_mask(1000, 7, 0.1)
    for base, cnt in ((3, 100), (8, 64), (517, 300)):
        assert torch.equal(keep_mask(cnt, 7, 0.1, base=base), full[base:base + cnt])
    a, b = keep_mask(n, 1, 0.5).float(), keep_mask(n, 2, 0.5).float()
    assert abs(((a - 0.5) * (b - 0.5)).mean().item()) < 2e-3
    # lag-1 and lag-8 autocorrelation within one stream
    for lag in (1, 2, 8):
        assert abs(((a[lag:] - 0.5) * (a[:-lag] - 0.5)).mean().item()) < 2e-3, lag


def test_activation_recompute_is_bit_identical():
    """--checkpoint-activations / --recompute-activations: each layer keeps only its inputs and
    re-runs its forward in backward; with dropout on, losses and gradients are unchanged."""
    B, S = 2, 16
    out = []
    for rc in (False, True):
        cfg = GPTConfig(num_layers=2, hidden_size=64, num_attention_heads=4, seq_length=16,
                        max_position_embeddings=16, vocab_size=100, hidden_dropout=0.1,
                        attention_dropout=0.1, recompute=rc)
        flat, ids, labels = _setup(cfg, B, S, seed=9)
        seed = torch.tensor([31], dtype=torch.int32)
        stage = GPTStage(cfg, flat.params, flat.grads, seed_t=seed, attn_seed_t=seed)
        stage.rt.grad_scale = 1.0 / (B * S)
        loss = stage.forward(ids=ids, labels=labels, B=B, S=S)
        loss.backward()
        out.append((float(loss), flat.grads))
    assert out[0][0] == out[1][0]
    for n in out[0][1]:
        assert torch.equal(out[0][1][n], out[1][1][n]), n


def test_first_micro_batch_overwrites_gemm_grads():
    """overwrite_wgrads: the first micro-batch's weight-gradient GEMMs write (beta = 0) and
    the per-step zero-fill clears only the other gradients -- same gradients and updates as
    zero-fill + accumulate, over two steps of two micro-batches with garbage left in the
    GEMM-written gradient ranges between steps."""
    from mxtrain.parallel import state as pstate
    from mxtrain.training import GPTTrainer, TrainConfig
    cfg = GPTConfig(num_layers=2, hidden_size=64, num_attention_heads=4, seq_length=16,
                    max_position_embeddings=16, vocab_size=128, hidden_dropout=0.0, attention_dropout=0.0)
    ps = pstate.initialize_model_parallel(device_type="cpu")
    g = torch.Generator().manual_seed(3)
    tokens = torch.randint(0, 128, (2, 2, 16), generator=g)
    labels = torch.randint(0, 128, (2, 2, 16), generator=g)
    runs = {}
    for ow in (False, True):
        tc = TrainConfig(micro_batch_size=2, global_batch_size=4, lr=1e-3, overwrite_wgrads=ow,
                         overlap_grad_reduce=False)
        tr = GPTTrainer(cfg, tc, ps, dtype=torch.float32)
        assert tr._overwrite == ow
        losses = []
        for _ in range(2):
            if ow:   # the overwritten ranges may hold anything before the step
                for n in tr.stage.gemm_grad_names():
                    tr.flat.grads[n].fill_(1e3)
            losses.append(float(tr.train_step(tokens, labels)))
        runs[ow] = (losses, {n: p.clone() for n, p in tr.flat.params.items()},
                    {n: p.clone() for n, p in tr.flat.grads.items()})
    assert runs[True][0] == runs[False][0]
    for n in runs[False][1]:
        assert torch.equal(runs[True][1][n], runs[False][1][n]), n
        assert torch.equal(runs[True][2][n], runs[False][2][n]), n


def test_each_micro_batch_draws_fresh_dropout_masks():
    """Gradient accumulation: micro-batches 0 and 1 of one step must not reuse the same
    hidden / attention dropout masks (Megatron draws a fresh mask on every call).  The same
    tokens fed as micro-batch 0 and micro-batch 1 give different losses; micro-batch 0 is
    unchanged against the un-indexed call (the bench's single micro-batch keeps its masks),
    and re-running micro-batch 1 (recompute / pipeline backward) reproduces it exactly."""
    from mxtrain.models.gpt import MICRO_SALT, SALT_ATTN
    from mxtrain.ops.attention import dropout_keep_mask
    cfg = GPTConfig(num_layers=2, hidden_size=64, num_attention_heads=4, seq_length=16,
                    max_position_embeddings=16, vocab_size=100, hidden_dropout=0.1, attention_dropout=0.1)
    B, S = 2, 16
    flat, ids, labels = _setup(cfg, B, S, seed=4)
    seed = torch.tensor([77], dtype=torch.int32)
    stage = GPTStage(cfg, flat.params, flat.grads, seed_t=seed, attn_seed_t=seed)
    stage.rt.grad_scale = 1.0 / (B * S)
    with torch.no_grad():
        l_plain = float(stage.forward(ids=ids, labels=labels, B=B, S=S))
        l0 = float(stage.forward(ids=ids, labels=labels, B=B, S=S, micro=0))
        l1 = float(stage.forward(ids=ids, labels=labels, B=B, S=S, micro=1))
        l1b = float(stage.forward(ids=ids, labels=labels, B=B, S=S, micro=1))
    assert l_plain == l0 and l1 == l1b and l0 != l1, (l_plain, l0, l1, l1b)
    rt = stage.rt
    assert rt.salt(1000, 0) != rt.salt(1000, 1) and rt.attn_salt(3, 0) == SALT_ATTN + 3
    m0 = dropout_keep_mask(B, S, 4, 77, rt.attn_salt(0, 0), 0.1)
    m1 = dropout_keep_mask(B, S, 4, 77, rt.attn_salt(0, 1), 0.1)
    assert not torch.equal(m0, m1) and rt.attn_salt(0, 1) == (SALT_ATTN + MICRO_SALT) & 0xFFFFFFFF
