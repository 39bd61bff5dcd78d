"""Numerics of every HIP kernel against the fp32 PyTorch reference of the same op.

The reference is the CPU path of the same mxtrain.ops function (plain fp32 torch), run on
the CPU copies of the GPU inputs.  Marked gpu: runs on an MI355X through gpurun.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from mxtrain import ops  # noqa: E402
from mxtrain.ops import attention as A  # noqa: E402
from mxtrain.ops import fused as Fu  # noqa: E402
from mxtrain.ops import norm as N  # noqa: E402
from mxtrain.ops import optim as O  # noqa: E402

DEV = "cuda"


def _close(a, b, atol, rtol=0.0, name=""):
    a = a.float().cpu()
    b = b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{name}: {bad} elements off, max err {err.max().item():.3e}"


def _bf(x):
    return x.to(torch.bfloat16)


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)
    assert torch.cuda.is_available()


@pytest.mark.parametrize("rows,cols", [(512, 768), (512, 1024), (4100, 1024), (512, 4096), (512, 8192),
                                       (256, 2600)])
def test_layernorm_fwd_bwd(rows, cols):
    x = _bf(torch.randn(rows, cols))
    g = _bf(1 + 0.1 * torch.randn(cols))
    b = _bf(0.1 * torch.randn(cols))
    dy = _bf(torch.randn(rows, cols))
    y, mean, rstd = N.layernorm_fwd(x.to(DEV), g.to(DEV), b.to(DEV))
    yr, meanr, rstdr = N.layernorm_fwd(x, g, b)
    _close(y, yr, 2e-2, 1e-2, "ln y")
    _close(mean, meanr, 1e-4, 0, "mean")
    _close(rstd, rstdr, 1e-3, 1e-3, "rstd")
    dg, db = torch.zeros(cols, dtype=torch.bfloat16, device=DEV), torch.zeros(cols, dtype=torch.bfloat16, device=DEV)
    dgr, dbr = torch.zeros(cols, dtype=torch.bfloat16), torch.zeros(cols, dtype=torch.bfloat16)
    dh, _ = N.norm_bwd(dy.to(DEV), None, x.to(DEV), mean, rstd, g.to(DEV), dgamma=dg, dbeta=db)
    dhr, _ = N.norm_bwd(dy, None, x, meanr, rstdr, g)
    N.norm_bwd(dy, None, x, meanr, rstdr, g, dgamma=dgr, dbeta=dbr)
    _close(dh, dhr, 3e-2, 2e-2, "ln dx")
    _close(dg, dgr, 0.5, 2e-2, "dgamma")
    _close(db, dbr, 0.5, 2e-2, "dbeta")


@pytest.mark.parametrize("rms,cols", [(False, 1024), (True, 1024), (False, 4096), (True, 5120)])
def test_bda_norm_with_dropout(rms, cols):
    rows = 256
    x = _bf(torch.randn(rows, cols))
    bias = _bf(0.1 * torch.randn(cols))
    res = _bf(torch.randn(rows, cols))
    g = _bf(1 + 0.1 * torch.randn(cols))
    b = _bf(0.1 * torch.randn(cols))
    seed = torch.tensor([4242], dtype=torch.int32)
    h, y, mean, rstd = N.bda_norm_fwd(x.to(DEV), bias.to(DEV), res.to(DEV), g.to(DEV), b.to(DEV),
                                      p=0.1, seed_t=seed.to(DEV), salt=5, rms=rms)
    hr, yr, meanr, rstdr = N.bda_norm_fwd(x, bias, res, g, b, p=0.1, seed_t=seed, salt=5, rms=rms)
    _close(h, hr, 2e-2, 1e-2, "h")  # identical masks -> only rounding differences
    _close(y, yr, 3e-2, 2e-2, "y")
    dy = _bf(torch.randn(rows, cols))
    dres = _bf(torch.randn(rows, cols))
    outs = [torch.zeros(cols, dtype=torch.bfloat16, device=DEV) for _ in range(3)]
    outr = [torch.zeros(cols, dtype=torch.bfloat16) for _ in range(3)]
    dh, dx = N.norm_bwd(dy.to(DEV), dres.to(DEV), h, mean, rstd, g.to(DEV), want_dx=True, p=0.1,
                        seed_t=seed.to(DEV), salt=5, rms=rms, dgamma=outs[0],
                        dbeta=None if rms else outs[1], dbias=outs[2])
    dhr, dxr = N.norm_bwd(dy, dres, hr, meanr, rstdr, g, want_dx=True, p=0.1, seed_t=seed,
                          salt=5, rms=rms, dgamma=outr[0], dbeta=None if rms else outr[1],
                          dbias=outr[2])
    _close(dh, dhr, 5e-2, 2e-2, "dh")
    _close(dx, dxr, 6e-2, 2e-2, "dx")
    _close(outs[0], outr[0], 1.0, 3e-2, "dgamma")
    _close(outs[2], outr[2], 1.0, 3e-2, "dbias")


@pytest.mark.parametrize("rows,cols", [(512, 4096), (300, 1000)])
def test_bias_gelu(rows, cols):
    x = _bf(torch.randn(rows, cols))
    b = _bf(0.1 * torch.randn(cols))
    y = Fu.bias_gelu_fwd(x.to(DEV), b.to(DEV))
    _close(y, Fu.bias_gelu_fwd(x, b), 2e-2, 1e-2, "gelu")
    dy = _bf(torch.randn(rows, cols))
    db = torch.zeros(cols, dtype=torch.bfloat16, device=DEV)
    dbr = torch.zeros(cols, dtype=torch.bfloat16)
    dx = Fu.bias_gelu_bwd(dy.to(DEV), x.to(DEV), b.to(DEV), dbias=db)
    dxr = Fu.bias_gelu_bwd(dy, x, b, dbias=dbr)
    _close(dx, dxr, 3e-2, 2e-2, "gelu dx")
    _close(db, dbr, 0.5, 2e-2, "gelu db")


def test_colsum():
    x = _bf(torch.randn(1000, 3072))
    out = torch.zeros(3072, dtype=torch.bfloat16, device=DEV)
    N.colsum(x.to(DEV), out)
    _close(out, x.float().sum(0), 0.3, 1e-2, "colsum")


def test_embedding_fwd_bwd():
    V, H, B, S = 1000, 256, 2, 128
    wte = _bf(torch.randn(V, H))
    wpe = _bf(torch.randn(S, H))
    ids = torch.randint(0, V, (B * S,))
    ids[:10] = 7  # repeated ids exercise the segmented reduction
    out = Fu.embed_fwd(ids.to(DEV), wte.to(DEV), wpe.to(DEV), seq=S)
    _close(out, Fu.embed_fwd(ids, wte, wpe, seq=S), 1e-2, 1e-2, "embed")
    dout = _bf(torch.randn(B * S, H))
    dw = torch.zeros(V, H, dtype=torch.bfloat16, device=DEV)
    dwr = torch.zeros(V, H, dtype=torch.bfloat16)
    Fu.embed_bwd(ids.to(DEV), dout.to(DEV), dw)
    Fu.embed_bwd(ids, dout, dwr)
    _close(dw, dwr, 5e-2, 1e-2, "embed bwd")
    dp = torch.zeros(S, H, dtype=torch.bfloat16, device=DEV)
    dpr = torch.zeros(S, H, dtype=torch.bfloat16)
    Fu.pos_embed_bwd(dout.to(DEV), dp, B, S)
    Fu.pos_embed_bwd(dout, dpr, B, S)
    _close(dp, dpr, 3e-2, 1e-2, "pos bwd")


@pytest.mark.parametrize("H,ntok,vocab_start", [(1024, 4096, 0), (4096, 2048, 0), (512, 1000, 300), (1024, 8192, 0)])
def test_embedding_bwd_sort_free(H, ntok, vocab_start):
    """csrc/fused.hip embed_bwd_scan_kernel (no torch.sort): repeated ids -- in runs, spread
    over the whole batch, across the 64-id scan chunks -- and ids outside a vocab shard,
    against the fp32 index_add reference; bit-reproducible from run to run; and the sort
    path it replaced (accumulation order may differ: bf16 tolerance)."""
    from mxtrain.ops import _lib
    V = 3000
    g = torch.Generator().manual_seed(H + ntok)
    ids = torch.randint(0, V + vocab_start, (ntok,), generator=g)
    ids[:70] = 5 + vocab_start            # a run across a chunk boundary
    ids[100::97] = 11 + vocab_start       # spread duplicates
    ids[-1] = 5 + vocab_start
    dout = _bf(torch.randn(ntok, H, generator=g))
    dw0 = _bf(torch.randn(V, H, generator=g) * 0.1)
    ref = dw0.clone()
    Fu.embed_bwd(ids, dout, ref, vocab_start=vocab_start)
    runs = []
    for _ in range(2):
        dw = dw0.to(DEV).clone()
        Fu.embed_bwd(ids.to(DEV), dout.to(DEV), dw, vocab_start=vocab_start)
        torch.cuda.synchronize()
        runs.append(dw.cpu())
    assert torch.equal(runs[0], runs[1])
    _close(runs[0], ref, 5e-2, 2e-2, "embed bwd (scan)")
    # the sort path (still used beyond the scan kernel's range)
    sdw = dw0.to(DEV).clone()
    sids, perm = torch.sort(ids.to(DEV))
    _lib.call("mx_embed_bwd", _lib.ptr(sids), _lib.ptr(perm), _lib.ptr(dout.to(DEV)), _lib.ptr(sdw), ntok, H,
              vocab_start, vocab_start + V, _lib.stream())
    _close(runs[0], sdw.cpu(), 5e-2, 2e-2, "scan vs sort")


def test_cross_entropy():
    rows, V = 256, 50304
    logits = _bf(3 * torch.randn(rows, V))
    labels = torch.randint(0, V, (rows,))
    labels[3] = -100
    lg = logits.to(DEV).clone()
    loss = Fu.cross_entropy_fwd_bwd(lg, labels.to(DEV), 1.0 / rows)
    lr = logits.clone().float()
    lossr = Fu.cross_entropy_fwd_bwd(lr, labels, 1.0 / rows)
    _close(loss, lossr, 2e-3, 1e-3, "ce loss")
    _close(lg, lr, 1e-4, 2e-2, "ce grad")


def test_adamw_and_norm():
    n = 64 * 1000
    master = torch.randn(n)
    grad = _bf(torch.randn(n))
    hyper = torch.tensor([1e-3, 0.9, 0.95, 1e-8, 0.1, 1 - 0.9, 1 - 0.95, 0.5, 1.0, 0.0])
    flags = (torch.arange(n // 64) % 3 != 0).to(torch.uint8)
    ns = O.sumsq_bf16(grad.to(DEV), 0.5, flags=flags.to(DEV))
    nsr = O.sumsq_bf16(grad, 0.5, flags=flags)
    _close(ns, nsr, 1e-1, 1e-4, "sumsq")
    m, v = torch.zeros(n), torch.zeros(n)
    md, vd, mad = m.to(DEV), v.to(DEV), master.to(DEV)
    pd = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    pr = torch.empty(n, dtype=torch.bfloat16)
    O.adamw_step(mad, md, vd, grad.to(DEV), pd, hyper.to(DEV), ns, flags.to(DEV))
    mr = master.clone()
    O.adamw_step(mr, m, v, grad, pr, hyper, nsr, flags)
    _close(mad, mr, 1e-6, 1e-5, "master")
    _close(pd, pr, 1e-2, 1e-2, "param")


ATTN_CASES = [
    # B, S, Hq, Hkv, D, causal, padded, dropout
    (2, 256, 4, 4, 64, True, False, 0.0),
    (1, 1024, 2, 2, 64, True, False, 0.0),
    (2, 128, 4, 4, 64, False, True, 0.0),
    (2, 200, 2, 2, 64, True, False, 0.0),
    (1, 256, 2, 2, 128, True, False, 0.0),
    (2, 128, 2, 2, 128, False, True, 0.0),
    # production GPT-3 6.7B head shape (S 2048, D 128, causal; single-pass 8-wave dK/dV)
    (1, 2048, 2, 2, 128, True, False, 0.0),
    # grouped-query attention (Hq != Hkv)
    (2, 512, 8, 2, 64, True, False, 0.0),
    (1, 512, 8, 2, 128, True, False, 0.0),
    # attention dropout (Megatron default 0.1): identical keep-mask in the reference
    (2, 256, 4, 4, 64, True, False, 0.1),
    (1, 1024, 2, 2, 64, True, False, 0.1),
    (2, 200, 2, 2, 64, True, False, 0.1),
    (2, 128, 4, 4, 64, False, True, 0.1),
    (1, 512, 4, 2, 128, True, False, 0.1),
    (2, 128, 2, 2, 128, False, True, 0.3),
    # D 128, causal, S not a multiple of the 128-key block (ragged single-pass dK/dV)
    (2, 200, 2, 2, 128, True, False, 0.1),
]


@pytest.mark.parametrize("B,S,Hq,Hkv,D,causal,padded,pdrop", ATTN_CASES)
def test_flash_attention_fwd_bwd(B, S, Hq, Hkv, D, causal, padded, pdrop):
    W = (Hq + 2 * Hkv) * D
    qkv = _bf(torch.randn(B * S, W))
    sl = (slice(0, Hq * D), slice(Hq * D, (Hq + Hkv) * D), slice((Hq + Hkv) * D, W))
    q, k, v = (qkv[:, c] for c in sl)
    klen = torch.tensor([S, S * 3 // 4][:B], dtype=torch.int32) if padded else None
    qkvd = qkv.to(DEV)
    qd, kd, vd = (qkvd[:, c] for c in sl)
    seed = torch.tensor([12345], dtype=torch.int32)
    kw = dict(dropout_p=pdrop, salt=77, head_offset=0, total_heads=Hq) if pdrop else {}
    o, lse, dm = A.attn_fwd(qd, kd, vd, B, S, Hq, Hkv, D, causal, klen.to(DEV) if padded else None,
                            seed_t=seed.to(DEV), **kw)
    orf, lser, dmr = A.attn_fwd(q, k, v, B, S, Hq, Hkv, D, causal, klen, seed_t=seed, **kw)
    _close(o, orf, 2e-2, 2e-2, "attn o")
    _close(lse, lser, 2e-3, 1e-3, "attn lse")
    do = _bf(torch.randn(B * S, Hq * D))
    dqkv = torch.empty_like(qkvd)
    A.attn_bwd(do.to(DEV), qd, kd, vd, o, lse, B, S, Hq, Hkv, D, causal,
               klen.to(DEV) if padded else None, dq=dqkv[:, sl[0]], dk=dqkv[:, sl[1]],
               dv=dqkv[:, sl[2]], dmask=dm, dropout_p=pdrop)
    dq, dk, dv = A.attn_bwd(do, q, k, v, orf, lser, B, S, Hq, Hkv, D, causal, klen, dmask=dmr,
                            dropout_p=pdrop)
    scale = max(dq.abs().max().item(), 1.0)
    _close(dqkv[:, sl[0]], dq, 3e-2 * scale, 3e-2, "dq")
    _close(dqkv[:, sl[1]], dk, 3e-2 * scale, 3e-2, "dk")
    _close(dqkv[:, sl[2]], dv, 3e-2 * scale, 3e-2, "dv")


@pytest.mark.parametrize("S,causal,pdrop,padded", [(1024, True, 0.1, False), (200, True, 0.0, False),
                                                   (256, False, 0.1, True)])
def test_flash_d128_single_pass_matches_two_pass(S, causal, pdrop, padded):
    """The single-pass 8-wave D 128 dK/dV kernel (S and dP once per subtile, exchanged
    through LDS) does the same fp32 operations in the same MFMA order as the two column-half
    passes, so dK / dV are bit-identical; dQ comes from the shared query-major kernel."""
    from mxtrain.ops import _lib
    B, H, D = 2, 4, 128
    torch.manual_seed(3)
    qkv = torch.randn(B * S, 3 * H * D, device=DEV).to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    do = torch.randn(B * S, H * D, device=DEV).to(torch.bfloat16)
    klen = torch.tensor([S, S * 3 // 4], dtype=torch.int32, device=DEV) if padded else None
    seed = torch.tensor([99], dtype=torch.int32, device=DEV)
    kw = dict(dropout_p=pdrop, salt=3, head_offset=0, total_heads=H) if pdrop else {}
    o, lse, dm = A.attn_fwd(q, k, v, B, S, H, H, D, causal, klen, seed_t=seed, **kw)
    outs = []
    old = _lib._fn("mx_flash_kmajor128_variant")(-1)
    try:
        for variant in (0, 1):   # single pass, two column-half passes
            _lib._fn("mx_flash_kmajor128_variant")(variant)
            dqkv = torch.zeros_like(qkv)
            A.attn_bwd(do, q, k, v, o, lse, B, S, H, H, D, causal, klen, dq=dqkv[:, :H * D],
                       dk=dqkv[:, H * D:2 * H * D], dv=dqkv[:, 2 * H * D:], dmask=dm, dropout_p=pdrop)
            torch.cuda.synchronize()
            outs.append(dqkv)
    finally:
        _lib._fn("mx_flash_kmajor128_variant")(old)
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("D,Hq,Hkv,pdrop", [(64, 4, 4, 0.1), (128, 4, 4, 0.1), (64, 8, 2, 0.0), (128, 4, 2, 0.0)])
def test_flash_bwd_bias_partials_are_column_sums(D, Hq, Hkv, pdrop):
    """The attention backward's QKV-bias partials (column sums of each 32-row group of
    [dq | dk | dv], from the kernels' fp32 accumulators) against sums of the bf16 outputs."""
    B, S = 2, 256
    torch.manual_seed(5)
    W = (Hq + 2 * Hkv) * D
    qkv = torch.randn(B * S, W, device=DEV).to(torch.bfloat16)
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    do = torch.randn(B * S, Hq * D, device=DEV).to(torch.bfloat16)
    seed = torch.tensor([11], dtype=torch.int32, device=DEV)
    kw = dict(dropout_p=pdrop, salt=2, head_offset=0, total_heads=Hq) if pdrop else {}
    o, lse, dm = A.attn_fwd(q, k, v, B, S, Hq, Hkv, D, True, None, seed_t=seed, **kw)
    dqkv = torch.zeros_like(qkv)
    part = torch.full((B * S // 32, W), float("nan"), device=DEV)
    A.attn_bwd(do, q, k, v, o, lse, B, S, Hq, Hkv, D, True, None, dq=dqkv[:, :Hq * D],
               dk=dqkv[:, Hq * D:(Hq + Hkv) * D], dv=dqkv[:, (Hq + Hkv) * D:], dmask=dm, dropout_p=pdrop,
               bias_partial=part)
    torch.cuda.synchronize()
    assert torch.isfinite(part).all()                       # every row / column written
    ref = dqkv.float().view(B * S // 32, 32, W).sum(1)
    scale = ref.abs().max().item()
    _close(part, ref, 2e-2 * scale + 1e-3, 1e-2, "bias partials")


def _crow(e, hh):
    return (e & 3) + 8 * (e >> 2) + 4 * hh


@pytest.mark.parametrize("S,causal", [(256, True), (200, False), (96, True), (320, False)])
def test_attention_dropout_mask_images(S, causal):
    """flash_dropmask_kernel's forward (query-on-lane) and backward (key-on-lane) bit images
    both decode to the reference keep-mask (dropout_keep_mask), and the drop rate is p."""
    B, Hq, p, salt = 2, 3, 0.1, 5
    NB = (S + 31) // 32
    seed = torch.tensor([424242], dtype=torch.int32, device=DEV)
    dm = A.dropmask(B, S, Hq, p, seed, salt, head_offset=1, total_heads=Hq + 2, causal=causal)
    torch.cuda.synchronize()
    ref = A.dropout_keep_mask(B, S, Hq, 424242, salt, p, head_offset=1, total_heads=Hq + 2)
    NKT, NQT = (S + 127) // 128, (S + 63) // 64
    fw = dm.fbits.cpu().view(B * Hq, NB, NKT, 64)
    bw = dm.bbits.cpu().view(B * Hq, NB, NQT, 64).to(torch.int64) & 0xFFFFFFFF
    P = NB * 32
    keepf = torch.zeros(B * Hq, P, P, dtype=torch.bool)
    keepb = torch.zeros(B * Hq, P, P, dtype=torch.bool)
    lane = torch.arange(64)
    for qb in range(NB):
        for kb in range(NB):
            if causal and kb > qb:
                continue
            wf = (fw[:, qb, kb // 4, :] >> (32 * ((kb & 3) >> 1))) & 0xFFFFFFFF     # [BH, 64]
            wb = bw[:, kb, qb // 2, :]
            for e in range(16):
                pf = 8 * (kb & 1) + 16 * (e & 1) + (e >> 1)
                pb = 8 * (qb & 1) + 16 * (e & 1) + (e >> 1)
                keepf[:, 32 * qb + (lane & 31), 32 * kb + _crow(e, lane >> 5)] = ((wf >> pf) & 1).bool()
                keepb[:, 32 * qb + _crow(e, lane >> 5), 32 * kb + (lane & 31)] = ((wb >> pb) & 1).bool()
    refp = ref.reshape(B * Hq, S, S)
    valid = torch.ones(S, S, dtype=torch.bool)
    if causal:
        valid = valid.tril()
    for got in (keepf[:, :S, :S], keepb[:, :S, :S]):
        assert torch.equal(got[:, valid], refp[:, valid])
    rate = 1.0 - refp[:, valid].float().mean().item()
    assert abs(rate - p) < 0.02, rate


def test_gpt_layer_gpu_matches_cpu_reference():
    """One full GPT stage step on the GPU (HIP kernels) vs the fp32 CPU path."""
    from mxtrain.models.gpt import GPTConfig, GPTStage, gpt_param_specs
    from mxtrain.parallel.buffers import FlatParams
    cfg = GPTConfig(num_layers=2, hidden_size=256, num_attention_heads=4, seq_length=128,
                    max_position_embeddings=128, vocab_size=512, hidden_dropout=0.0, attention_dropout=0.0)
    B, S = 2, 128
    specs = gpt_param_specs(cfg)
    fc = FlatParams(specs, "cpu", torch.float32)
    fc.initialize(torch.Generator().manual_seed(0), cfg.num_layers)
    fc.data.copy_(fc.data.to(torch.bfloat16).float())
    fg = FlatParams(specs, DEV, torch.bfloat16)
    fg.data.copy_(fc.data.to(torch.bfloat16))
    ids = torch.randint(0, cfg.vocab_size, (B * S,))
    labels = torch.randint(0, cfg.vocab_size, (B * S,))
    sc = GPTStage(cfg, fc.params, fc.grads)
    sg = GPTStage(cfg, fg.params, fg.grads)
    for st in (sc, sg):
        st.rt.grad_scale = 1.0 / (B * S)
    lc = sc.forward(ids=ids, labels=labels, B=B, S=S)
    lc.backward()
    lg = sg.forward(ids=ids.to(DEV), labels=labels.to(DEV), B=B, S=S)
    lg.backward()
    assert abs(float(lg) - float(lc)) < 2e-2, (float(lg), float(lc))
    for n in fc.grads:
        a, b = fg.grads[n].float().cpu(), fc.grads[n]
        rel = (a - b).norm() / (b.norm() + 1e-6)
        assert rel < 5e-2, (n, float(rel))


@pytest.mark.parametrize("H,KV,D,rd", [(16, 16, 64, 64), (8, 2, 128, 64), (4, 4, 128, 128)])
def test_rope_fwd_bwd(H, KV, D, rd):
    from mxtrain.ops.rope import apply_rope_
    B, S = 2, 256
    ld = (H + 2 * KV) * D
    x = _bf(torch.randn(B * S, ld))
    xd = x.to(DEV)
    for col0, nh in ((0, H), (H * D, KV)):
        apply_rope_(xd, col0, nh, D, S, rd, max_pos=S)
        apply_rope_(x, col0, nh, D, S, rd, max_pos=S)
    _close(xd, x, 2e-2, 1e-2, "rope fwd")
    y = xd.clone()
    for col0, nh in ((0, H), (H * D, KV)):
        apply_rope_(y, col0, nh, D, S, rd, max_pos=S, inverse=True)
        apply_rope_(x, col0, nh, D, S, rd, max_pos=S, inverse=True)
    _close(y, x, 2e-2, 1e-2, "rope inverse")
    # position ids override (e.g. packed / context-parallel shards)
    pid = torch.randint(0, 4096, (B * S,))
    z = _bf(torch.randn(B * S, H * D))
    zd = z.to(DEV)
    apply_rope_(zd, 0, H, D, S, rd, pos_ids=pid.to(DEV), max_pos=4096)
    apply_rope_(z, 0, H, D, S, rd, pos_ids=pid, max_pos=4096)
    _close(zd, z, 2e-2, 1e-2, "rope pos_ids")


def test_gpt_llama_style_layer_gpu_matches_cpu_reference():
    """RoPE + GQA + RMSNorm stage on the GPU (HIP kernels) vs the fp32 CPU path."""
    from mxtrain.models.gpt import GPTConfig, GPTStage, gpt_param_specs
    from mxtrain.parallel.buffers import FlatParams
    cfg = GPTConfig(num_layers=2, hidden_size=512, num_attention_heads=4, num_kv_heads=2,
                    seq_length=128, max_position_embeddings=128, vocab_size=512,
                    hidden_dropout=0.0, attention_dropout=0.0, normalization="rmsnorm", position_embedding="rope",
                    swiglu=True, ffn_hidden_size=1024)
    B, S = 2, 128
    specs = gpt_param_specs(cfg)
    fc = FlatParams(specs, "cpu", torch.float32)
    fc.initialize(torch.Generator().manual_seed(0), cfg.num_layers)
    fc.data.copy_(fc.data.to(torch.bfloat16).float())
    fg = FlatParams(specs, DEV, torch.bfloat16)
    fg.data.copy_(fc.data.to(torch.bfloat16))
    ids = torch.randint(0, cfg.vocab_size, (B * S,))
    labels = torch.randint(0, cfg.vocab_size, (B * S,))
    sc = GPTStage(cfg, fc.params, fc.grads)
    sg = GPTStage(cfg, fg.params, fg.grads)
    for st in (sc, sg):
        st.rt.grad_scale = 1.0 / (B * S)
    lc = sc.forward(ids=ids, labels=labels, B=B, S=S)
    lc.backward()
    lg = sg.forward(ids=ids.to(DEV), labels=labels.to(DEV), B=B, S=S)
    lg.backward()
    assert abs(float(lg.detach()) - float(lc.detach())) < 2e-2
    for n in fc.grads:
        a, b = fg.grads[n].float().cpu(), fc.grads[n]
        rel = (a - b).norm() / (b.norm() + 1e-6)
        assert rel < 5e-2, (n, float(rel))


@pytest.mark.parametrize("rows,f", [(512, 1024), (300, 2752)])
def test_bias_swiglu_fwd_bwd(rows, f):
    pre = _bf(torch.randn(rows, 2 * f))
    b = _bf(0.1 * torch.randn(2 * f))
    dy = _bf(torch.randn(rows, f))
    y = Fu.bias_swiglu_fwd(pre.to(DEV), b.to(DEV))
    _close(y, Fu.bias_swiglu_fwd(pre, b), 2e-2, 2e-2, "swiglu y")
    db = torch.zeros(2 * f, dtype=torch.bfloat16, device=DEV)
    dbr = torch.zeros(2 * f, dtype=torch.bfloat16)
    dp = Fu.bias_swiglu_bwd(dy.to(DEV), pre.to(DEV), b.to(DEV), dbias=db)
    dpr = Fu.bias_swiglu_bwd(dy, pre, b, dbias=dbr)
    _close(dp, dpr, 3e-2, 2e-2, "swiglu dpre")
    _close(db, dbr, 0.25, 2e-2, "swiglu dbias")


def test_graph_replay_matches_eager_with_flush():
    """hipGraph replays of the whole step (with a sync_params() flush mid-run, as eval /
    checkpointing do) give the eager trainer's losses, parameters and Adam moments bit for
    bit."""
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.parallel import state as pstate
    from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch
    ps = pstate.initialize_model_parallel()
    cfg = GPTConfig(num_layers=3, hidden_size=256, num_attention_heads=4, seq_length=256,
                    max_position_embeddings=256, vocab_size=1024)
    runs = []
    for graph in (False, True):
        tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=2, bucket_numel=400_000), ps)
        tok, lab = synthetic_batch(cfg, 1, 2, ps.device, torch.Generator().manual_seed(3))
        losses = [float(tr.train_step(tok, lab))]
        losses.append(float(tr.capture(tok, lab, warmup=1) if graph else tr.train_step(tok, lab)))
        losses += [float(tr.train_step(tok, lab)) for _ in range(2)]
        tr.sync_params()
        losses += [float(tr.train_step(tok, lab)) for _ in range(3)]
        torch.cuda.synchronize()
        tr.sync_params()
        runs.append((losses, tr.flat.data.clone(), tr.opt.exp_avg.clone()))
    assert runs[0][0] == runs[1][0], (runs[0][0], runs[1][0])
    assert torch.equal(runs[0][1], runs[1][1])
    assert torch.equal(runs[0][2], runs[1][2])


def test_moe_gpt_gpu_matches_cpu_and_captures():
    """MoE GPT (top-2, capacity routing, 4 experts) on the GPU vs the fp32 CPU path, then
    the same trainer captured in a hipGraph (static shapes end to end) and replayed."""
    from mxtrain.models.gpt import GPTConfig, GPTStage, gpt_param_specs
    from mxtrain.models.moe import moe_param_specs
    from mxtrain.parallel import state as pstate
    from mxtrain.parallel.buffers import FlatParams
    from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch
    cfg = GPTConfig(num_layers=2, hidden_size=256, num_attention_heads=4, seq_length=128,
                    max_position_embeddings=128, vocab_size=512, hidden_dropout=0.0, attention_dropout=0.0, num_experts=4,
                    expert_interval=1, moe_topk=2, moe_train_capacity_factor=2.0)
    B, S = 2, 128
    gen = torch.Generator().manual_seed(0)
    stages = []
    for dev, dt in (("cpu", torch.float32), (DEV, torch.bfloat16)):
        g2 = torch.Generator().manual_seed(0)
        d = FlatParams(gpt_param_specs(cfg), dev, dt)
        d.initialize(g2, cfg.num_layers)
        e = FlatParams(moe_param_specs(cfg, 0, 2, 1), dev, dt)
        e.initialize(g2, cfg.num_layers)
        if dev == "cpu":   # bf16-representable inputs for both
            d.data.copy_(d.data.to(torch.bfloat16).float())
            e.data.copy_(e.data.to(torch.bfloat16).float())
        st = GPTStage(cfg, d.params, d.grads, eparams=e.params, egrads=e.grads)
        st.rt.grad_scale = 1.0 / (B * S)
        st.rt.aux_scale = cfg.moe_loss_coeff
        stages.append((st, d, e))
    ids = torch.randint(0, cfg.vocab_size, (B * S,), generator=gen)
    labels = torch.randint(0, cfg.vocab_size, (B * S,), generator=gen)
    lc = stages[0][0].forward(ids=ids, labels=labels, B=B, S=S)
    lc.backward()
    lg = stages[1][0].forward(ids=ids.to(DEV), labels=labels.to(DEV), B=B, S=S)
    lg.backward()
    assert abs(float(lg.detach()) - float(lc.detach())) < 3e-2
    for (fc, fg) in ((stages[0][1], stages[1][1]), (stages[0][2], stages[1][2])):
        for n in fc.grads:
            a, b = fg.grads[n].float().cpu(), fc.grads[n]
            rel = (a - b).norm() / (b.norm() + 1e-6)
            assert rel < 6e-2, (n, float(rel))
    ps = pstate.initialize_model_parallel()
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=2), ps)
    tok, lab = synthetic_batch(cfg, 1, 2, ps.device, torch.Generator().manual_seed(1))
    l0 = float(tr.train_step(tok, lab))
    tr.capture(tok, lab, warmup=1)
    ls = [float(tr.train_step(tok, lab)) for _ in range(4)]
    torch.cuda.synchronize()
    assert all(x == x for x in ls) and ls[-1] < l0, (l0, ls)


@pytest.mark.parametrize("T,shapes,accumulate,strided,variant,splits", [
    (256, [(128, 128)], False, False, 0, 1),
    (1024, [(1024, 1024), (1024, 3072)], True, True, 6, 1),
    (512, [(1024, 1024), (3072, 1024)], False, True, -1, 0),
    (512, [(4096, 1024), (1024, 4096)], True, False, -1, 0),
    (4096, [(1024, 1024), (3072, 1024), (384, 256), (256, 640)], True, True, 0, 1),
    (4096, [(1024, 1024), (3072, 1024)], True, True, 2, 4),
    (2048, [(4096, 1024), (1024, 4096)], False, False, 2, 2),
    (1024, [(512, 256), (256, 512)], True, True, 1, 2),
])
def test_gemm_wgrad_group(T, shapes, accumulate, strided, variant, splits):
    """csrc/gemm.hip grouped dW = dY^T X against an fp32 reference (asymmetric data, strided
    dY/X rows, beta 0 and 1); an untileable problem in the group goes through torch."""
    from mxtrain.ops.gemm import wgrad_group
    g = torch.Generator(device="cuda").manual_seed(0)
    items, refs = [], []
    for (M, N) in shapes + [(200, 128)]:
        pad = 64 if strided else 0
        dy = torch.randn(T, M + pad, device="cuda", generator=g).to(torch.bfloat16)[:, :M]
        x = (torch.randn(T, N + pad, device="cuda", generator=g) + 0.25).to(torch.bfloat16)[:, pad:]
        gb = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
        ref = dy.float().t() @ x.float() + (gb.float() if accumulate else 0)
        items.append((gb, dy, x))
        refs.append(ref)
    if variant >= 0:   # forced tiles: the untileable extra problem goes through torch
        pass
    wgrad_group(items, accumulate=accumulate, variant=variant, splits=splits)
    wgrad_group(items[:-1], accumulate=True, variant=variant, splits=splits)   # second launch: tickets reset
    torch.cuda.synchronize()
    for (gb, dy, x), ref in zip(items[:-1], refs[:-1]):
        ref += dy.float().t() @ x.float()
    for (gb, _, _), ref in zip(items, refs):
        err = (gb.float() - ref).abs().max().item()
        assert err <= 0.01 * ref.abs().max().item() + 0.05, (gb.shape, err)


@pytest.mark.parametrize("graph,nm", [(False, 1), (True, 1), (False, 2)])
def test_deferred_colreduce_matches_immediate(graph, nm, monkeypatch):
    """LN / bias column reductions deferred to one batched launch at the end of backward
    (ops/norm.py ColReduceQueue) give the immediate path's trajectory: bit for bit with one
    micro-batch (same partials, same fixed-order sums), to bf16 rounding with two (one
    accumulate instead of one per micro-batch)."""
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.parallel import state as pstate
    from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch
    ps = pstate.initialize_model_parallel()
    cfg = GPTConfig(num_layers=3, hidden_size=256, num_attention_heads=4, seq_length=256,
                    max_position_embeddings=256, vocab_size=1024)
    runs = []
    for defer in ("0", "1"):
        monkeypatch.setenv("MXTRAIN_DEFER_COLREDUCE", defer)
        tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=2, global_batch_size=2 * nm), ps)
        assert (tr.stage.rt.colq is not None) == (defer == "1")
        tok, lab = synthetic_batch(cfg, nm, 2, ps.device, torch.Generator().manual_seed(3))
        losses = [float(tr.train_step(tok, lab)) for _ in range(2)]
        if graph:
            tr.capture(tok, lab, warmup=1)
        losses += [float(tr.train_step(tok, lab)) for _ in range(3)]
        torch.cuda.synchronize()
        tr.sync_params()
        if defer == "1":
            assert tr.stage.rt.colq.layout is not None and tr.stage.rt.colq.njobs > 0
        runs.append((losses, tr.flat.data.clone().float()))
    if nm == 1:
        assert runs[0][0] == runs[1][0], (runs[0][0], runs[1][0])
        assert torch.equal(runs[0][1], runs[1][1])
    else:
        for a, b in zip(runs[0][0], runs[1][0]):
            assert abs(a - b) < 2e-3 * max(1.0, abs(a)), (runs[0][0], runs[1][0])
        torch.testing.assert_close(runs[1][1], runs[0][1], rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("S,causal,L", [(1024, True, 3), (200, False, 2), (96, True, 1), (320, False, 1)])
def test_dropmask_wave_walk_matches_group_grid(S, causal, L):
    """The wave-walk dropout-mask kernel (default) writes exactly the words of the per-group
    grid kernel (variant 0) into both images of every layer, and nothing else."""
    from mxtrain.ops import _lib
    B, Hq, p, salt = 2, 3, 0.1, 9
    NB, NKT, NQT = (S + 31) // 32, (S + 127) // 128, (S + 63) // 64
    nf, nb = B * Hq * NB * NKT * 64, B * Hq * NB * NQT * 64
    seed = torch.tensor([13579], dtype=torch.int32, device=DEV)
    outs = []
    old = _lib._fn("mx_flash_dropmask_variant")(-1)
    try:
        for v in (0, 1):
            _lib._fn("mx_flash_dropmask_variant")(v)
            fb = torch.full((L, nf), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device=DEV)
            bb = torch.full((L, nb), 0x3C3C3C3C, dtype=torch.int32, device=DEV)
            _lib.call("mx_flash_dropmask_layers", _lib.ptr(seed), salt, float(p), B, S, Hq, 1, Hq + 2, int(causal),
                      L, _lib.ptr(fb[0]), _lib.ptr(bb[0]), 2 * nf, nb, _lib.stream())
            torch.cuda.synchronize()
            outs.append((fb.cpu(), bb.cpu()))
    finally:
        _lib._fn("mx_flash_dropmask_variant")(old)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert (outs[1][0] != 0x5A5A5A5A5A5A5A5A).any()


def test_dropmask_layers_match_per_layer_calls(monkeypatch):
    """All layers' attention-dropout images from one launch equal the per-layer ones (salt +
    layer), and a GPT training trajectory is unchanged bit for bit."""
    # (the images' dead causal blocks are never written, so the comparison is the training
    # trajectory, which reads every live word of every layer's images in fwd, dQ and dK/dV)
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.parallel import state as pstate
    from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch
    ps = pstate.initialize_model_parallel()
    cfg = GPTConfig(num_layers=3, hidden_size=256, num_attention_heads=4, seq_length=256,
                    max_position_embeddings=256, vocab_size=1024, attention_dropout=0.1)
    runs = []
    for on in ("0", "1"):
        monkeypatch.setenv("MXTRAIN_BATCH_DMASKS", on)
        tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=2), ps)
        tok, lab = synthetic_batch(cfg, 1, 2, ps.device, torch.Generator().manual_seed(5))
        losses = [float(tr.train_step(tok, lab)) for _ in range(3)]
        torch.cuda.synchronize()
        runs.append((losses, tr.flat.data.clone()))
    assert runs[0][0] == runs[1][0] and torch.equal(runs[0][1], runs[1][1])


# ------------------------------------------------------------------ forward / dgrad GEMMs
NT_VARIANTS = list(range(9))


@pytest.mark.parametrize("variant", NT_VARIANTS)
@pytest.mark.parametrize("epi", ["none", "bias", "gelu"])
def test_gemm_nt_forward_epilogues(variant, epi):
    """csrc/gemm_nt.hip forward (y = x w^T [+ b] [gelu]) against the fp32 reference, for
    every tile variant (one tile multiple in M, two in N, K = 3 K-steps ... )."""
    from mxtrain.ops import gemm as Gm
    bm, bn, _, _ = Gm._nt_tile(variant)
    M, N, K = 2 * bm, 3 * bn, 192
    x = _bf(torch.randn(M, K))
    w = _bf(torch.randn(N, K) * 0.1)
    b = _bf(torch.randn(N)) if epi != "none" else None
    out = Gm.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV) if b is not None else None, gelu=epi == "gelu",
                        variant=variant)
    ref = Gm.linear_fwd(x, w, b, gelu=epi == "gelu")
    if epi == "gelu":
        _close(out[1], ref[1], 2e-2, 1e-2, "pre-activation")
        _close(out[0], ref[0], 2e-2, 1e-2, "gelu")
    else:
        _close(out, ref, 2e-2, 1e-2, "y")


@pytest.mark.parametrize("variant", [0, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("gelu", [False, True])
def test_gemm_nt_dgrad_epilogues(variant, gelu):
    """dgrad dx = dy w (w K-major) and the fused GeLU' + bias-gradient epilogue."""
    from mxtrain.ops import gemm as Gm
    bm, bn, _, _ = Gm._nt_tile(variant)
    M, N, K = 2 * bm, 2 * bn, 320
    dy = _bf(torch.randn(M, K))
    w = _bf(torch.randn(K, N) * 0.1)
    h = _bf(torch.randn(M, N) * 2) if gelu else None
    db = _bf(torch.randn(N)) if gelu else None
    dbg = db.to(DEV) if gelu else None
    out = Gm.linear_dgrad(dy.to(DEV), w.to(DEV), gelu_aux=h.to(DEV) if gelu else None, dbias=dbg,
                          accumulate=True, variant=variant)
    ref = Gm.linear_dgrad(dy, w, gelu_aux=h, dbias=db, accumulate=True)
    _close(out, ref, 2e-2, 1e-2, "dx")
    if gelu:
        _close(dbg, db, 0.25, 2e-2, "dbias")


def test_gemm_nt_strided_inputs_and_plan():
    """Row-strided operands (views into a packed buffer, as the QKV / attention code passes
    them) and the automatic variant plan at the GPT-2 345M shapes."""
    from mxtrain.ops import gemm as Gm
    big = _bf(torch.randn(512, 3 * 1024)).to(DEV)
    x = big[:, 1024:2048]
    w = _bf(torch.randn(1024, 1024) * 0.05).to(DEV)
    y = Gm.linear_fwd(x, w)
    ref = (x.float() @ w.float().t())
    _close(y, ref, 3e-2, 1e-2, "strided")
    for (M, N, K, km) in [(4096, 3072, 1024, False), (4096, 4096, 1024, False), (4096, 1024, 4096, False),
                          (4096, 1024, 1024, False), (4096, 1024, 3072, True), (4096, 4096, 1024, True)]:
        assert Gm.nt_plan(M, N, K, km) >= 0, (M, N, K, km)


@pytest.mark.parametrize("S,causal,hoff", [(1024, True, 0), (200, False, 3), (384, True, 2)])
def test_flash_fwd_inkernel_dropout_bits_identical(S, causal, hoff):
    """The A/B variant of the attention forward that hashes its keep bits in-kernel
    (mx_flash_fwd_dgen) gives exactly the output and lse of the shipping forward fed the
    pre-pass image (mx_flash_dropmask) for the same (seed, salt, p, head offset)."""
    from mxtrain.ops import _lib
    from mxtrain.ops import attention as A
    B, H, D, p, salt, Hg = 2, 4, 64, 0.1, 77, 9
    g = torch.Generator(device=DEV).manual_seed(S)
    qkv = torch.randn(B * S, 3 * H * D, device=DEV, generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    seed = torch.tensor([4242], dtype=torch.int32, device=DEV)
    dm = A.dropmask(B, S, H, p, seed, salt, hoff, Hg, causal)
    o1, lse1, _ = A.attn_fwd(q, k, v, B, S, H, H, D, causal, dmask=dm)
    o2 = torch.empty_like(o1)
    lse2 = torch.empty_like(lse1)
    _lib.call("mx_flash_fwd_dgen", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), q.stride(0), k.stride(0), v.stride(0),
              _lib.ptr(o2), o2.stride(0), _lib.ptr(lse2), B, S, H, H, D, int(causal), None, 1.0 / D ** 0.5,
              _lib.ptr(seed), salt, p, hoff, Hg, _lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(o1, o2) and torch.equal(lse1, lse2)
