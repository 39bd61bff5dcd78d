"""csrc/batchnorm.hip: training-mode BatchNorm fused with the residual add and ReLU
(NHWC bf16, the ResNet-50 bottleneck tail of BASELINE config 5) against a plain PyTorch
fp32 reference of the same op: output, running statistics, dx / dgamma / dbeta / dres;
and run-to-run determinism (two-stage reductions, no atomics)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol, name):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    bad = (err > atol + rtol * b.abs()).sum().item()
    assert bad == 0, f"{name}: {bad} elements off, max err {err.max().item():.3e}"


@pytest.mark.parametrize("N,C,H,W,res,relu", [(8, 64, 28, 28, True, True), (4, 256, 14, 14, False, True),
                                              (16, 2048, 7, 7, True, True), (2, 128, 9, 11, False, False),
                                              (256, 64, 4, 4, True, False)])
def test_bn_act_matches_fp32(N, C, H, W, res, relu):
    from mxtrain.ops.batchnorm import bn_act
    g = torch.Generator(device=DEV).manual_seed(C + H)
    x32 = (torch.randn(N, C, H, W, device=DEV, generator=g) * 3 + 1.5)
    x = x32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r = (torch.randn(N, C, H, W, device=DEV, generator=g).to(torch.bfloat16)
         .contiguous(memory_format=torch.channels_last)) if res else None
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    ref_bn = torch.nn.BatchNorm2d(C).to(DEV)
    ref_bn.load_state_dict(bn.state_dict())
    xa = x.clone().requires_grad_(True)
    ra = r.clone().requires_grad_(True) if res else None
    y = bn_act(xa, bn, ra, relu)
    assert y.is_contiguous(memory_format=torch.channels_last)
    xr = x.float().clone().requires_grad_(True)
    rr = r.float().clone().requires_grad_(True) if res else None
    yr_pre = ref_bn(xr)
    if res:
        yr_pre = yr_pre + rr
    yr = F.relu(yr_pre) if relu else yr_pre
    _close(y, yr, 3e-2, 1e-2, "y")
    _close(bn.running_mean, ref_bn.running_mean, 1e-4, 1e-4, "running_mean")
    _close(bn.running_var, ref_bn.running_var, 1e-3, 1e-3, "running_var")
    dy = torch.randn(N, C, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    # the reference takes the ReLU mask from the kernel's output, so elements within rounding
    # of zero (batch statistics summed in another order) agree
    yr_pre.backward(torch.where(y.float() > 0, dy.float(), 0.0) if relu else dy.float())
    _close(xa.grad, xr.grad, 3e-2, 3e-2, "dx")
    # BN + ReLU without a residual recovers xhat from the bf16 output (ops/batchnorm.py RECON):
    # dgamma = sum dz xhat then carries the output's rounding, std ~ 2^-9 sqrt(sum (dz y)^2) / gamma
    # ~ 0.04 at these sizes, where the reference reads the same bf16 x exactly
    k = 5e-3 if (relu and not res) else 1e-3
    _close(bn.weight.grad, ref_bn.weight.grad, 0.05 + k * (N * H * W) ** 0.5, 1e-2, "dgamma")
    _close(bn.bias.grad, ref_bn.bias.grad, 0.05 + 1e-3 * (N * H * W) ** 0.5, 1e-2, "dbeta")
    if res:
        _close(ra.grad, rr.grad, 1e-2, 1e-2, "dres")


def test_bn_act_deterministic_and_eval():
    from mxtrain.ops.batchnorm import bn_act
    C = 256
    x = torch.randn(32, C, 14, 14, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for _ in range(2):
        bn = torch.nn.BatchNorm2d(C).to(DEV)
        xa = x.clone().requires_grad_(True)
        y = bn_act(xa, bn, None, True)
        y.backward(torch.ones_like(y))
        outs.append((y, xa.grad, bn.weight.grad, bn.running_var.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    bn.eval()
    ye = bn_act(x, bn, None, True)
    ref = F.relu(F.batch_norm(x.float(), bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.1, bn.eps))
    _close(ye, ref, 3e-2, 1e-2, "eval")


def test_resnet50_bn_step_uses_fused_paths():
    """One training step of the BN ResNet-50 (small batch) with bf16 autocast: finite loss,
    every BatchNorm a fused node, and the res3+ convolutions on the implicit-GEMM kernels."""
    from mxtrain.models.resnet import resnet50
    torch.manual_seed(0)
    net = resnet50(norm="bn", num_classes=1000).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 224, 224, device=DEV).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (8,), device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        logits = net(x)
        loss = F.cross_entropy(logits.float(), y)
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss)
    gn = sum(float(p.grad.float().norm() ** 2) for p in net.parameters() if p.grad is not None) ** 0.5
    assert gn > 0 and gn == gn
    assert all(p.grad is not None for p in net.parameters() if p.requires_grad)


@pytest.mark.parametrize("N,Cin,Cout,H,W,k,stride,split", [(2, 64, 64, 7, 7, 3, 1, True),
                                                          (32, 64, 256, 56, 56, 1, 1, False),
                                                          (64, 256, 128, 28, 28, 3, 2, False),
                                                          (16, 1024, 2048, 14, 14, 1, 2, False),
                                                          (3, 128, 192, 10, 13, 1, 1, False)])
def test_conv_epilogue_bn_statistics(N, Cin, Cout, H, W, k, stride, split):
    """The implicit-GEMM forward's epilogue writes per-64-row BatchNorm statistics of its
    (rounded) output: they match the block statistics of y in fp32, the stored y is the same
    bits as without them, and bn_act fed with them (merged to <= 512 blocks when there are
    more) matches bn_act's own statistics pass -- output, running statistics, batch count."""
    from mxtrain.ops import convwg
    from mxtrain.ops.batchnorm import bn_act
    g = torch.Generator(device=DEV).manual_seed(Cin + Cout + H)
    x = torch.randn(N, Cin, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=DEV, generator=g) / (Cin * k * k) ** 0.5 + 0.02).to(
        torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert convwg.fwd_supported(x, w, None, None, stride, k // 2, 1)
    y0 = convwg.conv_fwd(x, w, None, None, False, stride, k // 2, 1)
    y, pre = convwg.conv_fwd(x, w, None, None, False, stride, k // 2, 1, bn_stats=True)
    assert torch.equal(y0, y)
    if split:   # split-K launch: no epilogue statistics, bn_act runs its own pass
        assert pre is None
        return
    T = y.shape[0] * y.shape[2] * y.shape[3]
    nb = (T + 63) // 64
    assert pre.numel() == nb * 2 * Cout
    rows = y.permute(0, 2, 3, 1).reshape(T, Cout).float()
    pad = torch.full((nb * 64 - T, Cout), float("nan"), device=DEV)
    blk = torch.cat([rows, pad]).view(nb, 64, Cout)
    cnt = (~blk.isnan()).sum(1).float()
    mean = torch.nansum(blk, 1) / cnt
    m2 = torch.nansum((blk - mean[:, None]) ** 2, 1)
    pm, pq = pre.view(2, Cout, nb)   # channel-major [C][blocks]
    _close(pm.t(), mean, 1e-4, 1e-4, "block means")
    _close(pq.t(), m2, 1e-3 * 64, 2e-3, "block M2")
    gamma = torch.empty(Cout, device=DEV).uniform_(0.5, 1.5, generator=g)
    beta = torch.empty(Cout, device=DEV).uniform_(-0.5, 0.5, generator=g)
    outs = []
    for p in (None, pre):
        bn = torch.nn.BatchNorm2d(Cout).to(DEV)
        with torch.no_grad():
            bn.weight.copy_(gamma)
            bn.bias.copy_(beta)
        outs.append((bn_act(y, bn, None, True, pre=p), bn))
    (ya, bna), (yb, bnb) = outs
    _close(yb, ya, 2e-2, 1e-2, "bn_act with epilogue statistics")
    _close(bnb.running_mean, bna.running_mean, 1e-5, 1e-4, "running_mean")
    _close(bnb.running_var, bna.running_var, 1e-5, 1e-4, "running_var")
    assert int(bna.num_batches_tracked) == 1 and int(bnb.num_batches_tracked) == 1


@pytest.mark.parametrize("proj", [False, True])
def test_bn_bottleneck_residual_gradient_fused_into_conv1_dgrad(monkeypatch, proj):
    """Trainable-BN identity blocks: conv3's BN backward stashes the residual gradient and
    conv1's implicit-GEMM dgrad adds it in its store (one rounding) instead of autograd's
    separate add; projection blocks (``proj``): the shortcut conv's input gradient is parked
    and added the same way.  Against the unfused blocks and an fp32 run: same forward,
    gradients as close to fp32 as the unfused ones; the fused dgrad received the addend."""
    import copy
    from mxtrain.models.resnet import Bottleneck
    from mxtrain.ops import convwg
    seen = {"add": 0, "cls": 0}
    real = convwg.conv_dgrad

    def spy(*a, add=None, **k):
        seen["add"] += add is not None
        seen["cls"] += bool(k.get("class_out")) + bool(k.get("add_class"))
        return real(*a, add=add, **k)

    monkeypatch.setattr(convwg, "conv_dgrad", spy)
    torch.manual_seed(5)
    first = Bottleneck(256, 128, stride=2, norm="bn") if proj else Bottleneck(512, 128, norm="bn")
    blocks = torch.nn.Sequential(first, Bottleneck(512, 128, norm="bn")).to(DEV)
    blocks = blocks.to(memory_format=torch.channels_last)
    for m in blocks.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    cin = 256 if proj else 512
    x0 = torch.randn(4, cin, 48, 64, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = {}
    gy = None
    for fuse in (False, True):
        b2 = copy.deepcopy(blocks)
        for b in b2:
            b.fuse_backward = fuse
        seen["add"] = seen["cls"] = 0
        x = x0.clone().requires_grad_()
        y = b2(x)
        if gy is None:
            gy = torch.randn_like(y)
        y.backward(gy)
        torch.cuda.synchronize()
        out[fuse] = (y.detach().float(), x.grad.float(), [p.grad.float() for p in b2.parameters()], seen["add"],
                     seen["cls"])
    assert out[True][3] == 2 and out[False][3] == 0, (out[True][3], out[False][3])
    # 1 x 1 stride-2 conv1 and shortcut (stride_in_1x1): the parked dX is the compact parity class
    ws = first.shortcut.conv.weight.to(torch.bfloat16) if proj else None
    if proj and convwg.class_ok(ws, tuple(x0.shape), 2, 0, 1) and convwg.class_ok(
            first.conv1.conv.weight.to(torch.bfloat16), tuple(x0.shape), 2, 0, 1):
        assert out[True][4] == 2, out[True][4]
    if not proj:   # (fused BN pair: the shortcut BN's output is not rounded to bf16 before the add)
        assert torch.equal(out[False][0], out[True][0])
    b32 = copy.deepcopy(blocks).float()
    for b in b32:
        b.fuse_backward = False
    x32 = x0.float().requires_grad_()
    y32 = b32(x32)
    y32.backward(gy.float())
    ey_f = (out[True][0] - y32.detach()).abs().max().item()
    ey_u = (out[False][0] - y32.detach()).abs().max().item()
    assert ey_f <= 1.25 * ey_u + 1e-2, (ey_f, ey_u)
    e_f = (out[True][1] - x32.grad).abs().max().item()
    e_u = (out[False][1] - x32.grad).abs().max().item()
    assert e_f <= 1.25 * e_u + 1e-3 * x32.grad.abs().max().item(), (e_f, e_u)
    # weight gradients: as close to the fp32 run as the unfused ones (relative norm error)
    for a, c, r in zip(out[True][2], out[False][2], [p.grad.float() for p in b32.parameters()]):
        rn = float(r.norm()) + 1e-12
        ef, eu = float((a - r).norm()) / rn, float((c - r).norm()) / rn
        assert ef <= 1.25 * eu + 1e-3, (ef, eu)


@pytest.mark.parametrize("N,C,H,W,relu", [(4, 64, 112, 112, True), (2, 8, 7, 9, False), (3, 24, 10, 13, True),
                                          (1, 16, 1, 1, False)])
def test_maxpool3s2_matches_torch(N, C, H, W, relu):
    """The stem's 3x3 / 2 / pad-1 max-pool (csrc/pool.hip: one-byte window argmax, gathering
    backward) against F.max_pool2d: the same output bits and, with ReLU ties (many zeros per
    window: the first maximum in window order wins in both), the same input gradient."""
    from mxtrain.ops.epilogue import maxpool3s2
    g = torch.Generator(device=DEV).manual_seed(C + H)
    x = torch.randn(N, C, H, W, device=DEV, generator=g)
    if relu:
        x = torch.relu(x)
    x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xa = x.clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    y = maxpool3s2(xa)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert y.shape == yr.shape and torch.equal(y, yr)
    dy = torch.randn(y.shape, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    yr.backward(dy)
    _close(xa.grad, xr.grad, 1e-2, 1e-2, "dx")


@pytest.mark.parametrize("N,C,H,W", [(256, 2048, 7, 7), (3, 24, 5, 3), (2, 8, 1, 1)])
def test_global_avg_pool_matches_fp32(N, C, H, W):
    """The classifier head's pool (csrc/pool.hip mx_gap_fwd / mx_gap_bwd, fp32 accumulation)
    against x.float().mean((2, 3)) and its gradient; the HIP path must be the one taken."""
    from mxtrain.ops.epilogue import GlobalAvgPoolFn, global_avg_pool
    g = torch.Generator(device=DEV).manual_seed(C + H)
    x = torch.randn(N, C, H, W, device=DEV, generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    xa = x.clone().requires_grad_(True)
    xr = x.float().requires_grad_(True)
    y = global_avg_pool(xa)
    assert y.grad_fn is not None and type(y.grad_fn).__name__.startswith(GlobalAvgPoolFn.__name__)
    yr = xr.mean(dim=(2, 3))
    assert y.dtype == torch.float32 and y.shape == (N, C)
    _close(y, yr, 1e-5, 1e-5, "y")
    dy = torch.randn(N, C, device=DEV, generator=g)
    y.backward(dy)
    yr.backward(dy)
    assert xa.grad.dtype == torch.bfloat16 and xa.grad.is_contiguous(memory_format=torch.channels_last)
    _close(xa.grad.float(), xr.grad, 1e-5, 1e-2, "dx")


def test_cast_group_one_launch_copies_and_grads():
    """models/compute_weights.py CastGroup: bf16 compute copies of fp32 weights (channels_last
    and contiguous) from one csrc/cast.hip launch equal w.to(bf16) bit for bit, keep each
    weight's strides, and their fp32 gradients (one launch back) equal g.float()."""
    from mxtrain.models import compute_weights as cw
    ws = [torch.randn(64, 32, 3, 3, device=DEV).contiguous(memory_format=torch.channels_last),
          torch.randn(128, 64, 1, 1, device=DEV).contiguous(memory_format=torch.channels_last),
          torch.randn(24, 16, device=DEV), torch.randn(64, 3, 7, 7, device=DEV).contiguous(memory_format=torch.channels_last)]
    ws = [w.requires_grad_(True) for w in ws]
    gs = []
    with cw.CastGroup(ws):
        for w in ws:
            c = cw.cw(w, torch.bfloat16)
            assert c.dtype == torch.bfloat16 and c.stride() == w.stride()
            assert torch.equal(c, w.detach().to(torch.bfloat16))
            g = torch.randn(w.shape, device=DEV).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last if w.dim() == 4 else torch.contiguous_format)
            gs.append(g)
        loss = sum((cw.cw(w, torch.bfloat16).float() * g.float()).sum() for w, g in zip(ws, gs))
    loss.backward()
    for w, g in zip(ws, gs):
        assert w.grad.dtype == torch.float32 and w.grad.stride() == w.stride()
        torch.testing.assert_close(w.grad, g.float(), rtol=0, atol=0)


def test_normalize_u8_nhwc_helper_matches_torch():
    """ops/vision.py normalize_u8_nhwc (the ResNet-50 workload's input pass): uint8 NCHW ->
    normalised bf16 channels_last in one kernel, against the fp32 torch expression."""
    from mxtrain.ops.vision import normalize_u8_nhwc
    img = torch.randint(0, 256, (4, 3, 32, 48), dtype=torch.uint8, device=DEV)
    mean, std = (123.7, 116.3, 103.5), (58.4, 57.1, 57.4)
    x = normalize_u8_nhwc(img, mean, std)
    assert x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)
    ref = (img.float() - torch.tensor(mean, device=DEV).view(1, 3, 1, 1)) / torch.tensor(std, device=DEV).view(1, 3, 1, 1)
    _close(x, ref, 1e-2, 1e-2, "normalised")


def test_bn_relu_backward_stats_from_output_match_reading_x(monkeypatch):
    """BN + ReLU without a residual takes its backward statistics from the output
    (xhat = (y - beta) / gamma where the ReLU passed; x not re-read): the same dx / dgamma /
    dbeta as the pass that reads x, including channels whose gamma is zero (those threads
    read x)."""
    from mxtrain.ops import batchnorm as BN
    g = torch.Generator(device=DEV).manual_seed(7)
    x = (torch.randn(16, 64, 20, 20, device=DEV, generator=g) * 2 + 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(x.shape, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for recon in (False, True):
        monkeypatch.setattr(BN, "RECON", recon)
        bn = torch.nn.BatchNorm2d(64).to(DEV)
        with torch.no_grad():
            bn.weight.copy_(torch.linspace(0.3, 1.7, 64))
            bn.weight[:8] = 0.0
            bn.bias.copy_(torch.linspace(-0.4, 0.4, 64))
        xa = x.clone().requires_grad_(True)
        y = BN.bn_act(xa, bn, None, True)
        y.backward(dy)
        outs.append((y, xa.grad.float(), bn.weight.grad.clone(), bn.bias.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    _close(outs[1][1], outs[0][1], 2e-2, 2e-2, "dx")
    _close(outs[1][2], outs[0][2], 0.5, 1e-2, "dgamma")
    assert torch.equal(outs[1][3], outs[0][3])   # dbeta does not use xhat



def test_cast_group_deferred_wgrad_reductions_bit_identical(monkeypatch):
    """Under CastGroup the implicit-GEMM weight gradients' split-K reductions are deferred and
    run as one batched launch before the group's fp32 cast (ops/convwg.py defer_*): the same
    gradient bits as reducing each at once, and the batched launch actually ran."""
    import copy
    from mxtrain.models import compute_weights as cw
    from mxtrain.models.resnet import Bottleneck
    from mxtrain.ops import convwg
    torch.manual_seed(7)
    blocks = torch.nn.Sequential(Bottleneck(256, 128, stride=2, norm="bn"), Bottleneck(512, 128, norm="bn"))
    blocks = blocks.to(DEV).to(memory_format=torch.channels_last)
    x0 = torch.randn(8, 256, 32, 32, device=DEV).contiguous(memory_format=torch.channels_last)
    flushed = {"n": 0}
    real = convwg.defer_flush

    def spy(*a, **k):
        flushed["n"] += len(convwg._DEF["jobs"])
        return real(*a, **k)

    monkeypatch.setattr(convwg, "defer_flush", spy)
    grads = {}
    for defer in (False, True):
        monkeypatch.setattr(cw.CastGroup, "DEFER", defer)
        b = copy.deepcopy(blocks)
        flushed["n"] = 0
        with torch.autocast("cuda", dtype=torch.bfloat16):
            with cw.CastGroup([m.weight for m in b.modules() if isinstance(m, torch.nn.Conv2d)]):
                y = b(x0.to(torch.bfloat16))
        y.float().square().mean().backward()
        torch.cuda.synchronize()
        assert not convwg._DEF["on"], "deferral must be off after the last group's backward"
        grads[defer] = ([p.grad.clone() for p in b.parameters()], flushed["n"])
    assert grads[True][1] > 0 and grads[False][1] == 0, (grads[True][1], grads[False][1])
    for a, c in zip(grads[True][0], grads[False][0]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("N,C,H,W", [(16, 256, 14, 14), (4, 2048, 7, 7), (3, 64, 9, 11)])
def test_bn2_add_relu_matches_fp32(N, C, H, W):
    """ops/batchnorm.py bn2_add_relu (csrc/batchnorm.hip mx_bn2_*): relu(BN_a(xa) + BN_b(xb))
    as one node against fp32 torch -- output, both BNs' running statistics and batch counts,
    both input gradients and both BNs' dgamma / dbeta."""
    from mxtrain.ops.batchnorm import BN2AddReluFn, bn2_add_relu
    g = torch.Generator(device=DEV).manual_seed(C + H)
    cl = torch.channels_last
    xa = (torch.randn(N, C, H, W, device=DEV, generator=g) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    xb = (torch.randn(N, C, H, W, device=DEV, generator=g) - 0.3).to(torch.bfloat16).contiguous(memory_format=cl)
    bns = [torch.nn.BatchNorm2d(C).to(DEV) for _ in range(2)]
    for bn in bns:
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5, generator=g)
            bn.bias.uniform_(-0.5, 0.5, generator=g)
    refs = [torch.nn.BatchNorm2d(C).to(DEV) for _ in range(2)]
    for r, bn in zip(refs, bns):
        r.load_state_dict(bn.state_dict())
    a, b = xa.clone().requires_grad_(True), xb.clone().requires_grad_(True)
    y = bn2_add_relu(a, bns[0], b, bns[1])
    assert type(y.grad_fn).__name__.startswith(BN2AddReluFn.__name__)
    ar, br = xa.float().requires_grad_(True), xb.float().requires_grad_(True)
    pre = refs[0](ar) + refs[1](br)
    yr = torch.relu(pre)
    _close(y, yr, 3e-2, 1e-2, "y")
    for bn, r in zip(bns, refs):
        _close(bn.running_mean, r.running_mean, 1e-4, 1e-4, "running_mean")
        _close(bn.running_var, r.running_var, 1e-3, 1e-3, "running_var")
        assert int(bn.num_batches_tracked) == 1
    dy = torch.randn(y.shape, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    y.backward(dy)
    pre.backward(torch.where(y.float() > 0, dy.float(), 0.0))
    _close(a.grad, ar.grad, 3e-2, 3e-2, "dxa")
    _close(b.grad, br.grad, 3e-2, 3e-2, "dxb")
    M = N * H * W
    for bn, r in zip(bns, refs):
        _close(bn.weight.grad, r.weight.grad, 0.05 + 1e-3 * M ** 0.5, 1e-2, "dgamma")
        _close(bn.bias.grad, r.bias.grad, 0.05 + 1e-3 * M ** 0.5, 1e-2, "dbeta")


@pytest.mark.parametrize("N,C,H,W", [(8, 64, 56, 56), (3, 16, 13, 11)])
def test_bn_relu_maxpool_fold_matches_separate(N, C, H, W):
    """ops/batchnorm.py bn_relu_maxpool (the stem's BN + ReLU folded into pool0, csrc/pool.hip
    mx_maxpool3s2_fwd_bn / _bwd_relu): the same output bits and running statistics as
    bn_act + maxpool3s2, input / gamma / beta gradients as close to fp32 as theirs."""
    from mxtrain.ops.batchnorm import BNReluMaxPoolFn, bn_act, bn_relu_maxpool
    from mxtrain.ops.epilogue import maxpool3s2
    g = torch.Generator(device=DEV).manual_seed(C + H)
    x = (torch.randn(N, C, H, W, device=DEV, generator=g) * 2 - 0.3).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.5, 0.5, generator=g)
    bns = [copy_bn for copy_bn in (torch.nn.BatchNorm2d(C).to(DEV) for _ in range(3))]
    for b in bns:
        b.load_state_dict(bn.state_dict())
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya = bn_relu_maxpool(xa, bns[0])
    assert type(ya.grad_fn).__name__.startswith(BNReluMaxPoolFn.__name__)
    yb = maxpool3s2(bn_act(xb, bns[1], None, True))
    assert torch.equal(ya, yb)
    assert torch.equal(bns[0].running_mean, bns[1].running_mean) and torch.equal(bns[0].running_var, bns[1].running_var)
    assert int(bns[0].num_batches_tracked) == 1
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(torch.relu(bns[2](xr)), 3, 2, 1)
    dy = torch.randn(ya.shape, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ya.backward(dy)
    yb.backward(dy)
    yr.backward(dy.float())
    for name, a, b, r in (("dx", xa.grad, xb.grad, xr.grad), ("dgamma", bns[0].weight.grad, bns[1].weight.grad,
                                                                bns[2].weight.grad),
                          ("dbeta", bns[0].bias.grad, bns[1].bias.grad, bns[2].bias.grad)):
        ea = (a.float() - r).abs().max().item()
        eb = (b.float() - r).abs().max().item()
        assert ea <= 1.25 * eb + 1e-3 * r.abs().max().item(), (name, ea, eb)
