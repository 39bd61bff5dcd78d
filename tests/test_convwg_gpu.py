"""Implicit-GEMM convolution weight gradients (csrc/convwg.hip, ops/convwg.py) against the
plain PyTorch fp32 weight gradient of the same convolution (CPU), for 1x1 / strided 1x1 /
3x3 / dilated 3x3 filters, pixel counts that are not multiples of 64, several images,
fixed and planned split counts and accumulation into an existing gradient."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [
    # N, Cin, Cout, H, W, k, stride, pad, dil
    (1, 128, 256, 17, 23, 1, 1, 0, 1),
    (2, 256, 128, 16, 17, 1, 2, 0, 1),
    (1, 128, 128, 25, 42, 3, 1, 1, 1),
    (3, 256, 256, 14, 14, 3, 1, 1, 1),
    (1, 128, 128, 19, 21, 3, 1, 2, 2),
    (2, 128, 256, 9, 11, 3, 2, 1, 1),
    # Cin an odd multiple of 64 (ResNet res2 inputs: the last 128-column tile half padded)
    (2, 64, 64, 28, 30, 3, 1, 1, 1),
    (1, 64, 256, 20, 22, 1, 1, 0, 1),
    (2, 64, 128, 17, 19, 1, 2, 0, 1),
    (1, 192, 128, 15, 16, 3, 1, 1, 1),
]


def _ref(dy, x, w_shape, stride, pad, dil):
    return torch.ops.aten.convolution_backward(dy.float().cpu(), x.float().cpu(), torch.zeros(w_shape), None,
                                               [stride] * 2, [pad] * 2, [dil] * 2, False, [0, 0], 1,
                                               [False, True, False])[1]


def _inputs(N, Cin, Cout, H, W, k, stride, pad, dil, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, Cin, H, W, generator=g).to(torch.bfloat16)
    OH = (H + 2 * pad - dil * (k - 1) - 1) // stride + 1
    OW = (W + 2 * pad - dil * (k - 1) - 1) // stride + 1
    dy = torch.randn(N, Cout, OH, OW, generator=g).to(torch.bfloat16)
    cl = torch.channels_last
    return x.cuda().contiguous(memory_format=cl), dy.cuda().contiguous(memory_format=cl)


def _close(out, ref):
    err = (out.float().cpu() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-2 * scale + 1e-3, (err, scale)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("splits", [1, 3, 0])
def test_conv_wgrad_matches_fp32(case, splits):
    from mxtrain.ops import convwg
    N, Cin, Cout, H, W, k, stride, pad, dil = case
    x, dy = _inputs(*case)
    out = convwg.conv_wgrad(dy, x, (Cout, Cin, k, k), stride, pad, dil, splits=splits)
    torch.cuda.synchronize()
    assert out.is_contiguous(memory_format=torch.channels_last)
    _close(out, _ref(dy, x, (Cout, Cin, k, k), stride, pad, dil))


def test_conv_wgrad_accumulates_and_is_deterministic():
    from mxtrain.ops import convwg
    case = (2, 128, 128, 30, 31, 3, 1, 1, 1)
    N, Cin, Cout, H, W, k, stride, pad, dil = case
    x, dy = _inputs(*case, seed=3)
    a = convwg.conv_wgrad(dy, x, (Cout, Cin, k, k), stride, pad, dil, splits=5)
    b = convwg.conv_wgrad(dy, x, (Cout, Cin, k, k), stride, pad, dil, splits=5)
    assert torch.equal(a, b)
    base = torch.randn(Cout, k, k, Cin, device="cuda").to(torch.bfloat16).permute(0, 3, 1, 2)
    acc = base.clone(memory_format=torch.channels_last)
    convwg.conv_wgrad(dy, x, (Cout, Cin, k, k), stride, pad, dil, out=acc, beta=1.0, splits=5)
    torch.cuda.synchronize()
    _close(acc.float() - base.float(), _ref(dy, x, (Cout, Cin, k, k), stride, pad, dil))


@pytest.mark.parametrize("hw", [(20, 24), (64, 64)])   # input gradient: split-K / plain implicit GEMM
def test_conv_wg_autograd_matches_conv2d(hw):
    """The autograd Function: output as F.conv2d's (MIOpen), the input gradient as MIOpen's
    to bf16 rounding, the weight gradient matches the fp32 reference."""
    from mxtrain.ops import convwg
    torch.manual_seed(0)
    cl = torch.channels_last
    x = torch.randn(2, 128, *hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(256, 3, 3, 128, device="cuda") * 0.05).to(torch.bfloat16).permute(0, 3, 1, 2)
    x1, w1 = x.clone().requires_grad_(), w.detach().clone(memory_format=cl).requires_grad_()
    x2, w2 = x.clone().requires_grad_(), w.detach().clone(memory_format=cl).requires_grad_()
    assert convwg.supported(x1, w1, 1, 1, 1)
    assert convwg.dgrad_supported(w1, tuple(x.shape), 1)
    y1 = convwg.conv2d_wg(x1, w1, 1, 1, 1)
    y2 = torch.nn.functional.conv2d(x2, w2, None, 1, 1, 1)
    _close(y1.detach(), y2.detach().float().cpu())
    g = torch.randn_like(y1)
    y1.backward(g)
    y2.backward(g)
    _close(x1.grad, x2.grad.float().cpu())
    ref = _ref(g, x, tuple(w.shape), 1, 1, 1)
    _close(w1.grad, ref)


def _ref_dx(dy, w, x_shape, stride, pad, dil):
    return torch.ops.aten.convolution_backward(dy.float().cpu(), torch.zeros(x_shape), w.float().cpu(), None,
                                               [stride] * 2, [pad] * 2, [dil] * 2, False, [0, 0], 1,
                                               [True, False, False])[0]


@pytest.mark.parametrize("case", CASES + [(1, 128, 64, 13, 9, 3, 1, 1, 1),
                                  # split-K (few tiles: res5 at one image) and a plain one
                                  (1, 512, 512, 25, 42, 3, 1, 1, 1), (1, 512, 2048, 25, 42, 1, 1, 0, 1),
                                  (2, 256, 256, 40, 52, 3, 1, 1, 1)])
def test_conv_dgrad_matches_fp32(case):
    """K-step depth by shape (32 for the narrow reductions, else 64): the cases cover both."""
    _dgrad_case(case)


def _dgrad_case(case):
    from mxtrain.ops import convwg
    N, Cin, Cout, H, W, k, stride, pad, dil = case
    x, dy = _inputs(*case, seed=7)
    g = torch.Generator().manual_seed(11)
    w = (torch.randn(Cout, k, k, Cin, generator=g) * 0.1).to(torch.bfloat16).cuda().permute(0, 3, 1, 2)
    dx = convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil)
    torch.cuda.synchronize()
    assert dx.is_contiguous(memory_format=torch.channels_last)
    _close(dx, _ref_dx(dy, w, tuple(x.shape), stride, pad, dil))


@pytest.mark.parametrize("case", [(1, 64, 256, 40, 48, 1, 1, 0, 1), (2, 128, 128, 25, 42, 3, 1, 1, 1),
                                  (1, 256, 128, 50, 60, 1, 2, 0, 1), (1, 128, 256, 30, 33, 3, 1, 2, 2),
                                  # 128 x 64 tiles (Cout an odd multiple of 64: res2)
                                  (2, 64, 64, 50, 62, 3, 1, 1, 1), (1, 256, 64, 41, 37, 1, 1, 0, 1),
                                  (1, 128, 192, 30, 33, 1, 1, 0, 1),
                                  # split-K (few tiles: res5 / P5 at one image)
                                  (1, 512, 512, 25, 42, 3, 1, 1, 1), (1, 1024, 512, 50, 84, 1, 2, 0, 1),
                                  (1, 256, 256, 25, 42, 3, 1, 1, 1)])
@pytest.mark.parametrize("res", [False, True])
def test_conv_fwd_fused_epilogue_matches_fp32(case, res):
    """K-step depth by shape (32 for 1x1 / Cin <= 128, else 64): the cases cover both."""
    _fwd_case(case, res)


def _fwd_case(case, res):
    from mxtrain.ops import convwg
    N, Cin, Cout, H, W, k, stride, pad, dil = case
    x, dy = _inputs(*case, seed=5)
    g = torch.Generator().manual_seed(13)
    w = (torch.randn(Cout, k, k, Cin, generator=g) * 0.1).to(torch.bfloat16).cuda().permute(0, 3, 1, 2)
    b = torch.randn(Cout, generator=g).to(torch.bfloat16).cuda()
    r = torch.randn(dy.shape, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=torch.channels_last) \
        if res else None
    y = convwg.conv_fwd(x, w, b, r, True, stride, pad, dil)
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv2d(x.float().cpu(), w.float().cpu(), b.float().cpu(), stride, pad, dil)
    if res:
        ref = ref + r.float().cpu()
    ref = ref.relu()
    assert y.is_contiguous(memory_format=torch.channels_last) and y.shape == ref.shape
    _close(y, ref)


def test_conv_bias_act_all_implicit_gemm_matches_fp32():
    """ops.epilogue.conv_bias_act on the fully implicit-GEMM path (forward with the fused
    epilogue, ReLU-mask + bias gradient, input and weight gradients) against the same
    function in fp32 on the CPU."""
    from mxtrain.ops import convwg
    from mxtrain.ops.epilogue import conv_bias_act
    fwd0, convwg.FWD = convwg.FWD, True
    try:
        _fused_path_case(convwg, conv_bias_act)
    finally:
        convwg.FWD = fwd0


def _fused_path_case(convwg, conv_bias_act):
    torch.manual_seed(1)
    cl = torch.channels_last
    x = torch.randn(2, 128, 64, 64).to(torch.bfloat16)
    w = (torch.randn(256, 128, 3, 3) * 0.05).to(torch.bfloat16)
    b = (torch.randn(256) * 0.1).to(torch.bfloat16)
    r = torch.randn(2, 256, 64, 64).to(torch.bfloat16)
    g = torch.randn(2, 256, 64, 64).to(torch.bfloat16)
    xg = x.cuda().contiguous(memory_format=cl).requires_grad_()
    wg = w.cuda().contiguous(memory_format=cl).requires_grad_()
    bg = b.cuda().requires_grad_()
    rg = r.cuda().contiguous(memory_format=cl).requires_grad_()
    assert convwg.fwd_supported(xg, wg, bg, rg, 1, 1, 1) and convwg.dgrad_supported(wg, tuple(xg.shape), 1)
    y = conv_bias_act(xg, wg, bg, 1, 1, 1, relu=True, residual=rg)
    y.backward(g.cuda().contiguous(memory_format=cl))
    yc = torch.relu(torch.nn.functional.conv2d(x.float(), w.float(), b.float(), 1, 1) + r.float())
    _close(y.detach(), yc)
    # backward against fp32 with the ReLU mask of the bf16 forward (pre-activations near
    # zero may take the other side of the mask in fp32)
    dy = g.float() * (y.detach().float().cpu() > 0)
    dx, dw, _ = torch.ops.aten.convolution_backward(dy, x.float(), w.float(), None, [1, 1], [1, 1], [1, 1], False,
                                                    [0, 0], 1, [True, True, False])
    for got, ref in ((xg.grad, dx), (wg.grad, dw), (bg.grad, dy.sum((0, 2, 3))), (rg.grad, dy)):
        _close(got, ref)


@pytest.mark.parametrize("case", [(1, 128, 64, 13, 9, 3, 1, 1, 1), (2, 256, 128, 25, 42, 1, 1, 0, 1),
                                  (1, 512, 512, 25, 42, 3, 1, 1, 1)])
def test_conv_dgrad_add_and_relu_mask_epilogue(case):
    """dX + add, then * (mask > 0), in the dgrad store (the bottleneck's residual gradient and
    the producer's ReLU) against the fp32 reference of the same three ops; split-K cases
    (first and last) apply them in the ordered reduction, and repeat bitwise."""
    from mxtrain.ops import convwg
    N, Cin, Cout, H, W, k, stride, pad, dil = case
    x, dy = _inputs(*case, seed=17)
    g = torch.Generator().manual_seed(19)
    w = (torch.randn(Cout, k, k, Cin, generator=g) * 0.1).to(torch.bfloat16).cuda().permute(0, 3, 1, 2)
    cl = torch.channels_last
    add = torch.randn(x.shape, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=cl)
    mask = torch.randn(x.shape, generator=g).relu().to(torch.bfloat16).cuda().contiguous(memory_format=cl)
    dx = convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil, add=add, mask=mask)
    ref = (_ref_dx(dy, w, tuple(x.shape), stride, pad, dil) + add.float().cpu()) * (mask.float().cpu() > 0)
    _close(dx, ref)
    assert torch.equal(dx, convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil, add=add, mask=mask))


def test_bottleneck_backward_fusion_matches_unfused(monkeypatch):
    """models/resnet.py Bottleneck with the BlockLink backward fusion (ReLU masks in the
    consumers' dgrad stores, identity residual gradient added in conv1's dgrad) against the
    same blocks with fusion off: identical forward, input and weight gradients equal to bf16
    rounding (the fused path rounds once where the unfused one rounds the dgrad, then adds).
    Shapes sized so every conv takes the implicit-GEMM path (>= 64 output tiles)."""
    from mxtrain.models.resnet import Bottleneck
    from mxtrain.ops import convwg
    monkeypatch.setattr(convwg, "FWD", True)
    monkeypatch.setattr(convwg, "DGRAD", True)
    seen = {"add": 0, "mask": 0}
    real = convwg.conv_dgrad

    def spy(*a, add=None, mask=None, **k):
        seen["add"] += add is not None
        seen["mask"] += mask is not None
        return real(*a, add=add, mask=mask, **k)

    monkeypatch.setattr(convwg, "conv_dgrad", spy)
    torch.manual_seed(3)
    blocks = torch.nn.Sequential(Bottleneck(512, 128, stride=1), Bottleneck(512, 128, stride=1),
                                 Bottleneck(512, 256, stride=2)).cuda()
    for m in blocks.modules():
        if hasattr(m, "norm") and hasattr(m.norm, "running_var"):
            m.norm.running_var.uniform_(0.5, 2.0)
            m.norm.bias.uniform_(-0.2, 0.2)
    x0 = torch.randn(4, 512, 80, 96, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = None
    out = {}
    for fuse in (False, False, True):
        for b in blocks:
            b.fuse_backward = fuse
        seen.update(add=0, mask=0)
        blocks.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        y = blocks(x)
        if gy is None:
            gy = torch.randn_like(y)
        y.backward(gy)
        torch.cuda.synchronize()
        out[fuse] = (y.detach().float(), x.grad.float(),
                     [p.grad.float() for p in blocks.parameters() if p.grad is not None])
    # fused: conv2 + conv3 of all three blocks mask their input, conv1 of the two identity
    # blocks adds, and the second block's conv1 also masks (the first block's ReLU); the
    # projection block's conv1 adds its shortcut's dX and masks the second block's ReLU
    assert seen == {"add": 3, "mask": 8}, seen
    assert torch.equal(out[False][0], out[True][0])
    # the input gradient crosses all three blocks, and the fused path rounds each join once
    # where autograd rounds the dgrad and the add: judge both against an fp32 run of the same
    # blocks -- the fused gradient must be as close to it as the unfused one
    import copy
    b32 = copy.deepcopy(blocks).float()
    for b in b32:
        b.fuse_backward = False
    x32 = x0.float().requires_grad_()
    b32(x32).backward(gy.float())
    e_f = (out[True][1] - x32.grad).abs().max().item()
    e_u = (out[False][1] - x32.grad).abs().max().item()
    assert e_f <= 1.25 * e_u + 1e-3 * x32.grad.abs().max().item(), (e_f, e_u)
    assert len(out[True][2]) == len(out[False][2]) == 10
    for a, b in zip(out[True][2], out[False][2]):
        _close(a, b.cpu())


@pytest.mark.parametrize("cin,hw", [(256, (50, 84)), (512, (50, 84)), (2048, (26, 42))])
def test_conv_bias_act_upsampled_residual_matches_fp32(cin, hw):
    """FPN top-down join in the conv epilogue (ops/epilogue.py conv_bias_act res_up):
    conv1x1(x) + b + up2(r) against fp32 F.conv2d + F.interpolate, values and the input,
    weight, bias and residual gradients (the residual's = 2 x 2 block sums)."""
    import torch.nn.functional as F
    from mxtrain.ops import convwg
    from mxtrain.ops.epilogue import conv_bias_act
    g = torch.Generator().manual_seed(cin)
    cl = torch.channels_last
    H, W = hw      # (26, 42) at 2048 input channels: 18 tiles -> the split-K forward
    x = torch.randn(2 if H > 30 else 1, cin, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(256, cin, 1, 1, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(256, generator=g).to(torch.bfloat16)
    r = torch.randn(x.shape[0], 256, H // 2, W // 2, generator=g).to(torch.bfloat16)
    gy = torch.randn(x.shape[0], 256, H, W, generator=g)
    assert convwg.fwd_supported(x.cuda().contiguous(memory_format=cl), w.cuda().contiguous(memory_format=cl),
                                b.cuda(), r.cuda().contiguous(memory_format=cl), res_up=True)
    xs = [t.cuda().contiguous(memory_format=cl).requires_grad_() if t.dim() == 4 else t.cuda().requires_grad_()
          for t in (x, w, b, r)]
    y = conv_bias_act(xs[0], xs[1], xs[2], residual=xs[3], res_up=True)
    y.backward(gy.to(torch.bfloat16).cuda().contiguous(memory_format=cl))
    rs = [t.float().requires_grad_() for t in (x, w, b, r)]
    yr = F.conv2d(rs[0], rs[1], rs[2]) + F.interpolate(rs[3], scale_factor=2, mode="nearest")
    yr.backward(gy.to(torch.bfloat16).float())
    _close(y, yr.detach())
    for a, ref in zip(xs, rs):
        _close(a.grad, ref.grad)


def test_mask_head_conv_chain_fusion_matches_unfused():
    """models/maskrcnn.py MaskHead: conv i+1's dgrad store applies conv i's ReLU (BlockLink
    chain) -- identical forward, input and parameter gradients equal to the unfused head's
    to bf16 rounding (same bf16 path; an fp32 reference differs wherever a pre-activation
    near zero flips its ReLU mask under bf16, which max-error checks cannot tell from a bug)."""
    from mxtrain.models.maskrcnn import MaskHead
    torch.manual_seed(5)
    head = MaskHead(256, 256, 80)
    for m in head.convs:
        torch.nn.init.normal_(m.bias, std=0.1)
    head = head.cuda()
    x0 = torch.randn(96, 14, 14, 256).to(torch.bfloat16).cuda()
    gy = torch.randn(96, 80, 28, 28).to(torch.bfloat16).cuda().contiguous(memory_format=torch.channels_last)
    out = {}
    try:
        for fuse in (False, True):
            MaskHead.fuse_backward = fuse
            head.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_()
            y = head(x)
            y.backward(gy)
            torch.cuda.synchronize()
            out[fuse] = (y.detach().float(), x.grad.float(), [p.grad.float() for p in head.parameters()])
    finally:
        MaskHead.fuse_backward = True
    assert torch.equal(out[False][0], out[True][0])
    _close(out[True][1], out[False][1].cpu())
    for a, b in zip(out[True][2], out[False][2]):
        _close(a, b.cpu())


@pytest.mark.parametrize("case", [(1, 1024, 512, 50, 84, 1, 2, 0, 1), (1, 1024, 2048, 49, 83, 1, 2, 0, 1),
                                  (2, 512, 256, 40, 40, 1, 2, 0, 1), (1, 256, 256, 28, 30, 2, 2, 0, 1),
                                  (1, 128, 256, 31, 29, 2, 2, 0, 1), (1, 512, 1024, 30, 34, 1, 2, 0, 1)])
@pytest.mark.parametrize("epi", [False, True])
def test_conv_dgrad_stride_decomposed_matches_fp32(case, epi):
    """Stride-decomposed input gradient (1x1 / 2x2 filters at stride 2, odd and even image
    sizes): one GEMM per parity class plus the fill of the pixels no tap reaches, with and
    without the add / ReLU-mask epilogue, against the fp32 reference."""
    from mxtrain.ops import convwg
    N, Cin, Cout, H, W, k, stride, pad, dil = case
    assert convwg.decomposed(k, k, stride, pad, dil)
    x, dy = _inputs(*case, seed=23)
    g = torch.Generator().manual_seed(29)
    w = (torch.randn(Cout, k, k, Cin, generator=g) * 0.1).to(torch.bfloat16).cuda().permute(0, 3, 1, 2)
    cl = torch.channels_last
    add = mask = None
    if epi:
        add = torch.randn(x.shape, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=cl)
        mask = torch.randn(x.shape, generator=g).relu().to(torch.bfloat16).cuda().contiguous(memory_format=cl)
    dx = convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil, add=add, mask=mask)
    ref = _ref_dx(dy, w, tuple(x.shape), stride, pad, dil)
    if epi:
        ref = (ref + add.float().cpu()) * (mask.float().cpu() > 0)
    _close(dx, ref)


@pytest.mark.parametrize("case", [(2, 512, 256, 40, 40, 1, 2, 0, 1), (1, 256, 512, 31, 29, 1, 2, 0, 1)])
def test_conv_dgrad_parity_class_compact(case):
    """1 x 1 stride-2 input gradient as the compact parity class (class_out: dX[:, :, ::2, ::2]
    without the zero fill) and a compact class gradient as the add (add_class: added to the
    class pixels only) against the full-shape launches (ResNet projection blocks)."""
    from mxtrain.ops import convwg
    N, Cin, Cout, H, W, k, stride, pad, dil = case
    x, dy = _inputs(*case, seed=41)
    g = torch.Generator().manual_seed(43)
    w = (torch.randn(Cout, 1, 1, Cin, generator=g) * 0.1).to(torch.bfloat16).cuda().permute(0, 3, 1, 2)
    cl = torch.channels_last
    assert convwg.class_ok(w, tuple(x.shape), stride, pad, dil)
    full = convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil)
    c = convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil, class_out=True)
    assert c.shape == (N, Cin, (H + 1) // 2, (W + 1) // 2) and c.is_contiguous(memory_format=cl)
    assert torch.equal(c, full[:, :, ::2, ::2])
    mask = torch.randn(x.shape, generator=g).relu().to(torch.bfloat16).cuda().contiguous(memory_format=cl)
    spread = torch.zeros(x.shape, dtype=torch.bfloat16, device="cuda").contiguous(memory_format=cl)
    spread[:, :, ::2, ::2] = c
    a = convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil, add=c, mask=mask, add_class=True)
    b = convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil, add=spread, mask=mask)
    assert torch.equal(a, b)


def test_conv_transpose_bias_relu_matches_fp32():
    """Mask-head upsampling (2x2 stride-2 transposed conv + bias + ReLU) on
    ops/epilogue.py ConvTransposeBiasActFn: output and the input, weight and bias gradients
    against fp32 F.conv_transpose2d (gradients through the bf16 output's ReLU mask)."""
    import torch.nn.functional as F
    from mxtrain.ops.epilogue import ConvTransposeBiasActFn, _deconv_ok, conv_transpose_bias_act
    g = torch.Generator().manual_seed(31)
    cl = torch.channels_last
    x = torch.randn(48, 256, 14, 14, generator=g).to(torch.bfloat16)
    w = (torch.randn(256, 256, 2, 2, generator=g) * 0.05).to(torch.bfloat16)
    b = (torch.randn(256, generator=g) * 0.1).to(torch.bfloat16)
    gy = torch.randn(48, 256, 28, 28, generator=g).to(torch.bfloat16)
    xg = x.cuda().contiguous(memory_format=cl).requires_grad_()
    wg, bg = w.cuda().requires_grad_(), b.cuda().requires_grad_()
    assert _deconv_ok(xg, wg, bg, 2)
    y = conv_transpose_bias_act(xg, wg, bg, stride=2, relu=True)
    assert isinstance(y.grad_fn, ConvTransposeBiasActFn._backward_cls), y.grad_fn
    y.backward(gy.cuda().contiguous(memory_format=cl))
    xr, wr, br = (t.float().requires_grad_() for t in (x, w, b))
    yr = F.relu(F.conv_transpose2d(xr, wr, br, stride=2))
    _close(y.detach(), yr.detach())
    (F.conv_transpose2d(xr, wr, br, stride=2) * (y.detach().float().cpu() > 0)).backward(gy.float())
    for got, ref in ((xg.grad, xr.grad), (wg.grad, wr.grad), (bg.grad, br.grad)):
        _close(got, ref)


@pytest.mark.parametrize("case", [(1, 512, 512, 25, 42, 3, 1, 1, 1), (1, 1024, 512, 50, 84, 1, 2, 0, 1),
                                  (1, 256, 256, 25, 42, 3, 1, 1, 1)])
def test_split_k_last_arriver_matches_reduce_launch(case, monkeypatch):
    """Split-K forward / input gradient with the last-arriving split summing the partials in
    the kernel (split_last_arriver) is bit-identical to the separate reduction launch (same
    split-order fp32 sums, same epilogue)."""
    from mxtrain.ops import convwg
    N, Cin, Cout, H, W, k, stride, pad, dil = case
    x, dy = _inputs(*case, seed=21)
    g = torch.Generator().manual_seed(23)
    w = (torch.randn(Cout, k, k, Cin, generator=g) * 0.1).to(torch.bfloat16).cuda().permute(0, 3, 1, 2)
    b = (torch.randn(Cout, generator=g) * 0.1).to(torch.bfloat16).cuda()
    outs = []
    for in_kernel in (False, True):
        monkeypatch.setattr(convwg, "SPLIT_IN_KERNEL", in_kernel)
        y = convwg.conv_fwd(x, w, b, None, True, stride, pad, dil)
        dx = convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil) if convwg.dgrad_supported(
            w, tuple(x.shape), stride, pad, dil) else None
        torch.cuda.synchronize()
        outs.append((y, dx))
    assert torch.equal(outs[0][0], outs[1][0])
    if outs[0][1] is not None:
        assert torch.equal(outs[0][1], outs[1][1])


NARROW = [(2, 256, 16, 80, 104, 1, 1, 0, 1), (48, 256, 80, 28, 28, 1, 1, 0, 1), (4, 128, 24, 66, 68, 1, 1, 0, 1)]


@pytest.mark.parametrize("case", NARROW)
def test_narrow_cout_convs_match_fp32(case):
    """The narrow 1x1 heads (RPN objectness + box: 16 channels, mask logits: 80) on the
    implicit-GEMM kernels with zero-padded tiles: forward (+ bias), input gradient and weight
    gradient (split and unsplit) against fp32 PyTorch, and the fused autograd path."""
    from mxtrain.ops import convwg
    from mxtrain.ops.epilogue import conv_bias_act
    N, Cin, Cout, H, W, k, stride, pad, dil = case
    x, dy = _inputs(*case, seed=31)
    g = torch.Generator().manual_seed(37)
    w = (torch.randn(Cout, k, k, Cin, generator=g) * 0.1).to(torch.bfloat16).cuda().permute(0, 3, 1, 2)
    b = (torch.randn(Cout, generator=g) * 0.1).to(torch.bfloat16).cuda()
    assert convwg.fwd_supported(x, w, b, None, stride, pad, dil)
    y = convwg.conv_fwd(x, w, b, None, False, stride, pad, dil)
    yr = F.conv2d(x.float().cpu(), w.float().cpu(), b.float().cpu(), stride, pad, dil)
    _close(y, yr)
    assert convwg.dgrad_supported(w, tuple(x.shape), stride, pad, dil)
    _close(convwg.conv_dgrad(dy, w, tuple(x.shape), stride, pad, dil), _ref_dx(dy, w, tuple(x.shape), stride, pad, dil))
    for splits in (1, 4, 0):
        _close(convwg.conv_wgrad(dy, x, (Cout, Cin, k, k), stride, pad, dil, splits=splits),
               _ref(dy, x, (Cout, Cin, k, k), stride, pad, dil))
    xg = x.detach().clone().requires_grad_(True)
    wg = w.detach().clone().requires_grad_(True)
    bg = b.detach().clone().requires_grad_(True)
    out = conv_bias_act(xg, wg, bg, stride, pad, dil)
    assert "ConvBiasAct" in type(out.grad_fn).__name__, type(out.grad_fn)
    (out.float() * dy.float()).sum().backward()
    xr = x.float().cpu().requires_grad_(True)
    wr = w.float().cpu().requires_grad_(True)
    br = b.float().cpu().requires_grad_(True)
    (F.conv2d(xr, wr, br, stride, pad, dil) * dy.float().cpu()).sum().backward()
    _close(xg.grad, xr.grad)
    _close(wg.grad, wr.grad)
    _close(bg.grad, br.grad)


def test_projection_block_dx_fold_matches_autograd_add():
    """Bottleneck.fuse_projection: the projection shortcut's input gradient added in conv1's
    dgrad store (with the previous block's ReLU applied there too) gives the gradients of
    autograd's separate add + mask pass."""
    from mxtrain.models.resnet import Bottleneck
    torch.manual_seed(0)
    blk_a = Bottleneck(256, 64).cuda().to(torch.bfloat16)            # identity block
    blk_b = Bottleneck(256, 128, stride=2).cuda().to(torch.bfloat16)  # projection block
    x0 = torch.randn(2, 256, 48, 64, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gout = None
    res = []
    for fold in (False, True):
        Bottleneck.fuse_projection = fold
        for m in (blk_a, blk_b):
            for p in m.parameters():
                p.grad = None
        x = x0.clone().requires_grad_(True)
        y = blk_b(blk_a(x))
        if gout is None:
            gout = torch.randn_like(y)
        y.backward(gout)
        torch.cuda.synchronize()
        res.append([x.grad.float()] + [p.grad.float() for m in (blk_a, blk_b) for p in m.parameters()
                                       if p.grad is not None])
    Bottleneck.fuse_projection = True
    assert len(res[0]) == len(res[1])
    for a, b in zip(*res):
        assert (a - b).abs().max().item() <= 0.02 * a.abs().max().item() + 1e-3


@pytest.mark.gpu
def test_deferred_wgrad_shared_weight_matches_undeferred(monkeypatch):
    """a deferred split-K dW / db is unfinished until the FlatMaster flush, so it
    must never reach autograd's accumulation.  One FlatMaster compute copy (weight AND bias)
    feeds two convolutions (autograd sums their gradients) next to a single-use conv that
    may defer: the flat gradients after the step must match DEFER_WGRAD=False."""
    import copy
    from mxtrain.models.compute_weights import FlatMaster, cw
    from mxtrain.ops import convwg
    from mxtrain.ops.epilogue import conv_bias_act

    class Shared(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Conv2d(256, 256, 3, padding=1)
            self.b = torch.nn.Conv2d(256, 256, 3, padding=1)

        def compute_weight_specs(self):
            return [(p, None) for p in self.parameters()]

        def forward(self, x):
            wa, ba = cw(self.a.weight, torch.bfloat16), cw(self.a.bias, torch.bfloat16)
            wb, bb = cw(self.b.weight, torch.bfloat16), cw(self.b.bias, torch.bfloat16)
            y1 = conv_bias_act(x, wa, ba, padding=1, relu=True)     # shared: used twice
            y2 = conv_bias_act(y1, wa, ba, padding=1, relu=True)
            y3 = conv_bias_act(y2, wb, bb, padding=1, relu=False)   # single use: may defer
            return y3.float().pow(2).mean()

    torch.manual_seed(0)
    base = Shared().cuda()
    x = (torch.randn(2, 256, 64, 96, device="cuda") * 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    grads = {}
    jobs = {}
    real_flush = convwg.defer_flush

    def spy(keep_on=False):
        jobs[cur[0]] = jobs.get(cur[0], 0) + len(convwg._DEF["jobs"]) + len(convwg._DEF["cjobs"])
        return real_flush(keep_on)

    monkeypatch.setattr(convwg, "defer_flush", spy)
    cur = [None]
    for defer in (False, True):
        cur[0] = defer
        monkeypatch.setattr(convwg, "DEFER_WGRAD", defer)
        m = copy.deepcopy(base)
        opt = torch.optim.SGD(m.parameters(), lr=0.0, momentum=0.0)
        fm = FlatMaster(m, opt, 0.0)
        with fm.compute_weights():
            loss = m(x)
        loss.backward()
        fm.step(0.0)
        torch.cuda.synchronize()
        grads[defer] = fm.G.detach().clone()
        assert not convwg._DEF["on"], "deferral must be off after the step"
    assert jobs[False] == 0 and jobs[True] >= 1, jobs   # the single-use conv did defer
    torch.testing.assert_close(grads[True], grads[False], rtol=0, atol=0)
