"""Fused Mask R-CNN training targets (csrc/dettarget.hip) against their PyTorch definitions
(models/maskrcnn.py rpn_targets / sample_rois) on the same random draws: the sampled anchors
and RoIs must be identical, the regression targets equal to fp32 rounding.  Also the
two-launch long-row top-k (ragged last chunk, indices mapped in the merge stage) against
torch.topk, and the fused box encoder against the PyTorch formula."""
import types

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _fake_model():
    from mxtrain.models.maskrcnn import MaskRCNNConfig
    return types.SimpleNamespace(cfg=MaskRCNNConfig())


def _anchors(H, W):
    from mxtrain.models.maskrcnn import MaskRCNNConfig, level_anchors
    cfg = MaskRCNNConfig()
    lv = [level_anchors(s, z, cfg.anchor_ratios, (H + s - 1) // s, (W + s - 1) // s, DEV)
          for s, z in zip(cfg.anchor_strides, cfg.anchor_sizes)]
    return torch.cat(lv, 0)


def _gt(B, G, H, W, counts, seed):
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(B, G, 2, generator=g) * torch.tensor([W * 0.8, H * 0.8])
    wh = 8 + torch.rand(B, G, 2, generator=g) * torch.tensor([W * 0.4, H * 0.4])
    boxes = torch.cat([xy, xy + wh], -1)
    for b, c in enumerate(counts):
        boxes[b, c:] = 0
    return boxes.to(DEV), torch.tensor(counts, dtype=torch.int32, device=DEV)


@pytest.mark.parametrize("counts", [[5, 17], [0, 3, 30]])
def test_rpn_targets_fused_matches_torch(counts):
    from mxtrain.models.maskrcnn import MaskRCNN
    H, W = 320, 448
    B, G = len(counts), 32
    m = _fake_model()
    anchors = _anchors(H, W)
    gt, gc = _gt(B, G, H, W, counts, 1)
    hw = torch.tensor([[H - 13.0, W - 7.0]] * B, device=DEV)
    torch.cuda.manual_seed(11)
    ref = MaskRCNN.rpn_targets(m, anchors, gt, gc, hw)
    torch.cuda.manual_seed(11)
    got = MaskRCNN._rpn_targets_fused(m, anchors, gt, gc, hw)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    assert int(got[0].sum()) > 0 and int(got[1].sum()) > 0
    assert (got[0].sum(1) + got[1].sum(1) <= 256).all()
    torch.testing.assert_close(got[2], ref[2], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("counts", [[5, 17], [0, 3, 30]])
def test_sample_rois_fused_matches_torch(counts):
    from mxtrain.models.maskrcnn import MaskRCNN
    H, W = 320, 448
    B, G, K = len(counts), 32, 1000
    m = _fake_model()
    gt, gc = _gt(B, G, H, W, counts, 2)
    labels = torch.randint(1, 81, (B, G), device=DEV)
    g = torch.Generator().manual_seed(3)
    # proposals: jittered copies of the gt boxes (enough foreground) and random boxes
    base = gt.cpu()[:, torch.randint(0, G, (K,), generator=g)]
    props = (base + torch.randn(B, K, 4, generator=g) * 6).to(DEV)
    rnd = torch.rand(B, K, 2, generator=g) * torch.tensor([W, H]) * 0.9
    props[:, K // 2:] = torch.cat([rnd, rnd + 20], -1)[:, K // 2:].to(DEV)
    torch.cuda.manual_seed(5)
    ref = MaskRCNN.sample_rois(m, props, gt.float(), labels, gc)
    torch.cuda.manual_seed(5)
    got = MaskRCNN._sample_rois_fused(m, props, gt, labels, gc)
    rois, lab, gidx, tgt, is_fg, rois5, rois5_fg = got
    assert torch.equal(rois, ref[0]) and torch.equal(lab, ref[1]) and torch.equal(gidx, ref[2])
    assert torch.equal(is_fg, ref[4])
    torch.testing.assert_close(tgt, ref[3], rtol=1e-5, atol=1e-4)
    N = rois.shape[1]
    nfg = rois5_fg.shape[0] // B
    bi = torch.arange(B, device=DEV, dtype=torch.float32)
    assert torch.equal(rois5, torch.cat([bi[:, None, None].expand(B, N, 1), rois], -1).reshape(-1, 5))
    assert torch.equal(rois5_fg, torch.cat([bi[:, None, None].expand(B, nfg, 1), rois[:, :nfg]], -1).reshape(-1, 5))
    if sum(counts) > 0:
        assert int(is_fg.sum()) > 0


@pytest.mark.parametrize("n,k,largest", [(268_569, 128, False), (268_569, 256, False), (70_001, 100, True),
                                         (40_000, 2048, True)])
def test_topk_rows_long_matches_torch(n, k, largest):
    from mxtrain.ops import vision as V
    g = torch.Generator().manual_seed(n + k)
    x = torch.rand(3, n, generator=g)
    x[:, ::7] = 2.0                       # many ties (the rank-select keys)
    x = x.to(DEV)
    v, i = V.topk_rows(x, k, largest=largest)
    rv, _ = x.topk(k, dim=1, largest=largest)
    assert torch.equal(v, rv)
    assert torch.equal(torch.gather(x, 1, i), v)
    assert all(len(set(r.tolist())) == k for r in i.cpu())


def test_encode_boxes_fused_matches_torch():
    from mxtrain.ops import _lib
    from mxtrain.ops import vision as V
    g = torch.Generator().manual_seed(9)
    a = torch.rand(5000, 2, generator=g) * 500
    ref = torch.cat([a, a + 1 + torch.rand(5000, 2, generator=g) * 100], -1).to(DEV)
    b = torch.rand(5000, 2, generator=g) * 500
    gt = torch.cat([b, b + 1 + torch.rand(5000, 2, generator=g) * 100], -1).to(DEV)
    out = V.encode_boxes(ref, gt, (10.0, 10.0, 5.0, 5.0))
    _lib_on = _lib.use_hip(gt)
    assert _lib_on
    wx, wy, ww, wh = 10.0, 10.0, 5.0, 5.0
    rw = (ref[:, 2] - ref[:, 0]).clamp(min=1e-6)
    rh = (ref[:, 3] - ref[:, 1]).clamp(min=1e-6)
    gw = (gt[:, 2] - gt[:, 0]).clamp(min=1e-6)
    gh = (gt[:, 3] - gt[:, 1]).clamp(min=1e-6)
    exp = torch.stack([wx * (gt[:, 0] + 0.5 * gw - ref[:, 0] - 0.5 * rw) / rw,
                       wy * (gt[:, 1] + 0.5 * gh - ref[:, 1] - 0.5 * rh) / rh,
                       ww * torch.log(gw / rw), wh * torch.log(gh / rh)], 1)
    torch.testing.assert_close(out, exp, rtol=1e-5, atol=1e-4)


def test_rpn_canvas_unpack_flat_matches_per_level():
    """The one-launch flat unpack of the RPN head's canvas output (and its one-launch
    canvas gradient) equals the per-level slices (and their scattered gradients)."""
    from mxtrain.models.maskrcnn import _UnpackFlat, _UnpackLevels, level_canvas
    B, na, C = 2, 3, 16
    shapes = [(50, 84), (25, 42), (13, 21), (7, 11), (4, 6)]
    lay = level_canvas(shapes)
    Hc, Wc, offs = lay
    geo = [(y0, x0, h, w) for (y0, x0), (h, w) in zip(offs, shapes)]
    g = torch.Generator().manual_seed(4)
    o = torch.randn(B, C, Hc, Wc, generator=g).to(torch.bfloat16).to(DEV).contiguous(memory_format=torch.channels_last)
    o1 = o.detach().clone().requires_grad_(True)
    o2 = o.detach().clone().requires_grad_(True)
    ref = _UnpackLevels.apply(o1, geo, na)
    geo5, off = [], 0
    for y0, x0, h, w in geo:
        geo5 += [y0, x0, h, w, off]
        off += h * w * na
    lg, dl = _UnpackFlat.apply(o2, tuple(geo5), na, off)
    assert torch.equal(lg, torch.cat(ref[0::2], 1)) and torch.equal(dl, torch.cat(ref[1::2], 1))
    glg = torch.randn(lg.shape, generator=g).to(torch.bfloat16).to(DEV)
    gdl = torch.randn(dl.shape, generator=g).to(torch.bfloat16).to(DEV)
    (lg.float() * glg.float()).sum().backward(retain_graph=True)
    (dl.float() * gdl.float()).sum().backward()
    gl_lv, gd_lv, off = [], [], 0
    for _, _, h, w in geo:
        n = h * w * na
        gl_lv.append(glg[:, off:off + n])
        gd_lv.append(gdl[:, off:off + n])
        off += n
    loss = sum((r.float() * t.float()).sum() for r, t in zip(ref, [x for pair in zip(gl_lv, gd_lv) for x in pair]))
    loss.backward()
    assert torch.equal(o2.grad, o1.grad)


def test_fpn_fanout_gradient_sum():
    """_FanOut3: the three consumers' gradients of an FPN level (a strided canvas slice, two
    contiguous NHWC RoIAlign gradients, any of them absent) summed in one pass."""
    from mxtrain.models.maskrcnn import _FanOut3
    B, C, H, W = 2, 256, 25, 42
    cl = torch.channels_last
    g = torch.Generator().manual_seed(8)
    bf = lambda *s: torch.randn(*s, generator=g).to(torch.bfloat16).to(DEV)  # noqa: E731
    p = bf(B, C, H, W).contiguous(memory_format=cl).requires_grad_(True)
    canvas = bf(B, C, H + 30, W + 7).contiguous(memory_format=cl)
    ga = canvas[:, :, 10:10 + H, 3:3 + W]                   # canvas-gradient slice (strided)
    gb = bf(B, H, W, C).permute(0, 3, 1, 2)
    gc = bf(B, H, W, C).permute(0, 3, 1, 2)
    for use in ((1, 1, 1), (1, 1, 0), (0, 1, 1), (1, 0, 0)):
        p.grad = None
        a, b, c = _FanOut3.apply(p)
        loss = sum((o.float() * t.float()).sum() for o, t, u in zip((a, b, c), (ga, gb, gc), use) if u)
        loss.backward()
        exp = sum(t.float() for t, u in zip((ga, gb, gc), use) if u)
        torch.testing.assert_close(p.grad.float(), exp, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("B,L,pre,top", [(1, 5, 2000, 2000), (4, 5, 2000, 2000), (2, 3, 700, 1000), (3, 8, 64, 100)])
def test_merge_sorted_topk_matches_topk_rows(B, L, pre, top):
    """The post-NMS merge of L sorted level lists (with duplicated scores across and within
    lists and -inf tails) equals topk_rows over the flattened lists: values and indices."""
    from mxtrain.ops import vision as V
    g = torch.Generator().manual_seed(B * 100 + L)
    x = (torch.rand(B, L, pre, generator=g) * 50).round() / 50     # many ties
    x = torch.sort(x, dim=-1, descending=True)[0]
    nvalid = torch.randint(pre // 3, pre + 1, (B, L), generator=g)
    x[torch.arange(pre)[None, None] >= nvalid[..., None]] = -float("inf")
    x = x.to(DEV)
    v, i = V.merge_sorted_topk(x, top)
    rv, ri = V.topk_rows(x.reshape(B, L * pre), top)
    assert torch.equal(v, rv)
    assert torch.equal(i, ri)


def test_fpn_join_backward_matches_autograd_add():
    """FPN top-down join with the two gradients of each merged level summed inside the kernels
    (JoinLink: output conv dgrad store / 2x2 block-sum kernel) equals the unfused backward
    (autograd's add of the output conv's input gradient and the upsampling gradient)."""
    from mxtrain.models.maskrcnn import FPN
    torch.manual_seed(0)
    chans = [256, 512, 1024, 2048]
    shapes = [(48, 64), (24, 32), (12, 16), (6, 8)]
    fpn = FPN(chans, 256).to(DEV).to(torch.bfloat16)
    feats = [torch.randn(2, c, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
             for c, (h, w) in zip(chans, shapes)]
    gouts = None
    res = []
    for join in (False, True):
        FPN.join_backward = join
        fs = [f.detach().clone().requires_grad_(True) for f in feats]
        for p in fpn.parameters():
            p.grad = None
        outs = fpn(fs)
        if gouts is None:
            gouts = [torch.randn_like(o) for o in outs]
        sum((o.float() * g.float()).sum() for o, g in zip(outs, gouts)).backward()
        res.append([f.grad.float() for f in fs] + [p.grad.float() for p in fpn.parameters()])
    FPN.join_backward = True
    for a, b in zip(*res):
        torch.testing.assert_close(b, a, rtol=3e-2, atol=3e-2 * float(a.abs().max()) + 1e-3)


def test_fpn_join_graph_replay_matches_eager():
    """The FPN forward + backward with JoinLink captured in a hipGraph and replayed gives the
    eager gradients bit for bit (the parked-gradient protocol is host-side, fixed at capture)."""
    from mxtrain.models.maskrcnn import FPN
    torch.manual_seed(0)
    chans = [256, 512, 1024, 2048]
    shapes = [(96, 128), (48, 64), (24, 32), (12, 16)]
    fpn = FPN(chans, 256).to(DEV).to(torch.bfloat16)
    params = list(fpn.parameters())
    # the coarse levels' convs fall below the implicit-GEMM tile floor and run on MIOpen,
    # whose default solvers are not bit-reproducible run to run
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    feats = [torch.randn(2, c, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
             .requires_grad_(True) for c, (h, w) in zip(chans, shapes)]
    with torch.no_grad():
        gouts = [torch.randn_like(o) for o in fpn(feats)]

    def step():
        for p in params + feats:
            p.grad = None
        outs = fpn(feats)
        torch.autograd.backward(outs, gouts)
        return [t.grad for t in feats + params]

    ref = [g.clone() for g in step()]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    for p in params + feats:
        p.grad = None
    with torch.cuda.graph(g):
        outs = fpn(feats)
        torch.autograd.backward(outs, gouts)
    grads = [t.grad for t in feats + params]
    g.replay()
    torch.cuda.synchronize()
    torch.backends.cudnn.deterministic = det
    for a, b in zip(ref, grads):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N,H,W", [(2, 96, 160), (1, 101, 133), (1, 800, 1216)])
def test_fused_stem_pool_matches_fp32(N, H, W):
    """csrc/stem.hip (normalise + 7x7/2 conv + bias + ReLU + 3x3/2 max-pool from the uint8
    image) against the fp32 torch reference of the same op, odd sizes included (border
    windows, the last image's final bytes)."""
    from mxtrain.ops import stem as S
    torch.manual_seed(0)
    img = torch.randint(0, 256, (N, 3, H, W), dtype=torch.uint8, device=DEV)
    wf = (torch.randn(64, 3, 7, 7, device=DEV) * 0.05).to(torch.bfloat16)
    bf = (torch.randn(64, device=DEV) * 0.1).to(torch.bfloat16)
    mean, std = (123.675, 116.28, 103.53), (58.395, 57.12, 57.375)
    assert S.supported(img, wf, bf)
    got = S.stem_pool(img, wf, bf, mean, std).float()
    ref = S.stem_pool_ref(img, wf, bf, mean, std).float()
    assert got.shape == ref.shape
    err = (got - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("H,W", [(25, 42), (13, 21), (24, 40)])
def test_subsample2_matches_maxpool_1x1_stride2(H, W):
    """FPN P6 (mx_subsample2) forward and backward bit-identical to F.max_pool2d(x, 1, 2)."""
    from mxtrain.ops.epilogue import subsample2
    torch.manual_seed(0)
    x = torch.randn(2, 256, H, W, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = subsample2(xa), F.max_pool2d(xb, 1, 2)
    assert torch.equal(ya, yb)
    g = torch.randn_like(yb)
    ya.backward(g)
    yb.backward(g)
    assert torch.equal(xa.grad, xb.grad)


def test_rpn_head_relu_fold_matches_unfolded():
    """RPNHead.forward_levels with the 3x3 conv's ReLU applied in the 1x1's input-gradient
    store (BlockLink mask_in) gives the same gradients as the unfolded head."""
    from mxtrain.models.maskrcnn import RPNHead
    torch.manual_seed(0)
    head = RPNHead(256, 3).to(DEV).to(torch.bfloat16)
    shapes = [(64, 96), (32, 48), (16, 24), (8, 12), (4, 6)]
    P = [torch.randn(2, 256, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
         for h, w in shapes]
    outs = []
    for fold in (False, True):
        head.fold_relu = fold
        for p in head.parameters():
            p.grad = None
        Pg = [p.clone().requires_grad_(True) for p in P]
        lv = head.forward_levels(Pg)
        g = torch.Generator(device=DEV).manual_seed(3)
        loss = sum((l.float() * torch.randn(l.shape, device=DEV, generator=g)).sum()
                   + (d.float() * torch.randn(d.shape, device=DEV, generator=g)).sum() for l, d in lv)
        loss.backward()
        torch.cuda.synchronize()
        outs.append([p.grad.float().clone() for p in head.parameters()] + [p.grad.float().clone() for p in Pg])
    head.fold_relu = True
    for a, b in zip(*outs):
        assert (a - b).abs().max().item() <= 0.02 * a.abs().max().item() + 1e-3


def test_nms_merge_topk_matches_torch_tail():
    """ops/vision.py nms_merge_topk (one launch) against the torch tail it replaces: gathers of
    the NMS survivors' scores and boxes, -inf padding, the sorted-list merge and the final
    box gather -- bit-identical."""
    from mxtrain.ops import vision as V
    torch.manual_seed(0)
    B, L, pre, top = 2, 5, 300, 400
    P = B * L
    scores = torch.rand(P, pre, device=DEV).sort(1, descending=True).values
    scores[3, 250:] = -float("inf")
    c = torch.rand(P, pre, 2, device=DEV) * 500
    wh = 10 + torch.rand(P, pre, 2, device=DEV) * 60
    boxes = torch.cat([c, c + wh], -1).contiguous()
    cnt = torch.full((P,), pre, dtype=torch.int32, device=DEV)
    keep, _ = V.batched_nms_sorted(boxes, cnt, 0.7, pre, raw=True)
    b, s = V.nms_merge_topk(keep, scores, boxes, B, L, top)
    k64 = keep.long()
    valid = k64 >= 0
    ki = k64.clamp(min=0)
    kb = torch.gather(boxes, 1, ki[..., None].expand(-1, -1, 4)).view(B, L * pre, 4)
    ks = torch.where(valid, torch.gather(scores, 1, ki), torch.full_like(scores, -float("inf")))
    s_ref, i_ref = V.merge_sorted_topk(ks.view(B, L, pre), top)
    b_ref = torch.gather(kb, 1, i_ref[..., None].expand(-1, -1, 4))
    assert torch.equal(s, s_ref)
    assert torch.equal(b, b_ref)
