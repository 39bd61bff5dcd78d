"""Detection ops (K13-K15): RoIAlign / NMS / matching / decode.  CPU: the PyTorch
references against brute-force per-sample loops.  GPU: the HIP kernels against the fp32
references (forward values, RoIAlign gradients, exact NMS keep lists)."""
import math

import numpy as np
import pytest
import torch

from mxtrain.ops import vision as V


def _bilinear_loop(f, y, x):
    H, W = f.shape[0], f.shape[1]
    if y < -1 or y > H or x < -1 or x > W:
        return torch.zeros(f.shape[-1])
    y, x = max(y, 0.0), max(x, 0.0)
    yl, xl = int(y), int(x)
    if yl >= H - 1:
        yh = yl = H - 1
        y = float(yl)
    else:
        yh = yl + 1
    if xl >= W - 1:
        xh = xl = W - 1
        x = float(xl)
    else:
        xh = xl + 1
    ly, lx = y - yl, x - xl
    return ((1 - ly) * (1 - lx) * f[yl, xl] + (1 - ly) * lx * f[yl, xh] + ly * (1 - lx) * f[yh, xl] +
            ly * lx * f[yh, xh])


def _roi_align_loop(feat, roi, scale, PH, PW, sr):
    b, x1, y1, x2, y2 = roi.tolist()
    f = feat[int(b)]
    x0, y0 = x1 * scale - 0.5, y1 * scale - 0.5
    rw, rh = x2 * scale - 0.5 - x0, y2 * scale - 0.5 - y0
    out = torch.zeros(PH, PW, f.shape[-1])
    for ph in range(PH):
        for pw in range(PW):
            acc = 0
            for iy in range(sr):
                for ix in range(sr):
                    y = y0 + ph * rh / PH + (iy + 0.5) * rh / PH / sr
                    x = x0 + pw * rw / PW + (ix + 0.5) * rw / PW / sr
                    acc = acc + _bilinear_loop(f, y, x)
            out[ph, pw] = acc / (sr * sr)
    return out


def _rand_rois(R, B, H, W, gen):
    x1 = torch.rand(R, generator=gen) * W * 0.8
    y1 = torch.rand(R, generator=gen) * H * 0.8
    w = torch.rand(R, generator=gen) * W * 0.5 + 2
    h = torch.rand(R, generator=gen) * H * 0.5 + 2
    b = torch.randint(0, B, (R,), generator=gen).float()
    return torch.stack([b, x1, y1, x1 + w, y1 + h], 1)


def test_roi_align_reference_matches_loop():
    g = torch.Generator().manual_seed(0)
    feat = torch.randn(2, 12, 16, 8, generator=g)
    rois = _rand_rois(5, 2, 48, 64, g)
    out = V._ref_roi_align([feat], [0.25], rois, 3, 4, 2, True, 2, 224.0, 4)
    for r in range(5):
        torch.testing.assert_close(out[r], _roi_align_loop(feat, rois[r], 0.25, 3, 4, 2), rtol=1e-4, atol=1e-5)


def test_nms_and_match_reference():
    g = torch.Generator().manual_seed(1)
    xy = torch.rand(60, 2, generator=g) * 100
    boxes = torch.cat([xy, xy + torch.rand(60, 2, generator=g) * 40 + 5], 1)
    scores = torch.rand(60, generator=g)
    keep = V.nms(boxes, scores, 0.5)
    # greedy definition
    order = scores.argsort(descending=True).tolist()
    iou = V.box_iou(boxes, boxes)
    ref, supp = [], set()
    for i in order:
        if i in supp:
            continue
        ref.append(i)
        supp |= {j for j in range(60) if iou[i, j] > 0.5}
    assert keep.tolist() == ref
    gt = boxes[:7][None]
    mi, am, lq = V.match_boxes(boxes, gt, torch.tensor([7]))
    torch.testing.assert_close(mi[0], iou[:, :7].max(1).values)
    assert (lq[0, :7] >= 0).all()


def test_decode_inverts_encode():
    g = torch.Generator().manual_seed(2)
    ref = torch.cat([torch.rand(50, 2, generator=g) * 50, torch.rand(50, 2, generator=g) * 50 + 60], 1)
    gt = torch.cat([torch.rand(50, 2, generator=g) * 50, torch.rand(50, 2, generator=g) * 50 + 60], 1)
    w = (10.0, 10.0, 5.0, 5.0)
    torch.testing.assert_close(V.decode_boxes(ref, V.encode_boxes(ref, gt, w), w), gt, rtol=1e-4, atol=1e-3)


def _tiny_rois(R, B, gen):
    """Concentrated small boxes (what a random-init RPN proposes): most entries land in a
    few P2 tiles, which the tiled backward splits into several chunks + a combine pass."""
    cx = 300 + torch.rand(R, generator=gen) * 40
    cy = 200 + torch.rand(R, generator=gen) * 40
    w = 4 + torch.rand(R, generator=gen) * 20
    h = 4 + torch.rand(R, generator=gen) * 20
    b = torch.randint(0, B, (R,), generator=gen).float()
    return torch.stack([b, cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], 1)


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [True, False])
@pytest.mark.parametrize("out_hw", [7, 14])
@pytest.mark.parametrize("spread", ["spread", "tiny"])
def test_roi_align_gpu_fwd_bwd(tiled, out_hw, spread, monkeypatch):
    """Forward and both backward kernels (tiled -- the MFMA kernel at C = 256 -- / fp32
    atomics) vs the fp32 torch reference, on spread-out boxes and on concentrated tiny ones
    (split tiles); the tiled backward is also bitwise deterministic across runs."""
    monkeypatch.setattr(V, "_TILED", tiled)
    g = torch.Generator().manual_seed(3)
    B, C = 2, 256
    shapes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    scales = [1 / 4, 1 / 8, 1 / 16, 1 / 32]
    feats = [torch.randn(B, h, w, C, generator=g).bfloat16() for h, w in shapes]
    # (tiny: 9800 items -- 200 boxes at 7 x 7, 50 at 14 x 14 -- so no tile exceeds the
    # 16384-entry sort that keeps split tiles deterministic)
    rois = _rand_rois(300, B, 800, 1344, g) if spread == "spread" else _tiny_rois(9800 // (out_hw * out_hw), B, g)
    ref_in = [f.float().requires_grad_(True) for f in feats]
    ref = V._ref_roi_align(ref_in, scales, rois, out_hw, out_hw, 2, True, 2, 224.0, 4)
    fg = [f.cuda().requires_grad_(True) for f in feats]
    out = V.roi_align(fg, rois.cuda(), (out_hw, out_hw), scales)
    torch.testing.assert_close(out.float().cpu(), ref, rtol=2e-2, atol=2e-2)
    dout = torch.randn(ref.shape, generator=g)
    (ref * dout).sum().backward()
    (out.float() * dout.cuda()).sum().backward()
    for a, b in zip(fg, ref_in):
        bg = b.grad if b.grad is not None else torch.zeros_like(b)   # a level no RoI maps to
        err = (a.grad.float().cpu() - bg).norm() / (bg.norm() + 1e-6)
        assert err < 2e-2 or bg.norm() == 0 and a.grad.abs().max() == 0, float(err)
    if tiled:
        assert V.tiled_overflow() == 0
        first = [f.grad.clone() for f in fg]
        for f in fg:
            f.grad = None
        out = V.roi_align(fg, rois.cuda(), (out_hw, out_hw), scales)
        (out.float() * dout.cuda()).sum().backward()
        assert all(torch.equal(a, f.grad) for a, f in zip(first, fg))


@pytest.mark.gpu
@pytest.mark.parametrize("N,max_out", [(2000, 1000), (700, 700), (3000, 3000)])
def test_nms_match_decode_gpu(N, max_out):
    g = torch.Generator().manual_seed(4)
    P = 5
    xy = torch.rand(P, N, 2, generator=g) * 700
    boxes = torch.cat([xy, xy + torch.rand(P, N, 2, generator=g) * 120 + 4], 2)
    counts = torch.tensor([N, min(N, 1500), 64, 1, 0])
    kg, ng = V.batched_nms_sorted(boxes.cuda(), counts.cuda(), 0.7, max_out)
    kc, nc = V.batched_nms_sorted(boxes, counts, 0.7, max_out)
    assert ng.cpu().tolist() == nc.tolist()
    assert torch.equal(kg.cpu(), kc)
    anchors = boxes[0]
    gt = boxes[1:3, :20]
    gc = torch.tensor([20, 7])
    a = V.match_boxes(anchors.cuda(), gt.cuda(), gc.cuda())
    b = V.match_boxes(anchors, gt, gc)
    torch.testing.assert_close(a[0].cpu(), b[0], rtol=1e-5, atol=1e-6)
    same = a[0].cpu() > 0
    assert torch.equal(a[1].cpu()[same], b[1][same])
    assert torch.equal(a[2].cpu(), b[2])
    d = torch.randn(N, 4, generator=g)
    hw = torch.tensor([[800.0, 1344.0]])
    torch.testing.assert_close(V.decode_boxes(anchors.cuda(), d.cuda(), (10, 10, 5, 5), hw.cuda()).cpu(),
                               V.decode_boxes(anchors, d, (10, 10, 5, 5), hw), rtol=1e-4, atol=1e-2)


@pytest.mark.gpu
def test_crop_resize_mask_crops_gpu():
    """Packed-crop mask targets (HIP) == full-mask fp32 reference on the unpacked masks."""
    from mxtrain.data.coco import unpack_mask_crops
    g = torch.Generator().manual_seed(5)
    B, G, H, W = 2, 6, 320, 512
    table = torch.zeros(B, G, 5, dtype=torch.int32)
    parts, off = [], 0
    for b in range(B):
        for k in range(G - 1):                      # last slot is padding (w = h = 0)
            x0, y0 = int(torch.randint(0, W - 40, (1,), generator=g)), int(torch.randint(0, H - 40, (1,), generator=g))
            cw, ch = int(torch.randint(1, W - x0, (1,), generator=g)), int(torch.randint(1, H - y0, (1,), generator=g))
            c = (torch.rand(ch, cw, generator=g) > 0.4).to(torch.uint8)
            table[b, k] = torch.tensor([off, x0, y0, cw, ch])
            parts.append(c.reshape(-1))
            off += ch * cw
    flat = torch.cat(parts)
    full = unpack_mask_crops(flat, table, H, W).reshape(-1, H, W)
    R = 500
    gid = torch.randint(0, B * G, (R,), generator=g)
    xy = torch.rand(R, 2, generator=g) * torch.tensor([W, H]) - 20
    boxes = torch.cat([xy, xy + torch.rand(R, 2, generator=g) * 200 + 1], 1)
    ref = V.crop_resize_masks(full, boxes, gid)
    out = V.crop_resize_mask_crops(flat.cuda(), table.reshape(-1, 5).cuda(), H, W, boxes.cuda(), gid.cuda())
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-4, atol=1e-4)   # fma vs separate mul-add


@pytest.mark.gpu
@pytest.mark.parametrize("relu,res,bias_grad,k,cout", [(True, False, False, 3, 128), (False, False, True, 3, 128),
                                                       (True, True, False, 3, 128), (True, False, True, 3, 128),
                                                       (True, True, True, 1, 128), (False, False, True, 1, 128),
                                                       (True, True, True, 3, 120)])   # 120: non-power-of-two bias index
def test_conv_bias_act_gpu(relu, res, bias_grad, k, cout):
    """Fused conv epilogue (csrc/epilogue.hip) vs the fp32 torch reference: forward and
    the gradients of input, weight, bias and residual."""
    from mxtrain.ops import epilogue as E
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 64, 20, 24, generator=g)
    w = torch.randn(cout, 64, k, k, generator=g) * 0.05
    b = torch.randn(cout, generator=g)
    r = torch.randn(2, cout, 20, 24, generator=g)
    dout = torch.randn(2, cout, 20, 24, generator=g)

    def run(dev, dt, fused):
        xx = x.detach().clone().to(dev, dt).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        ww = w.detach().clone().to(dev, dt).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        bb = b.detach().clone().to(dev, dt).requires_grad_(bias_grad)
        rr = (r.detach().clone().to(dev, dt).contiguous(memory_format=torch.channels_last).requires_grad_(True)
              if res else None)
        if fused:
            y = E.conv_bias_act(xx, ww, bb, padding=k // 2, relu=relu, residual=rr)
        else:
            y = torch.nn.functional.conv2d(xx, ww, bb, padding=k // 2)
            y = y + rr if res else y
            y = torch.relu(y) if relu else y
        (y.float() * dout.to(dev)).sum().backward()
        grads = [xx.grad, ww.grad] + ([bb.grad] if bias_grad else []) + ([rr.grad] if res else [])
        return y.detach().float().cpu(), [t.float().cpu() for t in grads]

    y_ref, g_ref = run("cpu", torch.float32, False)
    y_t, g_t = run("cuda", torch.bfloat16, False)     # PyTorch's own bf16 path on the GPU
    y, gs = run("cuda", torch.bfloat16, True)
    assert (y - y_ref).abs().max() / y_ref.abs().max() < 2e-2
    errs = [(float((a - r).norm() / (r.norm() + 1e-6)), float((t - r).norm() / (r.norm() + 1e-6)))
            for a, t, r in zip(gs, g_t, g_ref)]
    for fused_err, torch_err in errs:   # as close to fp32 as the unfused bf16 ops are
        assert fused_err < max(2e-2, 1.5 * torch_err), errs


@pytest.mark.gpu
def test_level_topk_decode_gpu_matches_stable_reference():
    """csrc/vision.hip tk_*: top-k of bf16 logits per (image, level) with ties broken by the
    lower anchor index, decoded + clipped boxes, -inf padding of short levels."""
    g = torch.Generator().manual_seed(11)
    B, k = 2, 2000
    ns = [60000, 15000, 3800, 950, 240]
    # quantised logits: many exact ties, including at the k-th value
    lgs = [(torch.randint(-300, 300, (B, n), generator=g).float() / 64).to(torch.bfloat16) for n in ns]
    dls = [(0.3 * torch.randn(B, n, 4, generator=g)).to(torch.bfloat16) for n in ns]
    ans = []
    for n in ns:
        xy = torch.rand(n, 2, generator=g) * 800
        ans.append(torch.cat([xy, xy + torch.rand(n, 2, generator=g) * 200 + 8], 1))
    hw = torch.tensor([[800.0, 1216.0], [768.0, 1333.0]])
    bx, sc, cnt = V.level_topk_decode([t.cuda() for t in lgs], [t.cuda() for t in dls], [t.cuda() for t in ans],
                                      hw.cuda(), k)
    assert cnt == [min(k, n) for n in ns]
    bx, sc = bx.cpu(), sc.cpu()
    for li, (lg, dl, an) in enumerate(zip(lgs, dls, ans)):
        kk = min(k, lg.shape[1])
        for b in range(B):
            order = torch.sort(-lg[b].float(), stable=True).indices[:kk]
            torch.testing.assert_close(sc[b, li, :kk], lg[b].float()[order], rtol=0, atol=0)
            assert torch.all(sc[b, li, kk:] == -float("inf"))
            ref = V.decode_boxes(an[order], dl[b].float()[order], (1.0, 1.0, 1.0, 1.0), hw[b:b + 1])
            torch.testing.assert_close(bx[b, li, :kk], ref, rtol=1e-5, atol=1e-3)
    # a second call (histograms re-zeroed by the first) gives the same result
    bx2, sc2, _ = V.level_topk_decode([t.cuda() for t in lgs], [t.cuda() for t in dls], [t.cuda() for t in ans],
                                      hw.cuda(), k)
    assert torch.equal(sc2.cpu(), sc) and torch.equal(bx2.cpu(), bx)


@pytest.mark.gpu
def test_fused_detection_losses_match_torch():
    """csrc/detloss.hip: RPN, Fast R-CNN and mask losses (values and input gradients)
    against the torch formulas (ops/detloss.py *_ref) on the same bf16 inputs."""
    from mxtrain.ops import detloss as D
    g = torch.Generator().manual_seed(5)
    dev = "cuda"

    def run(fused, ref, inputs, grad_idx):
        xs = [t.clone().requires_grad_(i in grad_idx) for i, t in enumerate(inputs)]
        ys = [t.clone().requires_grad_(i in grad_idx) for i, t in enumerate(inputs)]
        a = fused(*xs)
        b = ref(*ys)
        a = a if isinstance(a, tuple) else (a,)
        b = b if isinstance(b, tuple) else (b,)
        for u, v in zip(a, b):
            torch.testing.assert_close(u.float(), v.float(), rtol=2e-4, atol=1e-5)
        w = [1.3, 0.7][:len(a)]
        sum(wi * u for wi, u in zip(w, a)).backward()
        sum(wi * v for wi, v in zip(w, b)).backward()
        for i in grad_idx:
            torch.testing.assert_close(xs[i].grad.float(), ys[i].grad.float(), rtol=2e-2, atol=2e-5)

    # RPN: B=2, A=5000
    B, A = 2, 5000
    lg = torch.randn(B, A, generator=g).to(torch.bfloat16).to(dev)
    dl = (0.2 * torch.randn(B, A, 4, generator=g)).to(torch.bfloat16).to(dev)
    enc = (0.2 * torch.randn(B, A, 4, generator=g)).to(dev)
    pos = (torch.rand(B, A, generator=g) < 0.02).to(dev)
    neg = ((torch.rand(B, A, generator=g) < 0.05) & ~pos.cpu()).to(dev)
    run(lambda a, b, c, d, e: D.rpn_loss(a, b, c, d, e, B * 256),
        lambda a, b, c, d, e: D.rpn_loss_ref(a, b, c, d, e, B * 256), [lg, dl, enc, pos, neg], (0, 1))
    # Fast R-CNN: N=1024 RoIs, 81 classes
    N, C = 1024, 81
    cl = torch.randn(N, C, generator=g).to(torch.bfloat16).to(dev)
    bd = (0.3 * torch.randn(N, C * 4, generator=g)).to(torch.bfloat16).to(dev)
    lab = torch.randint(0, C, (N,), generator=g).to(dev)
    fg = (lab > 0) & (torch.rand(N, generator=g) < 0.5).to(dev)
    tg = (0.3 * torch.randn(N, 4, generator=g)).to(dev)
    run(lambda a, b, c, d, e: D.frcnn_loss(a, b, c, d, e, N), lambda a, b, c, d, e: D.frcnn_loss_ref(a, b, c, d, e, N),
        [cl, bd, lab, tg, fg], (0, 1))
    # mask: R=64 RoIs, 80 classes, 28x28, channels_last logits
    R, K = 64, 80
    ml = torch.randn(R, K, 28, 28, generator=g).to(torch.bfloat16).to(dev).contiguous(memory_format=torch.channels_last)
    ml_lab = torch.randint(0, K + 1, (R,), generator=g).to(dev)
    tm = torch.rand(R, 28, 28, generator=g).to(dev)
    valid = (torch.rand(R, generator=g) < 0.7).float().to(dev)
    run(D.mask_loss, D.mask_loss_ref, [ml, ml_lab, tm, valid], (0,))


@pytest.mark.gpu
@pytest.mark.parametrize("R,n,k,largest", [(2, 10000, 2000, True), (4, 2100, 512, True), (2, 2100, 128, False),
                                           (1, 300, 300, True), (3, 32768, 2048, False), (8, 64, 1, True),
                                           # long rows: chunked two-stage (RPN anchor sampling)
                                           (2, 268569, 256, False), (1, 100000, 512, True), (2, 40000, 2048, True)])
def test_topk_rows_matches_torch(R, n, k, largest):
    """csrc/vision.hip topk_rows_kernel vs torch.topk: identical values; indices point at
    those values, are distinct, and order equal values by lower index (ties forced by
    -inf padding / repeated keys)."""
    from mxtrain.ops.vision import topk_rows
    g = torch.Generator(device="cuda").manual_seed(n + k)
    x = torch.rand(R, n, device="cuda", generator=g)
    x[:, ::7] = -float("inf") if largest else float("inf")     # many exact ties
    x[:, 1::5] = 0.5                                            # ties inside the selection
    v, i = topk_rows(x, k, largest=largest)
    rv, _ = x.topk(k, dim=1, largest=largest)
    torch.cuda.synchronize()
    assert torch.equal(v, rv)
    assert torch.equal(torch.gather(x, 1, i), v)
    for r in range(R):
        assert i[r].unique().numel() == k
        # equal values: lower index first
        same = v[r, 1:] == v[r, :-1]
        assert bool((i[r, 1:][same] > i[r, :-1][same]).all())


@pytest.mark.gpu
@pytest.mark.parametrize("n,k", [(8192, 100), (16384, 1000), (4100, 64)])
def test_topk_rows_ties_early_larger_keys_late(n, k):
    """The exit race of topk_rows_kernel's candidate scan: the threshold ties
    fill in the FIRST 1024-element chunk while every key above the threshold sits in later
    chunks, so the scan must keep going after the ties are complete and all waves must
    leave on the same chunk."""
    from mxtrain.ops.vision import topk_rows
    R = 6
    x = torch.zeros(R, n, device="cuda")
    x[:, : 2 * k] = 0.5                                # ties: threshold value, chunk 0 only
    n_gt = k // 2
    late = torch.linspace(1024, n - 1, n_gt, device="cuda").long()
    for r in range(R):
        x[r, late] = 1.0 + torch.arange(n_gt, device="cuda", dtype=torch.float32) / n_gt + r
    for _ in range(20):                                 # exercise many wave interleavings
        v, i = topk_rows(x, k, largest=True)
        rv, ri = x.topk(k, dim=1, largest=True)
        torch.cuda.synchronize()
        assert torch.equal(v, rv)
        assert torch.equal(torch.gather(x, 1, i), v)
        for r in range(R):
            assert i[r].unique().numel() == k
            # the tied part is the lowest indices, in order
            assert torch.equal(i[r, n_gt:].sort().values, torch.arange(k - n_gt, device="cuda"))


@pytest.mark.gpu
def test_rpn_level_canvas_pack_gpu():
    """models/maskrcnn.py _PackLevels on the GPU (csrc/vision.hip copy_rows_kernel): the
    canvas equals the levels placed by slicing, zeros elsewhere; the backward hands each
    level its slice of the canvas gradient."""
    from mxtrain.models.maskrcnn import _PackLevels, level_canvas
    g = torch.Generator().manual_seed(11)
    shapes = [(200, 336), (100, 168), (50, 84), (25, 42), (13, 21)]
    lay = level_canvas(shapes)
    assert lay is not None
    cl = torch.channels_last
    lv = [torch.randn(2, 256, h, w, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=cl).requires_grad_()
          for h, w in shapes]
    c = _PackLevels.apply(lay, *lv)
    Hc, Wc, offs = lay
    ref = torch.zeros(2, 256, Hc, Wc, dtype=torch.bfloat16)
    for (y0, x0), p in zip(offs, lv):
        ref[:, :, y0:y0 + p.shape[2], x0:x0 + p.shape[3]] = p.detach().cpu()
    assert torch.equal(c.detach().cpu(), ref)
    gc = torch.randn(c.shape, generator=g).to(torch.bfloat16).cuda()
    c.backward(gc)
    for (y0, x0), p in zip(offs, lv):
        assert torch.equal(p.grad.cpu(), gc[:, :, y0:y0 + p.shape[2], x0:x0 + p.shape[3]].cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("N,max_out", [(2000, 2000), (2000, 300), (130, 17), (4096, 1000)])
def test_nms_parallel_scan_matches_serial(N, max_out):
    """Boxes clustered around a few objects (long suppression chains inside a 64-box chunk):
    the fixed-point in-chunk scan (nms_keep_par_kernel) and the serial one give the greedy
    CPU result, including the max_out cut inside a chunk."""
    from mxtrain.ops import _lib
    g = torch.Generator().manual_seed(N + max_out)
    P = 4
    ctr = torch.rand(P, 12, 2, generator=g) * 600
    pick = torch.randint(0, 12, (P, N), generator=g)
    c = torch.gather(ctr, 1, pick[..., None].expand(P, N, 2)) + torch.randn(P, N, 2, generator=g) * 6
    wh = 30 + torch.rand(P, N, 2, generator=g) * 40
    boxes = torch.cat([c - wh / 2, c + wh / 2], -1)
    counts = torch.tensor([N, max(1, N - 77), 64, 0])
    kc, nc = V.batched_nms_sorted(boxes, counts, 0.7, max_out)
    old = _lib._fn("mx_nms_par")(-1)
    try:
        for par in (1, 0):
            _lib._fn("mx_nms_par")(par)
            kg, ng = V.batched_nms_sorted(boxes.cuda(), counts.cuda(), 0.7, max_out)
            assert ng.cpu().tolist() == nc.tolist(), par
            assert torch.equal(kg.cpu(), kc), par
    finally:
        _lib._fn("mx_nms_par")(old)
