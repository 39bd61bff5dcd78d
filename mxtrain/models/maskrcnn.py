"""Mask R-CNN, ResNet-50-FPN (tensorpack `ResNetFPNModel` with MODE_MASK=True MODE_FPN=True,
as the reference's MPIJob examples train it: examples/maskrcnn/train-maskrcnn-tensorpack.yaml,
SURVEY §2.11, §3.3).

MI355X-first data flow -- every per-step shape is static, so the whole step runs without
host synchronisation and can be replayed as a graph:

  images [B, 3, H, W] -> NHWC bf16 -> ResNet-50 (FrozenBN folded into convs, MIOpen NHWC)
  -> FPN P2..P6 -> RPN head (shared 3x3 conv)
  -> anchor targets: fused IoU/argmax/low-quality matching kernel (K15), sampling by
     random-key ranks (no nonzero()/host sync)
  -> proposals: per-(image, level) top-k, fused decode+clip kernel, one batched bitmask
     NMS launch over all B x 5 problems (K14)
  -> RoI sampling (fixed 512/img, fg first) -> multi-level RoIAlign 7x7 (K13, NHWC)
  -> 2FC box head; mask branch on the 128 fg slots/img: RoIAlign 14x14 -> 4 conv ->
     deconv -> per-class 28x28 logits; targets cropped from the instance masks in place
     by a kernel (no per-RoI mask copies).

Losses follow tensorpack: RPN BCE + Huber(1/9), Fast R-CNN CE + Huber(1) on class-specific
deltas (weights 10,10,5,5), mask sigmoid BCE.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.epilogue import (BlockLink, JoinLink, _conv_in_ok, conv_bias_act, conv_transpose_bias_act, fused_conv_ok,
                            subsample2)
from ..ops import detloss as D
from ..ops import vision as V
from ..ops import _lib
from ..ops import convwg
from ..ops import stem as stem_ops
from .compute_weights import ComputeWeights, cw
from .resnet import ConvNorm, resnet50


@dataclass
class MaskRCNNConfig:
    num_classes: int = 81                      # 80 COCO classes + background
    fpn_channels: int = 256
    anchor_sizes: Tuple[int, ...] = (32, 64, 128, 256, 512)
    anchor_ratios: Tuple[float, ...] = (0.5, 1.0, 2.0)
    anchor_strides: Tuple[int, ...] = (4, 8, 16, 32, 64)
    rpn_fg_thresh: float = 0.7
    rpn_bg_thresh: float = 0.3
    rpn_batch_per_im: int = 256
    rpn_fg_ratio: float = 0.5
    rpn_nms_thresh: float = 0.7
    train_per_level_topk: int = 2000
    train_post_nms_topk: int = 2000
    test_per_level_topk: int = 1000
    test_post_nms_topk: int = 1000
    frcnn_batch_per_im: int = 512
    frcnn_fg_ratio: float = 0.25
    frcnn_fg_thresh: float = 0.5
    bbox_reg_weights: Tuple[float, ...] = (10.0, 10.0, 5.0, 5.0)
    fc_dim: int = 1024
    mask: bool = True
    mask_size: int = 28
    mask_head_dim: int = 256
    result_score_thresh: float = 0.05
    test_nms_thresh: float = 0.5
    results_per_im: int = 100
    pixel_mean: Tuple[float, ...] = (123.675, 116.28, 103.53)
    pixel_std: Tuple[float, ...] = (58.395, 57.12, 57.375)


# ---------------------------------------------------------------------------- anchors
def level_anchors(stride: int, size: int, ratios, H: int, W: int, device) -> torch.Tensor:
    """[H*W*len(ratios), 4] anchors centred on stride-grid cells (tensorpack layout:
    cell-major, ratio-minor)."""
    base = []
    for r in ratios:
        w = size / math.sqrt(r)
        h = size * math.sqrt(r)
        base.append([-w / 2, -h / 2, w / 2, h / 2])
    base = torch.tensor(base, dtype=torch.float32, device=device)
    ys = (torch.arange(H, device=device, dtype=torch.float32) + 0.5) * stride
    xs = (torch.arange(W, device=device, dtype=torch.float32) + 0.5) * stride
    cy, cx = torch.meshgrid(ys, xs, indexing="ij")
    ctr = torch.stack([cx, cy, cx, cy], -1).reshape(-1, 1, 4)
    return (ctr + base[None]).reshape(-1, 4)


def _rank_select(key: torch.Tensor, want: torch.Tensor, eligible: torch.Tensor, max_want: int) -> torch.Tensor:
    """Per row: choose up to want[row] (<= max_want) random eligible entries (key = random
    uniform in [0, 1)); no host sync.

    The max_want smallest keys of a row (ineligible entries keyed 2.0) come from a bounded
    top-k (radix select + in-place sort of max_want values): unlike a full argsort of a
    ~270k-anchor row, which goes to a segmented device radix sort, it is safe inside a
    captured hipGraph step (workloads/maskrcnn/graphed.py)."""
    k = torch.where(eligible, key, torch.full_like(key, 2.0))
    m = min(max_want, k.shape[-1])
    kv, idx = V.topk_rows(k, m, largest=False)                     # ascending: position = rank
    take = (kv < 2.0) & (torch.arange(m, device=key.device)[None] < want[:, None])
    out = torch.zeros_like(eligible)
    out.scatter_(-1, idx, take)
    return out


def huber(x: torch.Tensor, delta: float) -> torch.Tensor:
    a = x.abs()
    return torch.where(a < delta, 0.5 * x * x, delta * (a - 0.5 * delta))


# ---------------------------------------------------------------------------- modules
class FPN(nn.Module):
    join_backward = True   # JoinLink fusion of the top-down join gradients (A/B switch)
    fast_p6 = True         # P6 subsample on csrc/epilogue.hip mx_subsample2 (A/B switch)

    def __init__(self, in_channels: Sequence[int], out: int = 256):
        super().__init__()
        self.lateral = nn.ModuleList([nn.Conv2d(c, out, 1) for c in in_channels])
        self.output = nn.ModuleList([nn.Conv2d(out, out, 3, padding=1) for _ in in_channels])
        for m in list(self.lateral) + list(self.output):
            nn.init.kaiming_uniform_(m.weight, a=1)
            nn.init.zeros_(m.bias)

    def forward(self, feats: List[torch.Tensor]) -> List[torch.Tensor]:
        dt = feats[0].dtype
        # top-down: lateral_i(C_i) + up2(merged_{i+1}); the join is the lateral conv's
        # residual, read nearest-upsampled by its epilogue (no upsampled tensor, no add pass)
        L = len(feats)
        lat = [None] * L
        m = self.lateral[L - 1]
        lat[L - 1] = conv_bias_act(feats[L - 1], cw(m.weight, dt), cw(m.bias, dt))
        # backward: level i's two gradients (output conv, next lateral's residual) summed inside
        # the kernels (ops/epilogue.py JoinLink) when both convs run the fused path
        link = JoinLink() if (torch.is_grad_enabled() and self.join_backward) else None
        joined = set()
        for i in range(L - 2, -1, -1):
            m = self.lateral[i]
            wl, bl, wo, bo = cw(m.weight, dt), cw(m.bias, dt), cw(self.output[i + 1].weight, dt), cw(self.output[i + 1].bias, dt)
            fuse = None
            if (link is not None and _conv_in_ok(feats[i], wl, bl, lat[i + 1])
                    and convwg.fwd_supported(feats[i], wl, bl, lat[i + 1], 1, 0, 1, res_up=True)
                    and fused_conv_ok(lat[i + 1], wo, bo, None, 1, 1, 1)):
                fuse = (link, i + 1, ("join_res",))
                joined.add(i + 1)
            lat[i] = conv_bias_act(feats[i], wl, bl, residual=lat[i + 1], res_up=True, fuse=fuse)
        outs = [conv_bias_act(x, cw(m.weight, dt), cw(m.bias, dt), padding=1,
                              fuse=(link, i, ("join_dx",)) if i in joined else None)
                for i, (x, m) in enumerate(zip(lat, self.output))]
        # P6 = max_pool2d(P5, 1, 2)
        outs.append(subsample2(outs[-1]) if self.fast_p6 else F.max_pool2d(outs[-1], 1, 2))
        return outs


class RPNHead(nn.Module):
    def __init__(self, c: int, na: int):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, padding=1)
        self.cls = nn.Conv2d(c, na, 1)
        self.box = nn.Conv2d(c, 4 * na, 1)
        for m in (self.conv, self.cls, self.box):
            nn.init.normal_(m.weight, std=0.01)
            nn.init.zeros_(m.bias)

    def forward(self, x):
        dt = x.dtype
        t = conv_bias_act(x, cw(self.conv.weight, dt), cw(self.conv.bias, dt), padding=1, relu=True)
        lg = conv_bias_act(t, cw(self.cls.weight, dt), cw(self.cls.bias, dt))
        bx = conv_bias_act(t, cw(self.box.weight, dt), cw(self.box.bias, dt))
        B = x.shape[0]
        # NHWC flatten -> [B, H*W*A] / [B, H*W*A, 4] (cell-major, anchor-minor)
        return lg.permute(0, 2, 3, 1).reshape(B, -1), bx.permute(0, 2, 3, 1).reshape(B, -1, 4)

    def forward_levels(self, P: List[torch.Tensor]):
        """The shared head over all FPN levels as ONE 3x3 conv and ONE 1x1 conv (cls and box
        weights stacked, padded to 8 output channels) on a canvas holding every level
        (``level_canvas``): 2 launches per direction instead of 15, and no gradient
        accumulation of the shared weights across levels.  Same math as ``forward`` per
        level: the levels sit 1 zero row / column apart, so the 3x3 window of a level
        pixel sees exactly its level's zero-padded neighbourhood; canvas pixels outside
        the levels get no gradient.  Returns ([B, H*W*A] logits, [B, H*W*A, 4] deltas)
        per level."""
        lay = level_canvas([(p.shape[2], p.shape[3]) for p in P])
        if lay is None or not self.pack_levels:
            return [self(p) for p in P]
        dt = P[0].dtype
        na = self.cls.weight.shape[0]
        x = _PackLevels.apply(lay, *P)
        # the 3x3 conv's ReLU mask is applied by the 1x1's input-gradient store (BlockLink
        # "mask_in"), so its backward has no mask pass (only the bias-gradient column sums)
        link = BlockLink() if (self.fold_relu and torch.is_grad_enabled()) else None
        t = conv_bias_act(x, cw(self.conv.weight, dt), cw(self.conv.bias, dt), padding=1, relu=True,
                          fuse=(link, 0, ()) if link is not None else None)
        pad = (-5 * na) % 8
        w = torch.cat([cw(self.cls.weight, dt), cw(self.box.weight, dt)]
                      + ([cw(self.cls.weight, dt).new_zeros(pad, *self.cls.weight.shape[1:])] if pad else []))
        b = torch.cat([cw(self.cls.bias, dt), cw(self.box.bias, dt)]
                      + ([cw(self.cls.bias, dt).new_zeros(pad)] if pad else []))
        w = w.contiguous(memory_format=torch.channels_last)
        fuse_o = None
        if link is not None and fused_conv_ok(t, w, b):
            link.premask[0] = True
            fuse_o = (link, 1, ("mask_in",))
        o = conv_bias_act(t, w, b, fuse=fuse_o)
        geo = [(y0, x0, p.shape[2], p.shape[3]) for (y0, x0), p in zip(lay[2], P)]
        if (o.is_cuda and o.dtype == torch.bfloat16 and o.is_contiguous(memory_format=torch.channels_last)
                and _lib.use_hip(o) and len(geo) <= 8):
            # flat [B, A] / [B, A, 4] of all levels in one launch; the per-level pairs are views
            geo5, off = [], 0
            for y0, x0, h, w in geo:
                geo5 += [y0, x0, h, w, off]
                off += h * w * na
            lg, dl = _UnpackFlat.apply(o, tuple(geo5), na, off)
            self.last_flat = (lg, dl)
            out, off = [], 0
            for _, _, h, w in geo:
                n = h * w * na
                out.append((lg[:, off:off + n], dl[:, off:off + n]))
                off += n
            return out
        flat = _UnpackLevels.apply(o, geo, na)
        self.last_flat = None
        return [(flat[2 * i], flat[2 * i + 1]) for i in range(len(P))]

    pack_levels = True
    fold_relu = True   # A/B switch for the ReLU fold above


def level_canvas(shapes):
    """Layout of FPN levels on one canvas: level 0 at the origin, the others left to right
    on a shelf below it, one zero row / column between neighbours.  Returns (Hc, Wc,
    [(y0, x0)] per level), or None when the shelf does not fit under level 0."""
    (h0, w0), rest = shapes[0], shapes[1:]
    if not rest:
        return None
    x, offs = 0, [(0, 0)]
    for h, w in rest:
        offs.append((h0 + 1, x))
        x += w + 1
    if x - 1 > w0:
        return None
    return h0 + 1 + max(h for h, _ in rest), w0, offs


class _PackLevels(torch.autograd.Function):
    """[B, C, Hc, Wc] canvas (channels_last, zero outside the levels) of the FPN levels;
    backward hands each level its slice of the canvas gradient (views, no copies)."""

    @staticmethod
    def forward(ctx, lay, *levels):
        Hc, Wc, offs = lay
        p0 = levels[0]
        B, C = p0.shape[0], p0.shape[1]
        c = torch.empty(B, C, Hc, Wc, dtype=p0.dtype, device=p0.device, memory_format=torch.channels_last)
        if (all(p.is_cuda and p.dtype == torch.bfloat16 and p.is_contiguous(memory_format=torch.channels_last)
                and p.data_ptr() % 16 == 0 for p in levels) and C % 8 == 0 and len(levels) <= 8
                and _lib.use_hip(p0)):
            # every canvas pixel written once: the levels copied, the gaps zeroed
            # (csrc/dettarget.hip rpn_pack_kernel)
            geo = []
            for (y0, x0), p in zip(offs, levels):
                geo += [y0, x0, p.shape[2], p.shape[3], 0]
            srcs = (ctypes.c_void_p * len(levels))(*[p.data_ptr() for p in levels])
            _lib.call("mx_rpn_pack", c.data_ptr(), srcs, (ctypes.c_int * len(geo))(*geo), len(levels), B, Hc, Wc, C,
                      _lib.stream())
        else:
            c.zero_()
            for (y0, x0), p in zip(offs, levels):
                c[:, :, y0:y0 + p.shape[2], x0:x0 + p.shape[3]].copy_(p)
        ctx.geo = [(y0, x0, p.shape[2], p.shape[3]) for (y0, x0), p in zip(offs, levels)]
        return c

    @staticmethod
    def backward(ctx, g):
        return (None,) + tuple(g[:, :, y0:y0 + h, x0:x0 + w] for y0, x0, h, w in ctx.geo)


class _UnpackLevels(torch.autograd.Function):
    """Per level ([B, h*w*A] logits, [B, h*w*A, 4] deltas) out of the head's canvas output
    [B, 5A(+pad), Hc, Wc]; backward writes every level's gradients into ONE zeroed canvas
    gradient (instead of a full-size zero tensor per slice)."""

    @staticmethod
    def forward(ctx, o, geo, na):
        ctx.geo, ctx.na, ctx.shape = geo, na, o.shape
        B = o.shape[0]
        out = []
        for y0, x0, h, w in geo:
            v = o[:, :, y0:y0 + h, x0:x0 + w].permute(0, 2, 3, 1)          # [B, h, w, 5A(+pad)]
            out += [v[..., :na].reshape(B, -1), v[..., na:5 * na].reshape(B, -1, 4)]
        return tuple(out)

    @staticmethod
    def backward(ctx, *gs):
        B, C, Hc, Wc = ctx.shape
        na = ctx.na
        ref = next(g for g in gs if g is not None)
        d = torch.zeros(B, Hc, Wc, C, dtype=ref.dtype, device=ref.device)     # NHWC memory
        for i, (y0, x0, h, w) in enumerate(ctx.geo):
            gl, gb = gs[2 * i], gs[2 * i + 1]
            if gl is not None:
                d[:, y0:y0 + h, x0:x0 + w, :na].copy_(gl.reshape(B, h, w, na))
            if gb is not None:
                d[:, y0:y0 + h, x0:x0 + w, na:5 * na].copy_(gb.reshape(B, h, w, 4 * na))
        return d.permute(0, 3, 1, 2), None, None


class _UnpackFlat(torch.autograd.Function):
    """The head's canvas output [B, C, Hc, Wc] (channels_last bf16) -> flat per-image anchor
    order of ALL levels: logits [B, A], deltas [B, A, 4] (level l at anchor offset off_l) in
    one launch (csrc/dettarget.hip rpn_unpack_kernel); backward builds the whole canvas
    gradient in one launch too.  The loss takes the flat tensors as they are and the
    proposal top-k per-level views of them: no per-level copies, no concatenation."""

    @staticmethod
    def forward(ctx, o, geo5, na, A):
        B, C, Hc, Wc = o.shape
        lg = torch.empty(B, A, dtype=o.dtype, device=o.device)
        dl = torch.empty(B, A, 4, dtype=o.dtype, device=o.device)
        arr = (ctypes.c_int * len(geo5))(*geo5)
        _lib.call("mx_rpn_unpack", o.data_ptr(), B, Hc, Wc, C, na, arr, len(geo5) // 5, A, lg.data_ptr(), dl.data_ptr(),
                  _lib.stream())
        ctx.geo5, ctx.na, ctx.A, ctx.shape = geo5, na, A, o.shape
        return lg, dl

    @staticmethod
    def backward(ctx, glg, gdl):
        B, C, Hc, Wc = ctx.shape
        ref = glg if glg is not None else gdl
        glg = glg.contiguous() if glg is not None else None
        gdl = gdl.contiguous() if gdl is not None else None
        d = torch.empty(B, Hc, Wc, C, dtype=ref.dtype, device=ref.device)
        arr = (ctypes.c_int * len(ctx.geo5))(*ctx.geo5)
        _lib.call("mx_rpn_pack_grad", _lib.ptr(glg), _lib.ptr(gdl), B, Hc, Wc, C, ctx.na, arr, len(ctx.geo5) // 5,
                  ctx.A, d.data_ptr(), _lib.stream())
        return d.permute(0, 3, 1, 2), None, None, None


class _FanOut3(torch.autograd.Function):
    """An FPN level (NCHW view of channels_last bf16) handed to its three consumers -- the
    RPN canvas, the box RoIAlign and the mask RoIAlign -- as three aliases, so backward gets
    their gradients separately and sums them in ONE pass (csrc/dettarget.hip add3_nhwc,
    the canvas slice read through its pitch) instead of autograd's two adds."""

    @staticmethod
    def forward(ctx, p):
        ctx.set_materialize_grads(False)
        ctx.shape = p.shape
        return p.view_as(p), p.view_as(p), p.view_as(p)

    @staticmethod
    def backward(ctx, ga, gb, gc):
        B, C, H, W = ctx.shape
        ref = next((g for g in (ga, gb, gc) if g is not None), None)
        if ref is None:
            return None
        cl = torch.channels_last
        a = ga
        if a is not None and not (a.stride(1) == 1 and a.stride(3) == C and a.data_ptr() % 16 == 0):
            a = a.contiguous(memory_format=cl)
        b = gb.contiguous(memory_format=cl) if gb is not None else None
        c = gc.contiguous(memory_format=cl) if gc is not None else None
        # (.contiguous returns an already-contiguous view as is, whatever its storage offset:
        # the kernel's 16-B vector loads need aligned b / c as well)
        if b is not None and b.data_ptr() % 16:
            b = b.clone(memory_format=cl)
        if c is not None and c.data_ptr() % 16:
            c = c.clone(memory_format=cl)
        out = torch.empty(B, H, W, C, dtype=ref.dtype, device=ref.device)
        _lib.call("mx_add3_nhwc", out.data_ptr(), _lib.ptr(a), a.stride(0) if a is not None else 0,
                  a.stride(2) if a is not None else 0, _lib.ptr(b), _lib.ptr(c), B, H, W, C, _lib.stream())
        return out.permute(0, 3, 1, 2)


def _fanout_ok(p: torch.Tensor) -> bool:
    return (p.is_cuda and p.dtype == torch.bfloat16 and p.is_contiguous(memory_format=torch.channels_last)
            and p.shape[1] % 8 == 0 and p.data_ptr() % 16 == 0 and _lib.use_hip(p))


class BoxHead(nn.Module):
    def __init__(self, c: int, fc: int, ncls: int):
        super().__init__()
        self.fc1 = nn.Linear(c * 49, fc)
        self.fc2 = nn.Linear(fc, fc)
        self.cls = nn.Linear(fc, ncls)
        self.box = nn.Linear(fc, ncls * 4)
        for m in (self.fc1, self.fc2):
            # tensorpack variance_scaling (fan_in, scale 1): std = 1 / sqrt(fan_in)
            nn.init.normal_(m.weight, std=1.0 / math.sqrt(m.weight.shape[1]))
            nn.init.zeros_(m.bias)
        nn.init.normal_(self.cls.weight, std=0.01)
        nn.init.normal_(self.box.weight, std=0.001)
        nn.init.zeros_(self.cls.bias)
        nn.init.zeros_(self.box.bias)

    def forward(self, x):
        dt = x.dtype
        x = x.reshape(x.shape[0], -1)
        x = F.relu(F.linear(x, cw(self.fc1.weight, dt), cw(self.fc1.bias, dt)), inplace=True)
        x = F.relu(F.linear(x, cw(self.fc2.weight, dt), cw(self.fc2.bias, dt)), inplace=True)
        # compute-dtype logits [R, C] and deltas [R, C * 4] (the fused losses read bf16)
        return (F.linear(x, cw(self.cls.weight, dt), cw(self.cls.bias, dt)),
                F.linear(x, cw(self.box.weight, dt), cw(self.box.bias, dt)))


class MaskHead(nn.Module):
    def __init__(self, c: int, dim: int, ncls: int):
        super().__init__()
        self.convs = nn.ModuleList([nn.Conv2d(c if i == 0 else dim, dim, 3, padding=1) for i in range(4)])
        self.deconv = nn.ConvTranspose2d(dim, dim, 2, stride=2)
        self.pred = nn.Conv2d(dim, ncls, 1)
        for m in list(self.convs) + [self.deconv]:
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            nn.init.zeros_(m.bias)
        nn.init.normal_(self.pred.weight, std=0.001)
        nn.init.zeros_(self.pred.bias)

    fuse_backward = True

    def forward(self, x):            # x: [R, 14, 14, C] NHWC -> [R, ncls, 28, 28]
        dt = x.dtype
        x = x.permute(0, 3, 1, 2)    # NCHW view of NHWC memory (channels_last)
        # backward fusion along the conv chain (ops/epilogue.py BlockLink): conv i+1's dgrad
        # store applies conv i's ReLU, so conv i skips its mask pass
        link = BlockLink() if self.fuse_backward else None
        for i, m in enumerate(self.convs):
            w, b = cw(m.weight, dt), cw(m.bias, dt)
            roles = ()
            if link is not None and i > 0 and fused_conv_ok(x, w, b, None, 1, 1, 1):
                link.premask[i] = True
                roles = ("mask_in",)
            x = conv_bias_act(x, w, b, padding=1, relu=True, fuse=(link, i + 1, roles) if link else None)
        x = conv_transpose_bias_act(x, cw(self.deconv.weight, dt), cw(self.deconv.bias, dt), stride=2, relu=True)
        return conv_bias_act(x, cw(self.pred.weight, dt), cw(self.pred.bias, dt))


# ---------------------------------------------------------------------------- model
class MaskRCNN(nn.Module):
    def __init__(self, cfg: Optional[MaskRCNNConfig] = None):
        super().__init__()
        self.cfg = cfg = cfg or MaskRCNNConfig()
        self.backbone = resnet50(norm="frozen")
        self.fpn = FPN(self.backbone.out_channels, cfg.fpn_channels)
        self.rpn = RPNHead(cfg.fpn_channels, len(cfg.anchor_ratios))
        self.box_head = BoxHead(cfg.fpn_channels, cfg.fc_dim, cfg.num_classes)
        self.mask_head = MaskHead(cfg.fpn_channels, cfg.mask_head_dim, cfg.num_classes - 1) if cfg.mask else None
        self.register_buffer("pixel_mean", torch.tensor(cfg.pixel_mean).view(1, 3, 1, 1), persistent=False)
        self.register_buffer("pixel_std", torch.tensor(cfg.pixel_std).view(1, 3, 1, 1), persistent=False)
        self._anchor_cache: Dict = {}

    # ------------------------------------------------------------------ helpers
    def compute_dtype(self, device):
        return torch.bfloat16 if device.type == "cuda" else torch.float32

    def anchors(self, shapes, device):
        key = (tuple(shapes), str(device))
        if key not in self._anchor_cache:
            cfg = self.cfg
            lv = [level_anchors(s, z, cfg.anchor_ratios, h, w, device)
                  for (h, w), s, z in zip(shapes, cfg.anchor_strides, cfg.anchor_sizes)]
            self._anchor_cache[key] = lv
        return self._anchor_cache[key]

    def _all_anchors(self, anchors_lv):
        """All levels' anchors [A, 4] (concatenated once per level-shape set)."""
        key = ("all", tuple(a.data_ptr() for a in anchors_lv))
        if key not in self._anchor_cache:
            self._anchor_cache[key] = torch.cat(anchors_lv, 0)
        return self._anchor_cache[key]

    # frozen stem + pool0 as one kernel straight from the uint8 image (ops/stem.py); A/B switch
    fused_stem = True

    def features(self, images: torch.Tensor):
        dt = self.compute_dtype(images.device)
        stem = self.backbone.stem
        if (self.fused_stem and images.is_cuda and images.dtype == torch.uint8 and dt == torch.bfloat16
                and stem.norm_kind == "frozen" and not stem.conv.weight.requires_grad and not ConvNorm.calibrating
                and _lib.use_hip(images)):
            wf, bf = stem._folded(stem.conv.weight, dt)
            if stem_ops.supported(images, wf, bf):
                x = stem_ops.stem_pool(images, wf, bf, self.cfg.pixel_mean, self.cfg.pixel_std)
                return self.fpn(self.backbone.forward_features(x, stem_done=True))
        x = None
        if (images.is_cuda and images.dtype == torch.uint8 and dt == torch.bfloat16 and images.is_contiguous()
                and (images.shape[2] * images.shape[3]) % 4 == 0 and _lib.use_hip(images)):
            # one pass: uint8 NCHW -> normalised bf16 NHWC (csrc/vision.hip normalize_u8_nhwc_kernel)
            B, _, H, W = images.shape
            x = torch.empty(B, H, W, 3, dtype=dt, device=images.device).permute(0, 3, 1, 2)
            _lib.call("mx_normalize_u8_nhwc", images.data_ptr(), x.data_ptr(), B, H, W,
                      ctypes.cast((ctypes.c_float * 3)(*self.cfg.pixel_mean), ctypes.c_void_p),
                      ctypes.cast((ctypes.c_float * 3)(*[1.0 / v for v in self.cfg.pixel_std]), ctypes.c_void_p),
                      _lib.stream())
        if x is None:
            x = ((images.float() - self.pixel_mean) / self.pixel_std).to(dt)
            x = x.contiguous(memory_format=torch.channels_last)
        c = self.backbone.forward_features(x)
        return self.fpn(c)      # P2..P6, NCHW views of channels_last memory

    @staticmethod
    def _nhwc(p: torch.Tensor) -> torch.Tensor:
        # channels_last memory viewed as [B, H, W, C] without a copy
        return p.permute(0, 2, 3, 1).contiguous()

    # ------------------------------------------------------------------ RPN
    def rpn_targets(self, anchors: torch.Tensor, gt_boxes, gt_count, img_hw):
        """(sel_pos, sel_neg [B, A] bool, encoded regression targets [B, A, 4] fp32) -- the
        PyTorch definition; the GPU path is _rpn_targets_fused (same draws, same math)."""
        cfg = self.cfg
        B = gt_boxes.shape[0]
        mi, am, lq = V.match_boxes(anchors, gt_boxes, gt_count)
        inside = ((anchors[None, :, 0] >= 0) & (anchors[None, :, 1] >= 0) &
                  (anchors[None, :, 2] <= img_hw[:, 1:2]) & (anchors[None, :, 3] <= img_hw[:, 0:1]))
        pos = ((mi >= cfg.rpn_fg_thresh) | (lq >= 0)) & inside
        neg = (mi < cfg.rpn_bg_thresh) & ~pos & inside
        g = torch.rand(mi.shape, device=mi.device)
        nfg_max = int(cfg.rpn_batch_per_im * cfg.rpn_fg_ratio)
        sel_pos = _rank_select(g, torch.full((B,), nfg_max, device=mi.device), pos, nfg_max)
        npos = sel_pos.sum(1)
        sel_neg = _rank_select(g, cfg.rpn_batch_per_im - npos, neg, cfg.rpn_batch_per_im)
        matched = torch.where(lq >= 0, lq, am).clamp(min=0)
        tgt_boxes = torch.gather(gt_boxes, 1, matched[..., None].expand(-1, -1, 4))
        enc = V.encode_boxes(anchors[None].expand(B, -1, -1).reshape(-1, 4), tgt_boxes.reshape(-1, 4)).view(B, -1, 4)
        return sel_pos, sel_neg, enc

    def _rpn_targets_fused(self, anchors, gt_boxes, gt_count, img_hw):
        """rpn_targets in 8 launches (csrc/dettarget.hip): match, the random keys, one
        labelling pass (inside / pos / neg keys + regression targets), two bounded top-k
        selections and the selection scatter -- instead of ~40 PyTorch kernels."""
        cfg = self.cfg
        B, G = gt_boxes.shape[:2]
        A = anchors.shape[0]
        dev = anchors.device
        gtf = gt_boxes.float().contiguous()
        mi, am, lq = V.match_boxes(anchors, gtf, gt_count, int32=True)
        g = torch.rand((B, A), device=dev)
        keys = torch.empty(2 * B, A, dtype=torch.float32, device=dev)   # positive rows, then negative rows
        kpos, kneg = keys[:B], keys[B:]
        enc = torch.empty(B, A, 4, dtype=torch.float32, device=dev)
        sel_pos = torch.empty(B, A, dtype=torch.bool, device=dev)
        sel_neg = torch.empty_like(sel_pos)
        an = anchors.float().contiguous()
        hw = img_hw.float().contiguous()
        _lib.call("mx_rpn_keys", _lib.ptr(an), A, B, _lib.ptr(mi), _lib.ptr(am), _lib.ptr(lq), _lib.ptr(hw),
                  _lib.ptr(g), _lib.ptr(gtf), G, float(cfg.rpn_fg_thresh), float(cfg.rpn_bg_thresh), _lib.ptr(kpos),
                  _lib.ptr(kneg), _lib.ptr(enc), _lib.ptr(sel_pos), _lib.ptr(sel_neg), _lib.stream())
        nfg_max = min(int(cfg.rpn_batch_per_im * cfg.rpn_fg_ratio), A)
        nb = min(cfg.rpn_batch_per_im, A)
        # both selections in one (two-launch) long-row top-k: the nfg_max smallest positive
        # keys are the first nfg_max of that row's nb smallest (sorted, ties by index)
        kk = max(nfg_max, nb)
        v2, i2 = V.topk_rows(keys, kk, largest=False)
        _lib.call("mx_rpn_select", _lib.ptr(v2), _lib.ptr(i2), nfg_max, _lib.ptr(v2[B:]), _lib.ptr(i2[B:]), nb, kk,
                  int(cfg.rpn_batch_per_im), A, B, _lib.ptr(sel_pos), _lib.ptr(sel_neg), _lib.stream())
        return sel_pos, sel_neg, enc

    def _fused_targets_ok(self, t: torch.Tensor) -> bool:
        return self.fused_targets and _lib.use_hip(t)

    fused_targets = True

    def rpn_losses(self, logits, deltas, anchors, gt_boxes, gt_count, img_hw):
        cfg = self.cfg
        B = logits.shape[0]
        if self._fused_targets_ok(logits) and gt_boxes.shape[1] > 0:
            sel_pos, sel_neg, enc = self._rpn_targets_fused(anchors, gt_boxes, gt_count, img_hw)
        else:
            sel_pos, sel_neg, enc = self.rpn_targets(anchors, gt_boxes, gt_count, img_hw)
        # BCE over the sampled anchors / #sampled, huber(1/9) over the positives / (B * 256)
        return D.rpn_loss(logits, deltas, enc, sel_pos, sel_neg, B * cfg.rpn_batch_per_im)

    @torch.no_grad()
    def proposals(self, logits_lv, deltas_lv, anchors_lv, img_hw, training: bool):
        """Per image top proposals [B, K, 4] (+ scores [B, K]); static K."""
        cfg = self.cfg
        B = logits_lv[0].shape[0]
        pre = cfg.train_per_level_topk if training else cfg.test_per_level_topk
        post = cfg.train_post_nms_topk if training else cfg.test_post_nms_topk
        # per (image, level): top-k logits (sorted) + decoded, clipped boxes, -inf padded
        bxs, scs, counts = V.level_topk_decode(logits_lv, deltas_lv, anchors_lv, img_hw, pre)
        L = len(counts)
        boxes = bxs.reshape(B * L, pre, 4)                                       # problem = (image, level)
        scores = scs.reshape(B * L, pre)
        ck = ("nms_counts", tuple(counts), B, str(boxes.device))
        if ck not in self._anchor_cache:   # (no host->device copy inside a captured step)
            self._anchor_cache[ck] = torch.tensor(counts, dtype=torch.int32, device=boxes.device).repeat(B)
        cnt = self._anchor_cache[ck]
        keep, _ = V.batched_nms_sorted(boxes, cnt, cfg.rpn_nms_thresh, pre, raw=True)
        # each image's top `post` survivors over its levels (every level's list is sorted)
        b, s = V.nms_merge_topk(keep, scores, boxes, B, L, min(post, L * pre))
        return b.detach(), s.detach()

    # ------------------------------------------------------------------ RoI sampling
    @torch.no_grad()
    def sample_rois(self, props, gt_boxes, gt_labels, gt_count):
        """Returns rois [B, N, 4] (fg first), labels [B, N] (0 = bg), matched gt [B, N],
        regression targets [B, N, 4], fg mask [B, N]; N = frcnn_batch_per_im.  The PyTorch
        definition; the GPU path is _sample_rois_fused (same draws, same math)."""
        cfg = self.cfg
        B, G = gt_boxes.shape[:2]
        gvalid = torch.arange(G, device=props.device)[None] < gt_count[:, None]
        gtb = torch.where(gvalid[..., None], gt_boxes, torch.full_like(gt_boxes, -1e4))  # invalid gt -> far away
        cand = torch.cat([props, gtb], 1)                                                  # [B, K+G, 4]
        cvalid = torch.cat([torch.ones(props.shape[:2], dtype=torch.bool, device=props.device), gvalid], 1)
        mi, am, _ = V.match_boxes(cand, gt_boxes, gt_count, low_quality=False)
        fg = (mi >= cfg.frcnn_fg_thresh) & cvalid
        bg = (mi < cfg.frcnn_fg_thresh) & cvalid
        N = cfg.frcnn_batch_per_im
        nfg = int(N * cfg.frcnn_fg_ratio)
        r = torch.rand(mi.shape, device=mi.device)
        sel_fg = _rank_select(r, torch.full((B,), nfg, device=mi.device), fg, nfg)
        key = torch.where(sel_fg, 2.0 + r, torch.where(bg, 1.0 + r, torch.zeros_like(r)))
        _, idx = V.topk_rows(key, N)                                                       # fg first, then bg
        rois = torch.gather(cand, 1, idx[..., None].expand(-1, -1, 4))
        is_fg = torch.gather(sel_fg, 1, idx)
        g = torch.gather(am.clamp(min=0), 1, idx)
        labels = torch.where(is_fg, torch.gather(gt_labels, 1, g), torch.zeros_like(g))
        mgt = torch.gather(gt_boxes, 1, g[..., None].expand(-1, -1, 4))
        tgt = V.encode_boxes(rois.reshape(-1, 4), mgt.reshape(-1, 4), cfg.bbox_reg_weights).view(B, N, 4)
        return rois, labels, g, tgt, is_fg

    @torch.no_grad()
    def _sample_rois_fused(self, props, gt_boxes, gt_labels, gt_count):
        """sample_rois in 8 launches (csrc/dettarget.hip): candidates (proposals + valid gt),
        match, the random keys, fg keys, bounded top-k of the fg, the ordering keys, top-k of
        the N slots and one gather pass (RoI, fg flag, matched gt, label, regression target,
        and the [batch, box] RoIAlign rows of all slots / of the fg slots) -- instead of ~45
        PyTorch kernels.  Returns sample_rois' tuple + (rois5, rois5_fg)."""
        cfg = self.cfg
        B, K = props.shape[:2]
        G = gt_boxes.shape[1]
        C = K + G
        N = cfg.frcnn_batch_per_im
        nfg = int(N * cfg.frcnn_fg_ratio)
        dev = props.device
        gtf = gt_boxes.float().contiguous()
        gc = gt_count.to(torch.int32).contiguous()
        cand = torch.empty(B, C, 4, dtype=torch.float32, device=dev)
        cvalid = torch.empty(B, C, dtype=torch.uint8, device=dev)
        _lib.call("mx_roi_candidates", _lib.ptr(props.float().contiguous()), K, _lib.ptr(gtf), _lib.ptr(gc), G, B,
                  _lib.ptr(cand), _lib.ptr(cvalid), _lib.stream())
        mi, am, _ = V.match_boxes(cand, gtf, gc, low_quality=False, int32=True)
        r = torch.rand((B, C), device=dev)
        fgk = torch.empty(B, C, dtype=torch.float32, device=dev)
        _lib.call("mx_roi_fgkey", _lib.ptr(mi), _lib.ptr(cvalid), _lib.ptr(r), B * C, float(cfg.frcnn_fg_thresh),
                  _lib.ptr(fgk), _lib.stream())
        kf = min(nfg, C)
        vf, i_f = V.topk_rows(fgk, kf, largest=False)
        sel_fg = torch.empty(B, C, dtype=torch.bool, device=dev)
        key = torch.empty(B, C, dtype=torch.float32, device=dev)
        _lib.call("mx_roi_order", _lib.ptr(vf), _lib.ptr(i_f), kf, _lib.ptr(mi), _lib.ptr(cvalid), _lib.ptr(r), C, B,
                  float(cfg.frcnn_fg_thresh), _lib.ptr(sel_fg), _lib.ptr(key), _lib.stream())
        _, idx = V.topk_rows(key, N)
        rois = torch.empty(B, N, 4, dtype=torch.float32, device=dev)
        labels = torch.empty(B, N, dtype=torch.int64, device=dev)
        gidx = torch.empty(B, N, dtype=torch.int64, device=dev)
        tgt = torch.empty(B, N, 4, dtype=torch.float32, device=dev)
        is_fg = torch.empty(B, N, dtype=torch.bool, device=dev)
        rois5 = torch.empty(B * N, 5, dtype=torch.float32, device=dev)
        rois5_fg = torch.empty(B * nfg, 5, dtype=torch.float32, device=dev)
        wx, wy, ww, wh = cfg.bbox_reg_weights
        _lib.call("mx_roi_gather", _lib.ptr(idx), N, nfg, B, _lib.ptr(cand), C, _lib.ptr(sel_fg), _lib.ptr(am),
                  _lib.ptr(gt_labels.long().contiguous()), _lib.ptr(gtf), G, float(wx), float(wy), float(ww), float(wh),
                  _lib.ptr(rois), _lib.ptr(labels), _lib.ptr(gidx), _lib.ptr(tgt), _lib.ptr(is_fg), _lib.ptr(rois5),
                  _lib.ptr(rois5_fg), _lib.stream())
        return rois, labels, gidx, tgt, is_fg, rois5, rois5_fg

    @staticmethod
    def _with_batch(boxes: torch.Tensor) -> torch.Tensor:
        B, N, _ = boxes.shape
        bi = torch.arange(B, device=boxes.device, dtype=torch.float32)[:, None, None].expand(B, N, 1)
        return torch.cat([bi, boxes.float()], -1).reshape(-1, 5)

    # ------------------------------------------------------------------ forward
    def compute_weight_specs(self):
        """[(trainable parameter, fold scale or None)] for the batched bf16 compute
        copies (models/compute_weights.py): folded frozen-BN convs carry their scale."""
        cache = self.__dict__.get("_cw_cache")
        if cache is None:
            convs = [m for m in self.modules() if isinstance(m, ConvNorm)]
            cache = self.__dict__["_cw_cache"] = [convs, list(self.parameters()), None, None]
        convs, params, key, specs = cache
        # the list only changes when frozen statistics are rewritten (calibration,
        # checkpoint load: version bumps) or parameters are (un)frozen
        # (device and storage identity too: .to(device) / load_state_dict(assign=True)
        # replace the buffers with fresh version-0 tensors)
        nkey = (tuple((m.norm.running_var._version + m.norm.running_mean._version + m.norm.weight._version
                       + m.norm.bias._version, m.norm.running_var.data_ptr(), m.norm.running_mean.data_ptr(),
                       m.norm.weight.data_ptr(), m.norm.bias.data_ptr())
                      for m in convs if m.norm_kind == "frozen"),
                tuple((p.requires_grad, p.data_ptr()) for p in params),
                str(params[0].device) if params else "")
        if nkey == key:
            return specs
        specs = []
        folded = set()
        for m in convs:
            sf = m.fold_scale_full()
            if sf is not None:
                specs.append((m.conv.weight, sf))
                folded.add(id(m.conv.weight))
        for p in params:
            if p.requires_grad and id(p) not in folded:
                specs.append((p, None))
        cache[2], cache[3] = nkey, specs
        return specs

    def forward(self, images, img_hw, gt_boxes=None, gt_labels=None, gt_count=None, gt_masks=None,
                gt_mask_table=None):
        if images.device.type != "cuda" or not torch.is_grad_enabled():
            return self._forward(images, img_hw, gt_boxes, gt_labels, gt_count, gt_masks, gt_mask_table)
        fm = self.__dict__.get("_flat_master")
        if fm is not None:   # persistent compute copies kept current by the fused optimizer
            with fm.compute_weights():
                return self._forward(images, img_hw, gt_boxes, gt_labels, gt_count, gt_masks, gt_mask_table)
        # under data parallelism several cast nodes, so gradient buckets become ready in
        # backward order (all-reduce overlapped with backward); one node on a single GPU
        groups = 8 if (torch.distributed.is_available() and torch.distributed.is_initialized()
                       and torch.distributed.get_world_size() > 1) else 1
        with ComputeWeights(self.compute_weight_specs(), self.compute_dtype(images.device), groups=groups):
            return self._forward(images, img_hw, gt_boxes, gt_labels, gt_count, gt_masks, gt_mask_table)

    def _forward(self, images, img_hw, gt_boxes=None, gt_labels=None, gt_count=None, gt_masks=None,
                 gt_mask_table=None):
        """Training: returns dict of losses.  images [B,3,H,W] (padded), img_hw [B,2] real
        sizes, gt_* padded to G per image; gt_masks uint8 [B, G, H, W], or (with
        gt_mask_table int32 [B, G, 5]) the flat uint8 buffer of packed instance crops."""
        cfg = self.cfg
        P = self.features(images)
        # training: the RoIAlign levels reach the FPN through _FanOut3 (one fused gradient sum
        # per level for the canvas / box / mask consumers)
        fan = (self.training and self.fused_targets and torch.is_grad_enabled()
               and all(_fanout_ok(p) for p in P[:4]))
        if fan:
            f3 = [_FanOut3.apply(p) for p in P[:4]]
            P_rpn = [f[0] for f in f3] + list(P[4:])
            P_box = [f[1] for f in f3]
            P_mask = [f[2] for f in f3]
        else:
            P_rpn = P_box = P_mask = P
        lv = self.rpn.forward_levels(P_rpn)
        logits_lv = [l for l, _ in lv]
        deltas_lv = [d for _, d in lv]
        anchors_lv = self.anchors([(p.shape[2], p.shape[3]) for p in P], images.device)
        img_hw = img_hw.float()
        if not self.training:
            return self.inference(P, logits_lv, deltas_lv, anchors_lv, img_hw)
        anchors = self._all_anchors(anchors_lv)
        flat = getattr(self.rpn, "last_flat", None)
        self.rpn.last_flat = None
        lg_all, dl_all = flat if flat is not None else (torch.cat(logits_lv, 1), torch.cat(deltas_lv, 1))
        rpn_cls, rpn_box = self.rpn_losses(lg_all, dl_all, anchors, gt_boxes, gt_count, img_hw)
        props, _ = self.proposals(logits_lv, deltas_lv, anchors_lv, img_hw, True)
        rois5 = rois5_fg = None
        if self._fused_targets_ok(props) and gt_boxes.shape[1] > 0:
            rois, labels, gidx, tgt, is_fg, rois5, rois5_fg = self._sample_rois_fused(props, gt_boxes, gt_labels,
                                                                                       gt_count)
        else:
            rois, labels, gidx, tgt, is_fg = self.sample_rois(props, gt_boxes.float(), gt_labels, gt_count)
        B, N = labels.shape
        feats = [self._nhwc(p) for p in P_box[:4]]
        scales = [1.0 / s for s in cfg.anchor_strides[:4]]
        roi_feat = V.roi_align(feats, rois5 if rois5 is not None else self._with_batch(rois), (7, 7), scales)
        cls_logits, box_deltas = self.box_head(roi_feat)
        lab = labels.reshape(-1)
        # softmax CE (mean) + huber(1) of the labelled class's deltas over the fg RoIs / (B * N)
        cls_loss, box_loss = D.frcnn_loss(cls_logits, box_deltas, lab, tgt.reshape(-1, 4), is_fg.reshape(-1), B * N)
        out = {"rpn_cls_loss": rpn_cls, "rpn_box_loss": rpn_box, "fastrcnn_cls_loss": cls_loss,
               "fastrcnn_box_loss": box_loss}
        if self.mask_head is not None:
            nfg = int(N * cfg.frcnn_fg_ratio)
            fg_rois = rois[:, :nfg]
            fg_valid = is_fg[:, :nfg].float().reshape(-1)   # (one strided cast, then a view)
            fg_lab = labels[:, :nfg].reshape(-1)
            mfeats = [self._nhwc(p) for p in P_mask[:4]]
            mf = V.roi_align(mfeats, rois5_fg if rois5_fg is not None else self._with_batch(fg_rois), (14, 14),
                             scales)
            ml = self.mask_head(mf)                                               # [R, 80, 28, 28]
            G = (gt_mask_table if gt_mask_table is not None else gt_masks).shape[1]
            ck = ("gt_base", B, G, str(images.device))
            if ck not in self._anchor_cache:   # (constant per shape: no arange / mul in the step)
                self._anchor_cache[ck] = torch.arange(B, device=images.device)[:, None] * G
            flat_gid = (self._anchor_cache[ck] + gidx[:, :nfg]).reshape(-1)
            if gt_mask_table is not None:
                tgt_m = V.crop_resize_mask_crops(gt_masks, gt_mask_table.reshape(-1, 5), images.shape[2],
                                                 images.shape[3], fg_rois.reshape(-1, 4), flat_gid, cfg.mask_size)
            else:
                tgt_m = V.crop_resize_masks(gt_masks.reshape(-1, *gt_masks.shape[2:]), fg_rois.reshape(-1, 4),
                                            flat_gid, cfg.mask_size)
            # per-RoI mean BCE of the labelled class's mask vs (target >= 0.5), over valid fg RoIs
            out["maskrcnn_loss"] = D.mask_loss(ml, fg_lab, tgt_m, fg_valid)
        # one stack + one reduction instead of a chain of scalar adds
        out["total_loss"] = torch.stack([v.float() for v in out.values()]).sum()
        return out

    @torch.no_grad()
    def inference(self, P, logits_lv, deltas_lv, anchors_lv, img_hw):
        cfg = self.cfg
        props, _ = self.proposals(logits_lv, deltas_lv, anchors_lv, img_hw, False)
        B, K, _ = props.shape
        feats = [self._nhwc(p) for p in P[:4]]
        scales = [1.0 / s for s in cfg.anchor_strides[:4]]
        roi_feat = V.roi_align(feats, self._with_batch(props), (7, 7), scales)
        cls_logits, box_deltas = self.box_head(roi_feat)
        cls_logits = cls_logits.float()
        box_deltas = box_deltas.float().view(cls_logits.shape[0], -1, 4)
        prob = cls_logits.softmax(-1).view(B, K, -1)[..., 1:]                    # [B, K, C]
        C = prob.shape[-1]
        ref = props.reshape(-1, 1, 4).expand(-1, C, 4).reshape(-1, 4)
        dec = V.decode_boxes(ref, box_deltas[:, 1:].reshape(-1, 4), cfg.bbox_reg_weights, img_hw,
                             rows_per_img=K * C).view(B, K, C, 4)
        # per (image, class) NMS problems, boxes sorted by class score
        sc = prob.permute(0, 2, 1)                                                 # [B, C, K]
        sc = torch.where(sc >= cfg.result_score_thresh, sc, torch.full_like(sc, -1.0))
        s_sorted, order = sc.sort(dim=-1, descending=True)
        bx = dec.permute(0, 2, 1, 3)
        bx = torch.gather(bx, 2, order[..., None].expand(-1, -1, -1, 4))
        cnt = (s_sorted >= 0).sum(-1).to(torch.int32).reshape(-1)
        keep, nk = V.batched_nms_sorted(bx.reshape(B * C, K, 4), cnt, cfg.test_nms_thresh, cfg.results_per_im)
        valid = keep >= 0
        ki = keep.clamp(min=0)
        kb = torch.gather(bx.reshape(B * C, K, 4), 1, ki[..., None].expand(-1, -1, 4)).view(B, C * cfg.results_per_im, 4)
        ks = torch.where(valid, torch.gather(s_sorted.reshape(B * C, K), 1, ki),
                         torch.full_like(ki, -1, dtype=torch.float32)).view(B, -1)
        kl = torch.arange(1, C + 1, device=ks.device)[None, :, None].expand(B, C, cfg.results_per_im).reshape(B, -1)
        s, i = ks.topk(cfg.results_per_im, dim=1)
        boxes = torch.gather(kb, 1, i[..., None].expand(-1, -1, 4))
        labels = torch.gather(kl, 1, i)
        res = {"boxes": boxes, "scores": s, "labels": labels, "valid": s > 0}
        if self.mask_head is not None:
            mf = V.roi_align(feats, self._with_batch(boxes), (14, 14), scales)
            ml = self.mask_head(mf)
            ml = torch.gather(ml, 1, (labels.reshape(-1) - 1).clamp(min=0)[:, None, None, None].expand(
                -1, 1, *ml.shape[2:]))
            res["masks"] = ml.squeeze(1).float().sigmoid().view(B, cfg.results_per_im, cfg.mask_size, cfg.mask_size)
        return res
