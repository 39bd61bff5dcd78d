"""ResNet-50 (torchvision-free) for the Mask R-CNN backbone (FrozenBN) and
the Ray Train ResNet-50 config (BatchNorm, BASELINE config 5).

MI355X layout: activations are channels_last (NHWC) bf16 so MIOpen runs its NHWC
implicit-GEMM (MFMA) convolutions and no layout transposes appear between layers;
parameters stay fp32 masters (cast per forward, AMP style).

``norm="frozen"``  FrozenBatchNorm: a fixed per-channel affine (tensorpack
                   BACKBONE.NORM=FreezeBN); with random-init weights it is the identity
                   transform, applied as conv bias so it costs no extra pass.
``norm="bn"``      trainable BatchNorm2d (ImageNet classification training).
"""
from __future__ import annotations

import contextlib
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import compute_weights as _cw
from ..ops import convwg
from ..ops.batchnorm import bn2_add_relu, bn_act, bn_relu_maxpool
from ..ops.epilogue import BlockLink, ConvBiasActFn, conv_bias_act, fused_conv_ok, global_avg_pool, maxpool3s2


# trainable BN: batch statistics from the producing conv's epilogue (A/B switch, scripts/resnet_ab.py)
BN_EPILOGUE_STATS = True


def _conv_nobias(x, w, stride, padding, dilation, fuse=None, bnpre=None):
    """conv2d without bias for the trainable-BN path: bf16 NHWC activations go through the
    implicit-GEMM kernels where they tile (forward, input and weight gradients), then the
    MIOpen-forward + implicit-GEMM-weight-gradient path, else torch (autocast / fp32).
    ``fuse`` (BlockLink, k, roles): honoured on the first path only; role "take_res" sets
    the link's taker so the block's last BN hands its residual gradient to this conv's dgrad.
    ``bnpre`` (list): on the first path receives the epilogue's BatchNorm statistics of the
    output (ops/batchnorm.py bn_act ``pre``)."""
    if x.is_cuda and x.dtype == torch.bfloat16:
        wb = _cw.cw(w, torch.bfloat16)   # (one-launch compute copies under ResNet.forward)
        if convwg.fwd_supported(x, wb, None, None, stride, padding, dilation):
            if fuse is not None and "take_res" in fuse[2]:
                fuse[0].taker = True
            return ConvBiasActFn.apply(x, wb, None, None, False, stride, padding, dilation, fuse, False, bnpre)
        if convwg.supported(x, wb, stride, padding, dilation):
            return convwg.conv2d_wg(x, wb, stride, padding, dilation)
        return F.conv2d(x, wb, None, stride, padding, dilation)
    return F.conv2d(x, w.to(x.dtype), None, stride, padding, dilation)


class FrozenBN(nn.Module):
    def __init__(self, c: int, eps: float = 1e-5):
        super().__init__()
        self.register_buffer("weight", torch.ones(c))
        self.register_buffer("bias", torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.eps = eps

    def scale_shift(self):
        s = self.weight * torch.rsqrt(self.running_var + self.eps)
        return s, self.bias - self.running_mean * s


class ConvNorm(nn.Module):
    """conv (no bias) + norm (+ ReLU).  FrozenBN is folded into the conv (weight scale +
    bias) at forward time, so the frozen affine never touches activations separately."""

    def __init__(self, cin, cout, k, stride=1, padding=0, norm="frozen", relu=True, dilation=1):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride, padding, dilation=dilation, bias=False)
        nn.init.kaiming_normal_(self.conv.weight, mode="fan_out", nonlinearity="relu")
        self.norm_kind = norm
        self.norm = FrozenBN(cout) if norm == "frozen" else nn.BatchNorm2d(cout)
        self.relu = relu
        self._fold = None   # (key, per-channel scale, folded weight or None, bias) -- see _folded()

    calibrating = False

    def forward(self, x, residual=None, relu=None, fuse=None):
        """act(conv(x) [+ folded FrozenBN] (+ residual)); ``relu`` overrides the module's
        activation (the bottleneck applies its ReLU after the residual add).  ``fuse`` =
        (BlockLink, k, roles): the bottleneck's backward-fusion contract (ops/epilogue.py),
        honoured only when this conv runs the all-implicit-GEMM ConvBiasActFn path."""
        relu = self.relu if relu is None else relu
        dt = x.dtype
        w = self.conv.weight
        if self.norm_kind == "frozen" and ConvNorm.calibrating:
            # data-dependent init of a random backbone: set the frozen statistics so this
            # conv's output is zero-mean / unit-variance per channel (LSUV-style)
            with torch.no_grad():
                y = F.conv2d(x.float(), w.float(), None, self.conv.stride, self.conv.padding, self.conv.dilation)
                self.norm.running_mean.copy_(y.mean(dim=(0, 2, 3)))
                self.norm.running_var.copy_(y.var(dim=(0, 2, 3), unbiased=False) + 1e-5)
                self.norm.weight.fill_(1.0)
                self.norm.bias.zero_()
        if self.norm_kind == "frozen":
            wf, bf = self._folded(w, dt)
            if fuse is not None:
                link, k, roles = fuse
                if fused_conv_ok(x, wf, bf, residual, self.conv.stride, self.conv.padding, self.conv.dilation):
                    if "mask_in" in roles:
                        link.premask[k - 1] = True     # conv k-1 leaves its ReLU mask to this dgrad
                    if "take_res" in roles:
                        link.taker = True
                    if "mask_prev" in roles:
                        link.prev.premask[3] = True    # the previous block's conv3 likewise
                else:
                    fuse = None
            # one MIOpen conv + one fused bias (+ residual) (+ ReLU) pass (ops/epilogue.py)
            return conv_bias_act(x, wf, bf, self.conv.stride, self.conv.padding, self.conv.dilation, relu=relu,
                                 residual=residual, fuse=fuse)
        # trainable BatchNorm: the convolution on csrc/convwg.hip where it tiles (implicit-GEMM
        # forward / input / weight gradients), then ONE fused BN (+ residual) (+ ReLU) node
        # (ops/batchnorm.py, csrc/batchnorm.hip)
        # (identity blocks: conv1 role "take_res" adds the residual gradient that conv3's BN
        # backward stashes, role "stash_res" -- see Bottleneck.forward)
        # (the BN statistics of the conv output come from the conv's epilogue: bnpre)
        link, roles = (fuse[0], fuse[2]) if fuse is not None else (None, ())
        pre = [] if self.norm.training and BN_EPILOGUE_STATS else None
        y = _conv_nobias(x, w, self.conv.stride, self.conv.padding, self.conv.dilation,
                         fuse=fuse if ("take_res" in roles or "stash_dx" in roles) else None, bnpre=pre)
        return bn_act(y, self.norm, residual=residual, relu=relu, link=link if "stash_res" in roles else None,
                      pre=pre[0] if pre else None)

    def conv_pre(self, x, fuse=None):
        """The trainable-BN path's convolution alone: (conv output, its epilogue BN statistics
        or None) -- for a consumer applying this BN itself (ops/batchnorm.py bn2_add_relu)."""
        pre = [] if self.norm.training and BN_EPILOGUE_STATS else None
        y = _conv_nobias(x, self.conv.weight, self.conv.stride, self.conv.padding, self.conv.dilation,
                         fuse=fuse, bnpre=pre)
        return y, (pre[0] if pre else None)

    def fused_ok(self, x) -> bool:
        """This conv (frozen norm) would run ConvBiasActFn on input x, honouring a BlockLink."""
        if self.norm_kind != "frozen" or ConvNorm.calibrating:
            return False
        wf, bf = self._folded(self.conv.weight, x.dtype)
        return fused_conv_ok(x, wf, bf, None, self.conv.stride, self.conv.padding, self.conv.dilation)

    def _folded(self, w: torch.Tensor, dt: torch.dtype):
        """FrozenBN folded into the conv: weight * s (per output channel) and bias
        b - mean * s.  The frozen statistics change only through in-place writes
        (calibration, checkpoint load), which bump the tensors' version counters, so the
        per-channel affine -- and, for a conv whose weight is frozen too (stem and res2,
        FREEZE_AT=2), the folded bf16 weight -- is cached against those versions instead
        of being recomputed with ~8 small kernels per conv on every step."""
        n = self.norm
        frozen_w = not w.requires_grad
        key = (n.weight._version, n.bias._version, n.running_mean._version, n.running_var._version,
               w._version if frozen_w else -1, w.data_ptr() if frozen_w else 0, dt, w.device)
        c = self._fold
        if c is None or c[0] != key:
            with torch.no_grad():
                s, b = n.scale_shift()
                s4 = s[:, None, None, None].contiguous()
                c = self._fold = (key, s4, (w * s4).to(dt) if frozen_w else None, b.to(dt))
        _, s4, wf, bf = c
        if wf is None:
            wf = _cw.cw(w, dt) if _cw.has(w) else (w * s4).to(dt)
        return wf, bf

    def fold_scale_full(self) -> Optional[torch.Tensor]:
        """The FrozenBN scale broadcast to the conv weight's shape (cached against the
        statistics' versions), for the batched compute-weight fold
        (models/compute_weights.py); None unless this is a trainable frozen-BN conv."""
        w = self.conv.weight
        if self.norm_kind != "frozen" or not w.requires_grad:
            return None
        n = self.norm
        key = (n.weight._version, n.bias._version, n.running_mean._version, n.running_var._version, w.device)
        c = getattr(self, "_sfull", None)
        if c is None or c[0] != key:
            with torch.no_grad():
                s, _ = n.scale_shift()
                c = self._sfull = (key, s[:, None, None, None].expand_as(w).contiguous())
        return c[1]


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, norm="frozen", stride_in_1x1=True):
        super().__init__()
        cout = width * 4
        s1, s3 = (stride, 1) if stride_in_1x1 else (1, stride)
        self.conv1 = ConvNorm(cin, width, 1, s1, 0, norm)
        self.conv2 = ConvNorm(width, width, 3, s3, 1, norm)
        self.conv3 = ConvNorm(width, cout, 1, 1, 0, norm, relu=False)
        self.shortcut = ConvNorm(cin, cout, 1, stride, 0, norm, relu=False) if (stride != 1 or cin != cout) else None
        if norm == "bn":
            nn.init.zeros_(self.conv3.norm.weight)   # zero-init last BN gamma (standard ResNet recipe)

    # backward fusion inside the block (ops/epilogue.py BlockLink): the dgrads of conv2 /
    # conv3 apply conv1's / conv2's ReLU in their stores, and an identity block's residual
    # gradient is added in conv1's dgrad store instead of by autograd (FrozenBN path).
    # Across blocks: an identity block's input is the previous block's ReLU output and its
    # conv1 dgrad store already holds that input's whole gradient (dgrad + residual), so it
    # applies the previous block's ReLU too ("mask_prev") and the previous conv3 skips its
    # mask pass.  The link travels on the output tensor (``_mx_link``).
    fuse_backward = True

    # projection blocks: the shortcut conv's input gradient is parked too ("stash_dx") and
    # added in conv1's dgrad store, which then holds the block input's whole gradient and can
    # apply the previous block's ReLU as in an identity block (autograd's add of the two
    # input gradients and the previous conv3's mask pass disappear).  The shortcut's backward
    # always runs before conv1's: both become ready after conv3's, and the engine takes the
    # later-created node (the shortcut) first; conv1 checks it (ops/epilogue.py).
    fuse_projection = True

    def forward(self, x):
        ident = self.shortcut is None
        if self.conv1.norm_kind == "bn":
            # trainable BatchNorm, identity block: the residual's gradient (conv3's BN backward)
            # is added in conv1's dgrad store instead of by a separate autograd add
            if self.fuse_backward and ident and torch.is_grad_enabled():
                link = BlockLink()
                a1 = self.conv1(x, fuse=(link, 1, ("take_res",)))
                a2 = self.conv2(a1)
                return self.conv3(a2, residual=x, relu=True, fuse=(link, 3, ("stash_res",)))
            # projection block: the shortcut conv's input gradient is parked and added in conv1's
            # dgrad store (the same contract as the FrozenBN path below)
            if self.fuse_backward and self.fuse_projection and torch.is_grad_enabled() and self._bn_proj_ok(x):
                link = BlockLink()
                a1 = self.conv1(x, fuse=(link, 1, ("take_res", "take_dx")))
                a2 = self.conv2(a1)
                # (the shortcut conv is created after conv2 and before conv3, so its backward
                # still runs before conv1's: see fuse_projection)
                yd, pd = self.shortcut.conv_pre(x, fuse=(link, 0, ("stash_dx",)))
                y3, p3 = self.conv3.conv_pre(a2)
                # conv3's BN + the shortcut's BN + ReLU as one node (no shortcut BN output tensor)
                return bn2_add_relu(y3, self.conv3.norm, yd, self.shortcut.norm, p3, pd)
            a1 = self.conv1(x)
            a2 = self.conv2(a1)
            idt = x if ident else self.shortcut(x)
            return self.conv3(a2, residual=idt, relu=True)
        link = BlockLink() if self.fuse_backward and self.conv1.norm_kind == "frozen" else None
        proj = link is not None and not ident and self.fuse_projection and self.shortcut.fused_ok(x)
        prev = getattr(x, "_mx_link", None) if (link is not None and (ident or proj)) else None
        r1 = ("take_res", "mask_prev") if prev is not None else (("take_res",) if (ident or proj) else ())
        if proj:
            r1 = r1 + ("take_dx",)
        if prev is not None:
            link.prev = prev
        a1 = self.conv1(x, fuse=(link, 1, r1) if link else None)
        a2 = self.conv2(a1, fuse=(link, 2, ("mask_in",)) if link else None)
        idt = x if ident else self.shortcut(x, fuse=(link, 0, ("stash_dx",)) if proj else None)
        out = self.conv3(a2, residual=idt, relu=True,
                         fuse=(link, 3, ("mask_in", "stash_res") if ident else ("mask_in",)) if link else None)
        if link is not None:
            out._mx_link = link
        return out


    def _bn_proj_ok(self, x) -> bool:
        """Both convs reading x (conv1, shortcut) take the implicit-GEMM forward (so conv1's
        backward finds the shortcut's parked dX); shape-only check with bf16 meta weights."""
        if self.shortcut is None or not (x.is_cuda and x.dtype == torch.bfloat16):
            return False
        for cn in (self.conv1, self.shortcut):
            wm = torch.empty(cn.conv.weight.shape, dtype=torch.bfloat16, device="meta")
            if not convwg.fwd_supported(x, wm, None, None, cn.conv.stride, cn.conv.padding, cn.conv.dilation):
                return False
        return True


class ResNet(nn.Module):
    def __init__(self, depth: int = 50, norm: str = "frozen", num_classes: Optional[int] = None,
                 freeze_at: int = 2, stride_in_1x1: bool = True):
        super().__init__()
        blocks = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3)}[depth]
        self.stem = ConvNorm(3, 64, 7, 2, 3, norm)
        self.freeze_at = freeze_at if norm == "frozen" else 0
        stages = []
        cin = 64
        for i, (n, w) in enumerate(zip(blocks, (64, 128, 256, 512))):
            layers = []
            for j in range(n):
                layers.append(Bottleneck(cin, w, (1 if i == 0 else 2) if j == 0 else 1, norm, stride_in_1x1))
                cin = w * 4
            stages.append(nn.Sequential(*layers))
        self.stages = nn.ModuleList(stages)
        self.out_channels = [256, 512, 1024, 2048]
        self.fc = nn.Linear(2048, num_classes) if num_classes else None
        if self.freeze_at:
            # tensorpack freezes the stem and res2 (FREEZE_AT=2)
            for p in self.stem.parameters():
                p.requires_grad_(False)
            for p in self.stages[0].parameters():
                p.requires_grad_(False)

    def forward_features(self, x, stem_done: bool = False) -> List[torch.Tensor]:
        """C2..C5; ``stem_done``: x is already the pooled stem output (ops/stem.py)."""
        if not stem_done:
            if self.stem.norm_kind == "bn" and self.stem.norm.training:
                # stem BN + ReLU folded into pool0 (ops/batchnorm.py bn_relu_maxpool)
                y, pre = self.stem.conv_pre(x)
                x = bn_relu_maxpool(y, self.stem.norm, pre)
            else:
                x = self.stem(x)
                x = maxpool3s2(x)   # (NHWC bf16: csrc/pool.hip; else F.max_pool2d(x, 3, 2, 1))
        outs = []
        for st in self.stages:
            x = st(x)
            outs.append(x)
        return outs   # C2..C5 (strides 4..32)

    def _casts(self, x):
        """Trainable-BN model under bf16 autocast: every conv weight's bf16 copy from one
        launch (and their fp32 gradients from one), instead of a cast kernel per weight each
        way (models/compute_weights.py CastGroup)."""
        if (self.stem.norm_kind != "bn" or not x.is_cuda or not torch.is_grad_enabled()
                or not torch.is_autocast_enabled("cuda") or torch.get_autocast_dtype("cuda") != torch.bfloat16):
            return contextlib.nullcontext()
        dp = torch.distributed.is_available() and torch.distributed.is_initialized()
        return _cw.CastGroup([m.conv.weight for m in self.modules() if isinstance(m, ConvNorm)],
                             groups=8 if dp else 1)

    def forward(self, x):
        with self._casts(x):
            c = self.forward_features(x)
        if self.fc is None:
            return c
        pooled = global_avg_pool(c[-1])   # (fp32 [N, C]; NHWC bf16: csrc/pool.hip, +0.5%)
        return self.fc(pooled)


@torch.no_grad()
def calibrate_frozen_bn(resnet: ResNet, images: torch.Tensor):
    """Give a random-init FrozenBN ResNet sane statistics: one forward pass over
    ``images`` (normalised NCHW) in which every FrozenBN takes the batch statistics of its
    conv output.  Without this a BN-free random ResNet-50 has activations growing by
    orders of magnitude through the 16 residual blocks."""
    ConvNorm.calibrating = True
    try:
        resnet.forward_features(images.float())
    finally:
        ConvNorm.calibrating = False


def resnet50(norm="frozen", num_classes=None, **kw) -> ResNet:
    return ResNet(50, norm, num_classes, **kw)
