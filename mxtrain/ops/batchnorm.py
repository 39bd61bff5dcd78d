"""Training-mode BatchNorm fused with the residual add and ReLU, NHWC bf16 (csrc/batchnorm.hip).

``bn_act(x, bn, residual, relu)`` computes ``act(BatchNorm(x) (+ residual))`` for an
``nn.BatchNorm2d`` ``bn`` whose affine parameters / running statistics stay fp32 (AMP
style): one statistics pass, a per-channel finalize (running statistics updated in place,
deterministic two-stage reductions) and one apply pass forward -- after a convolution on
csrc/convwg.hip the statistics come from that convolution's epilogue instead of a pass over
x; a statistics pass, a finalize and one pass producing dx (and the residual's gradient)
backward.  The ResNet-50
bottleneck's BN -> add -> ReLU tail is a single autograd node.  Evaluation mode (or the
CPU) uses the running statistics through the same apply kernel / plain torch ops.

Reference: the Ray Train Lightning ResNet-50 config (BASELINE.json config 5,
/root/reference/charts/machine-learning/training/raytrain/templates/train.yaml:142-221).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib


def _nhwc_ok(t: Optional[torch.Tensor]) -> bool:
    return t is None or (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 4
                         and t.is_contiguous(memory_format=torch.channels_last) and t.data_ptr() % 16 == 0)


ENABLED = True   # module switch (A/B runs: scripts/resnet_ab.py)
# backward statistics of BN + ReLU (no residual) from the output: xhat = (y - beta) / gamma
# where the ReLU passed (csrc/batchnorm.hip bn_bwd_stats_kernel kRecon), x not re-read
RECON = True   # (the test compares both passes)


def supported(x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> bool:
    return (ENABLED and _lib.use_hip(x) and _nhwc_ok(x) and _nhwc_ok(residual) and x.shape[1] % 8 == 0
            and (residual is None or residual.shape == x.shape))


def _scratch(M: int, C: int, device) -> torch.Tensor:
    return torch.empty(_lib.query64("mx_bn_scratch", M, C), dtype=torch.float32, device=device)


class BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, running_mean, running_var, momentum: float, eps: float, relu: bool,
                link=None, nbt=None, pre=None):
        N, C, H, W = x.shape
        M = N * H * W
        y = torch.empty_like(x, memory_format=torch.channels_last)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        g32 = gamma.detach().float().contiguous()
        b32 = beta.detach().float().contiguous()
        _lib.call("mx_bn_fwd", x.data_ptr(), _lib.ptr(residual), y.data_ptr(), g32.data_ptr(), b32.data_ptr(),
                  mean.data_ptr(), rstd.data_ptr(), _lib.ptr(running_mean), _lib.ptr(running_var), M, C,
                  float(eps), float(momentum), int(relu), _scratch(M, C, x.device).data_ptr(), _lib.ptr(nbt),
                  _lib.ptr(pre), _lib.stream())
        ctx.relu, ctx.has_res = relu, residual is not None
        ctx.link = link
        ctx.save_for_backward(x, y, mean, rstd, g32, b32)
        ctx.pdtypes = (gamma.dtype, beta.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, rstd, g32, b32 = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        N, C, H, W = x.shape
        M = N * H * W
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dres = torch.empty_like(x, memory_format=torch.channels_last) if ctx.has_res else None
        dg = torch.empty(C, dtype=torch.float32, device=x.device)
        db = torch.empty_like(dg)
        _lib.call("mx_bn_bwd", dy.data_ptr(), y.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                  g32.data_ptr(), dx.data_ptr(), _lib.ptr(dres), dg.data_ptr(), db.data_ptr(), 0, M, C,
                  int(ctx.relu), _scratch(M, C, x.device).data_ptr(), b32.data_ptr(),
                  int(RECON and ctx.relu and not ctx.has_res), _lib.stream())
        link = ctx.link
        if dres is not None and link is not None and link.taker and ctx.needs_input_grad[3]:
            # identity residual (ops/epilogue.py BlockLink): conv1's dgrad store adds it to the
            # block input's gradient, so autograd's add of the input's two gradients disappears
            link.stash.append(dres)
            dres = None
        return (dx, dg.to(ctx.pdtypes[0]), db.to(ctx.pdtypes[1]), dres, None, None, None, None, None, None, None,
                None)


def _stat_ptrs(*ts) -> "ctypes.Array":
    import ctypes
    return (ctypes.c_int64 * len(ts))(*[t.data_ptr() for t in ts])


class BN2AddReluFn(torch.autograd.Function):
    """relu(BN_a(xa) + BN_b(xb)) in training mode (csrc/batchnorm.hip mx_bn2_*): the ResNet
    projection block's tail -- conv3's BN and the shortcut's BN -- without the shortcut BN's
    output tensor.  Each BN's statistics / running statistics / batch count as ``bn_act``
    (mx_bn_fwd with y = null, from the convs' epilogue statistics when given); one apply
    pass forward; backward one statistics pass (the shared dz) and one apply pass writing
    both input gradients."""

    @staticmethod
    def forward(ctx, xa, ga, ba, xb, gb, bb, bufs_a, bufs_b):
        N, C, H, W = xa.shape
        M = N * H * W
        dev = xa.device
        stats = []
        for x, g, b, (rm, rv, mom, eps, nbt, pre) in ((xa, ga, ba, bufs_a), (xb, gb, bb, bufs_b)):
            mean = torch.empty(C, dtype=torch.float32, device=dev)
            rstd = torch.empty_like(mean)
            g32 = g.detach().float().contiguous()
            b32 = b.detach().float().contiguous()
            _lib.call("mx_bn_fwd", x.data_ptr(), 0, 0, g32.data_ptr(), b32.data_ptr(), mean.data_ptr(),
                      rstd.data_ptr(), _lib.ptr(rm), _lib.ptr(rv), M, C, float(eps), float(mom), 0,
                      _scratch(M, C, dev).data_ptr(), _lib.ptr(nbt), _lib.ptr(pre), _lib.stream())
            stats += [mean, rstd, g32, b32]
        y = torch.empty_like(xa, memory_format=torch.channels_last)
        ptrs = _stat_ptrs(*stats)
        _lib.call("mx_bn2_apply", xa.data_ptr(), xb.data_ptr(), y.data_ptr(), ptrs, M, C, _lib.stream())
        ctx.save_for_backward(xa, xb, y, *stats)
        ctx.pdtypes = (ga.dtype, ba.dtype, gb.dtype, bb.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        xa, xb, y, *stats = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        N, C, H, W = xa.shape
        M = N * H * W
        dxa = torch.empty_like(xa, memory_format=torch.channels_last)
        dxb = torch.empty_like(xb, memory_format=torch.channels_last)
        grads = [torch.empty(C, dtype=torch.float32, device=xa.device) for _ in range(4)]
        scratch = torch.empty(2 * _lib.query64("mx_bn_scratch", M, C), dtype=torch.float32, device=xa.device)
        _lib.call("mx_bn2_bwd", dy.data_ptr(), y.data_ptr(), xa.data_ptr(), xb.data_ptr(), _stat_ptrs(*stats),
                  dxa.data_ptr(), dxb.data_ptr(), *[t.data_ptr() for t in grads], M, C, scratch.data_ptr(),
                  _lib.stream())
        dga, dba, dgb, dbb = (t.to(d) for t, d in zip(grads, ctx.pdtypes))
        return dxa, dga, dba, dxb, dgb, dbb, None, None


def _bufs(bn: torch.nn.BatchNorm2d, pre):
    mom = bn.momentum
    nbt = None
    if bn.track_running_stats and bn.num_batches_tracked is not None:
        if mom is None:
            bn.num_batches_tracked.add_(1)
            mom = 1.0 / float(bn.num_batches_tracked)
        else:
            nbt = bn.num_batches_tracked
    return (bn.running_mean if bn.track_running_stats else None, bn.running_var if bn.track_running_stats else None,
            0.0 if mom is None else mom, bn.eps, nbt, pre)


def bn2_add_relu(xa: torch.Tensor, bn_a: torch.nn.BatchNorm2d, xb: torch.Tensor, bn_b: torch.nn.BatchNorm2d,
                 pre_a: Optional[torch.Tensor] = None, pre_b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """relu(bn_a(xa) + bn_b(xb)); one fused node when both BNs train on the HIP path, else
    the two-layer form (bn_b's output as bn_a's residual)."""
    if (DUAL and bn_a.training and bn_b.training and supported(xa, xb) and xa.shape == xb.shape
            and xb.data_ptr() % 16 == 0 and xa.data_ptr() % 16 == 0):
        return BN2AddReluFn.apply(xa, bn_a.weight, bn_a.bias, xb, bn_b.weight, bn_b.bias, _bufs(bn_a, pre_a),
                                  _bufs(bn_b, pre_b))
    return bn_act(xa, bn_a, residual=bn_act(xb, bn_b, None, False, pre=pre_b), relu=True, pre=pre_a)


# (+2.9 % ResNet-50 img/s through the launcher: profiles/r6/resnet_launcher_ab_bn2_add_relu.txt)
DUAL = True


def _rows_per_block(M: int) -> int:   # (csrc/batchnorm.hip rows_per_block)
    return max(64, (M + 511) // 512)


class BNReluMaxPoolFn(torch.autograd.Function):
    """max_pool2d(relu(BN(x)), 3, 2, 1) in training mode -- the ResNet stem's BN, ReLU and pool0
    -- without the BN + ReLU output tensor: the statistics pass and finalize (mx_bn_fwd with
    y = null), then the pool reads x and applies relu(x scale + shift) on load
    (csrc/pool.hip mx_maxpool3s2_fwd_bn); backward the pool's gather masks the ReLU from the
    pooled output (mx_maxpool3s2_bwd_relu) and a plain BN backward reads dz and x."""

    @staticmethod
    def forward(ctx, x, gamma, beta, bufs):
        rm, rv, mom, eps, nbt, pre = bufs
        N, C, H, W = x.shape
        M = N * H * W
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        g32 = gamma.detach().float().contiguous()
        b32 = beta.detach().float().contiguous()
        scratch = _scratch(M, C, x.device)
        _lib.call("mx_bn_fwd", x.data_ptr(), 0, 0, g32.data_ptr(), b32.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                  _lib.ptr(rm), _lib.ptr(rv), M, C, float(eps), float(mom), 0, scratch.data_ptr(), _lib.ptr(nbt),
                  _lib.ptr(pre), _lib.stream())
        rpb = _rows_per_block(M)
        off = 2 * ((M + rpb - 1) // rpb) * C   # scale, shift follow the partials (mx_bn_fwd)
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty((N, OH, OW, C), dtype=x.dtype, device=x.device)
        arg = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=x.device)
        _lib.call("mx_maxpool3s2_fwd_bn", x.data_ptr(), y.data_ptr(), arg.data_ptr(), N, H, W, C,
                  scratch[off:].data_ptr(), scratch[off + C:].data_ptr(), _lib.stream())
        ctx.save_for_backward(x, y, arg, mean, rstd, g32, b32)
        ctx.pdtypes = (gamma.dtype, beta.dtype)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, g):
        x, y, arg, mean, rstd, g32, b32 = ctx.saved_tensors
        N, C, H, W = x.shape
        M = N * H * W
        g = g.contiguous(memory_format=torch.channels_last)
        dz = torch.empty((N, H, W, C), dtype=x.dtype, device=x.device)
        _lib.call("mx_maxpool3s2_bwd_relu", g.data_ptr(), arg.data_ptr(), y.data_ptr(), dz.data_ptr(), N, H, W, C,
                  _lib.stream())
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dg = torch.empty(C, dtype=torch.float32, device=x.device)
        db = torch.empty_like(dg)
        _lib.call("mx_bn_bwd", dz.data_ptr(), 0, x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), g32.data_ptr(),
                  dx.data_ptr(), 0, dg.data_ptr(), db.data_ptr(), 0, M, C, 0, _scratch(M, C, x.device).data_ptr(),
                  b32.data_ptr(), 0, _lib.stream())
        return dx, dg.to(ctx.pdtypes[0]), db.to(ctx.pdtypes[1]), None


def bn_relu_maxpool(x: torch.Tensor, bn: torch.nn.BatchNorm2d, pre: Optional[torch.Tensor] = None) -> torch.Tensor:
    """max_pool2d(relu(bn(x)), 3, 2, 1): one fused node in training mode on the HIP path."""
    from .epilogue import maxpool3s2
    if POOL_FOLD and bn.training and supported(x) and x.dtype == torch.bfloat16 and x.data_ptr() % 16 == 0:
        return BNReluMaxPoolFn.apply(x, bn.weight, bn.bias, _bufs(bn, pre))
    return maxpool3s2(bn_act(x, bn, None, True, pre=pre))


# (+0.9 % ResNet-50 img/s through the launcher: profiles/r6/resnet_launcher_ab_stem_bn_pool_fold.txt)
POOL_FOLD = True


def bn_act_ref(x, gamma, beta, residual, running_mean, running_var, momentum, eps, relu, training=True):
    """The same op in plain torch (fp32 math): the CPU path and the tests' reference."""
    y = F.batch_norm(x.float(), running_mean, running_var, gamma.float(), beta.float(), training, momentum, eps)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = F.relu(y)
    return y.to(x.dtype)


def bn_act(x: torch.Tensor, bn: torch.nn.BatchNorm2d, residual: Optional[torch.Tensor] = None,
           relu: bool = False, link=None, pre: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(bn(x) (+ residual)) for an ``nn.BatchNorm2d`` (training: batch statistics and
    running-statistics update; eval: running statistics).  ``link``: a BlockLink whose taker
    (the block's conv1) adds the residual's gradient in its dgrad store.  ``pre``: x's
    per-64-row statistics from the producing convolution's epilogue (ops/convwg.py
    conv_fwd ``bn_stats``): the forward then never re-reads x for them."""
    if supported(x, residual):
        mom = bn.momentum
        nbt = None
        if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
            # (the torch fallback below counts the batch inside nn.BatchNorm2d.forward)
            if mom is None:   # cumulative moving average, as nn.BatchNorm2d
                bn.num_batches_tracked.add_(1)
                mom = 1.0 / float(bn.num_batches_tracked)
            else:             # counted by the statistics finalize kernel
                nbt = bn.num_batches_tracked
        if mom is None:
            mom = 0.0
        if bn.training:
            return BNActFn.apply(x, bn.weight, bn.bias, residual, bn.running_mean if bn.track_running_stats else None,
                                 bn.running_var if bn.track_running_stats else None, mom, bn.eps, relu, link, nbt,
                                 pre)
        # eval: y = act(x * scale + shift (+ res)) with the running statistics
        s = bn.weight.float() * torch.rsqrt(bn.running_var.float() + bn.eps)
        h = bn.bias.float() - bn.running_mean.float() * s
        y = torch.empty_like(x, memory_format=torch.channels_last)
        N, C, H, W = x.shape
        _lib.call("mx_bn_apply", x.data_ptr(), _lib.ptr(residual), y.data_ptr(), s.contiguous().data_ptr(),
                  h.contiguous().data_ptr(), N * H * W, C, int(relu), _lib.stream())
        return y
    y = bn(x)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y
