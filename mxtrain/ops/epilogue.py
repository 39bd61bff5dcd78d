"""Fused convolution epilogues for NHWC bf16 CNNs (csrc/epilogue.hip).

``conv_bias_act(x, w, b, ..., relu, residual)`` = act(conv(x, w) + b (+ residual)): MIOpen
runs the convolution without its bias and one HIP pass applies bias, residual and ReLU in
place; the backward fuses the ReLU mask with the bias gradient's column sums.  Replaces
PyTorch's channels_last path (conv, broadcast bias add, clamp, residual add, clamp) --
2-4 extra passes over every activation and as many launches per conv.

CPU / non-channels_last tensors take the plain PyTorch ops (same math).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from . import convwg

_ENABLED = True


def _rows_cols(y: torch.Tensor):
    return y.numel() // y.shape[1], y.shape[1]


def _nhwc(t: Optional[torch.Tensor]) -> bool:
    return t is None or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


class BiasActFn(torch.autograd.Function):
    """y <- act(y + b (+ res)) in place on the conv output y (channels_last bf16)."""

    @staticmethod
    def forward(ctx, y, b, res, relu: bool):
        M, C = _rows_cols(y)
        _lib.call("mx_bias_act_fwd", _lib.ptr(y), _lib.ptr(b), _lib.ptr(res), M, C, int(relu), _lib.stream())
        ctx.mark_dirty(y)
        ctx.relu, ctx.has_res, ctx.want_db = relu, res is not None, b is not None and b.requires_grad
        ctx.bdtype = b.dtype if b is not None else None
        convwg.note_use(b)
        ctx.bkey = b.data_ptr() if b is not None else None
        if relu:
            ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        relu, want_db = ctx.relu, ctx.want_db and ctx.needs_input_grad[1]
        if not relu and not want_db:
            return g, None, (g if ctx.has_res else None), None
        if not _nhwc(g):
            g = g.contiguous(memory_format=torch.channels_last)
        M, C = _rows_cols(g)
        dy = torch.empty_like(g) if relu else g
        db = torch.empty(C, dtype=torch.bfloat16, device=g.device) if want_db else None
        nparts = _lib.query("mx_bias_act_bwd_parts", M, C)
        partial, flags = _colsum_partial(g.device, nparts, C, db, ctx.bdtype, ctx.bkey)
        out = ctx.saved_tensors[0] if relu else None
        _lib.call("mx_bias_act_bwd", _lib.ptr(g), _lib.ptr(out), _lib.ptr(dy), _lib.ptr(db), _lib.ptr(partial),
                  M, C, int(relu), flags, _lib.stream())
        if db is not None and db.dtype != ctx.bdtype:
            db = db.to(ctx.bdtype)
        return dy, db, (dy if ctx.has_res else None), None


def _bias_act_bwd(g, out, relu: bool, want_db: bool, bdtype=torch.bfloat16, bkey=None):
    """(dy, db) of y = act(conv + b (+ res)): the ReLU mask and the bias-gradient column sums
    in one pass (csrc/epilogue.hip)."""
    if not _nhwc(g):
        g = g.contiguous(memory_format=torch.channels_last)
    if not relu and not want_db:
        return g, None
    M, C = _rows_cols(g)
    dy = torch.empty_like(g) if relu else g
    db = torch.empty(C, dtype=torch.bfloat16, device=g.device) if want_db else None
    nparts = _lib.query("mx_bias_act_bwd_parts", M, C)
    partial, flags = _colsum_partial(g.device, nparts, C, db, bdtype, bkey)
    _lib.call("mx_bias_act_bwd", _lib.ptr(g), _lib.ptr(out), _lib.ptr(dy), _lib.ptr(db), _lib.ptr(partial),
              M, C, int(relu), flags, _lib.stream())
    return dy, db


def _colsum_partial(device, nparts: int, C: int, db: Optional[torch.Tensor], bdtype=torch.bfloat16, key=None):
    """(fp32 partial buffer, mx_bias_act_bwd flags): the bias gradient's column sums are
    deferred to the step's batched flush (ops/convwg.py) when that is on, else reduced at once
    (also when the caller casts db right away: a deferred db is only final after the flush)."""
    if db is None:
        return None, 0
    if bdtype != torch.bfloat16:
        return torch.empty(nparts * C, dtype=torch.float32, device=device), 0
    reg = convwg.defer_colsum(device, nparts, C, db, key)
    if reg is not None:
        return reg, 2
    return torch.empty(nparts * C, dtype=torch.float32, device=device), 0


class BlockLink:
    """Backward-fusion contract between the convolutions of one bottleneck block (built by
    models/resnet.py; every field is decided in the forward, read in the backward):

    * ``premask[k]``: the consumer of conv k's output (conv k+1) multiplies its input
      gradient by (its input > 0) in its dgrad store -- conv k's ReLU -- so conv k's
      backward skips its own ReLU-mask pass;
    * ``stash``: identity residual: conv3's backward puts the residual branch's gradient
      here instead of returning it, and conv1's backward adds it in its dgrad store (conv1
      always runs after conv3 in backward: data dependency), so autograd's separate add
      of the block input's two gradients disappears;
    * role "mask_prev" (conv1 of an identity block whose input is the previous block's
      ReLU output): its dgrad store, which then holds the input's whole gradient, also
      applies that ReLU (``prev.premask[3]``).  Masking is idempotent, so a consumer that
      masks a gradient its producer masks too is only wasted work, never wrong."""

    __slots__ = ("premask", "stash", "taker", "prev")

    def __init__(self):
        self.premask = {}
        self.stash = []
        self.taker = False    # conv1 runs ConvBiasActFn with role "take_res" (set in its forward)
        self.prev = None      # the previous block's link when conv1 has role "mask_prev"


class JoinLink(BlockLink):
    """FPN top-down join (models/maskrcnn.py FPN): merged level i has two consumers, its 3 x 3
    output conv (role "join_dx", key i) and the next lateral conv, which reads it
    nearest-upsampled as its residual (role "join_res", key i).  Whichever backward runs
    first parks its gradient in ``join[i]`` (the output conv its dX, the lateral conv its
    full-resolution residual gradient) and returns None for the level; the second returns
    the level's whole gradient from one pass, fp32 2 x 2 block sum + dX, rounded once -- the
    same arithmetic in either order (eager and captured steps must agree bit for bit) -- so
    autograd's separate add and the upsampling gradient's reduce + cast passes disappear."""

    __slots__ = ("join",)

    def __init__(self):
        super().__init__()
        self.join = {}


# projection blocks with 1 x 1 stride-2 convs (A/B switch): the shortcut's parked input
# gradient holds only the (0, 0) parity class (ops/convwg.py conv_dgrad class_out)
# (+1.4 % ResNet-50 img/s: profiles/r6/resnet_launcher_ab_class_stash.txt)
CLASS_STASH = True


def _class_spread(c: torch.Tensor, x_shape, s: int) -> torch.Tensor:
    """A compact parity-class gradient [N, C, ceil(H / s), ceil(W / s)] at its pixels of X's shape."""
    full = torch.zeros(x_shape, dtype=c.dtype, device=c.device, memory_format=torch.channels_last)
    full[:, :, ::s, ::s] = c
    return full


class ConvBiasActFn(torch.autograd.Function):
    """act(conv2d(x, w) + b (+ res)) with every direction on csrc/convwg.hip where it tiles:
    forward = one implicit-GEMM launch with the epilogue fused; backward = the ReLU mask +
    bias-gradient pass, then the implicit-GEMM input and weight gradients.  With a
    ``BlockLink`` (``fuse`` = (link, k, role)): role "mask_in" folds the producer's ReLU
    into this conv's dgrad, role "stash_res" hands the residual gradient to conv1, role
    "take_res" adds it (see BlockLink)."""

    @staticmethod
    def forward(ctx, x, w, b, res, relu: bool, stride, padding, dilation, fuse=None, res_up=False, bnpre=None):
        # bnpre: a list that receives the epilogue's BatchNorm statistics of y (or None) for
        # the trainable-BN ResNet (ops/batchnorm.py bn_act ``pre``)
        if bnpre is not None:
            y, pre = convwg.conv_fwd(x, w, b, res, relu, stride, padding, dilation, res_up=res_up, bn_stats=True)
            bnpre.append(pre)
        else:
            y = convwg.conv_fwd(x, w, b, res, relu, stride, padding, dilation, res_up=res_up)
        ctx.conf = (list(convwg._pair(stride)), list(convwg._pair(padding)), list(convwg._pair(dilation)))
        ctx.relu, ctx.has_res, ctx.res_up = relu, res is not None, res_up
        ctx.bdtype = b.dtype if b is not None else None
        ctx.fuse = fuse
        convwg.note_use(w)
        convwg.note_use(b)
        ctx.wkey, ctx.bkey = w.data_ptr(), (b.data_ptr() if b is not None else None)
        ctx.save_for_backward(x, w, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, out = ctx.saved_tensors
        st, pd, dl = ctx.conf
        want_db = ctx.needs_input_grad[2]
        link, k, roles = ctx.fuse if ctx.fuse is not None else (None, -1, ())
        # a premasked gradient already carries this conv's ReLU (the consumer's dgrad store
        # applied it): only the bias gradient, if any, is left -- column sums of g itself
        relu = ctx.relu and not (link is not None and link.premask.get(k))
        dy, db = _bias_act_bwd(g, out, relu, want_db, ctx.bdtype, ctx.bkey)
        if db is not None and db.dtype != ctx.bdtype:
            db = db.to(ctx.bdtype)
        dres = dy if ctx.has_res else None
        if dres is not None and ctx.res_up:
            if "join_res" in roles and k in link.join:     # the output conv's dX came first
                dres = down2_sum(dres, link.join.pop(k))
            elif "join_res" in roles:                      # park the full-resolution gradient
                link.join[k] = dres
                dres = None
            else:
                dres = down2_sum(dres)
        if dres is not None and "stash_res" in roles and link.taker and ctx.needs_input_grad[3]:
            link.stash.append(dres)
            dres = None
        if "take_dx" in roles and ctx.needs_input_grad[0] and link.taker and not link.stash:
            # (the projection shortcut's dX must already be parked: see models/resnet.py)
            raise RuntimeError("BlockLink: conv1 ran before the projection shortcut's backward")
        add = link.stash.pop() if "take_res" in roles and link.stash else None
        join_first = join_last = None
        if "join_dx" in roles:   # (the same sum, fp32 2 x 2 block + bf16 dX, whichever comes first)
            if k in link.join:
                join_last = link.join.pop(k)
            else:
                join_first = True
        mask = x if ("mask_in" in roles or "mask_prev" in roles) else None
        dx = dw = None
        # (Cin = 64 tiles half padded: even with MIOpen at the ResNet res2 shapes, so MIOpen keeps them;
        # a plain hipBLASLt GEMM on the NHWC views loses to MIOpen there too, dgrad 92 vs 59 us,
        # wgrad 1017 vs 47 us: profiles/r6/resnet_gemm_dgrad_1x1_rejected.txt)
        wg_hip = ctx.needs_input_grad[1] and convwg.cout_ok(w.shape[0]) and w.shape[1] % 128 == 0
        if ctx.needs_input_grad[0]:
            # a 1 x 1 stride-2 projection shortcut parks only the pixels its filter reaches
            # (compact parity class, no zero fill); conv1 adds them in its own class launch when
            # it is such a conv too (stride_in_1x1), else they are spread to X's shape first
            cls_out = (CLASS_STASH and "stash_dx" in roles and link.taker and add is None and mask is None
                       and convwg.class_ok(w, tuple(x.shape), st, pd, dl))
            add_cls = add is not None and getattr(add, "_mx_class", 0)
            if add_cls:
                s = add._mx_class
                if not (convwg.class_ok(w, tuple(x.shape), st, pd, dl) and list(st) == [s, s]):
                    add = _class_spread(add, tuple(x.shape), s)
                    add_cls = 0
            if cls_out:
                dx = convwg.conv_dgrad(dy, w, tuple(x.shape), st, pd, dl, class_out=True)
                dx._mx_class = st[0]
            elif convwg.dgrad_supported(w, tuple(x.shape), st, pd, dl) and (add is None or add.data_ptr() % 16 == 0):
                dx = convwg.conv_dgrad(dy, w, tuple(x.shape), st, pd, dl, add=add, mask=mask, add_class=bool(add_cls))
            else:
                dx = torch.ops.aten.convolution_backward(dy, x, w, None, st, pd, dl, False, [0, 0], 1,
                                                         [True, False, False])[0]
                if add is not None:
                    dx = dx + add
                if mask is not None:
                    dx = torch.where(mask > 0, dx, torch.zeros_like(dx))
            if "stash_dx" in roles and link.taker and dx is not None:
                link.stash.append(dx)   # conv1's dgrad store adds it (role "take_dx")
                dx = None
            if join_first:
                link.join[k] = dx
                dx = None
            elif join_last is not None:
                dx = down2_sum(join_last, dx)
        elif add is not None:
            raise RuntimeError("BlockLink: residual gradient stashed for a conv without an input gradient")
        if ctx.needs_input_grad[1]:
            if wg_hip:   # (narrow Cout: zero-padded row tile)
                dw = convwg.conv_wgrad(dy, x, tuple(w.shape), st, pd, dl, key=ctx.wkey)
            else:
                dw = torch.ops.aten.convolution_backward(dy, x, w, None, st, pd, dl, False, [0, 0], 1,
                                                         [False, True, False])[1]
        return dx, dw, db, dres, None, None, None, None, None, None, None


class Subsample2Fn(torch.autograd.Function):
    """max_pool2d(x, 1, 2) of an NHWC bf16 tensor -- FPN P6 = every second row / column of P5 --
    on csrc/epilogue.hip mx_subsample2 in both directions (torch's max-pool kernels: ~10 us
    forward, ~37 us backward on these few-KB tensors)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        ctx.shape = (N, C, H, W)
        y = torch.empty((N, (H + 1) // 2, (W + 1) // 2, C), dtype=x.dtype, device=x.device)
        _lib.call("mx_subsample2", x.data_ptr(), y.data_ptr(), N, H, W, C, 0, _lib.stream())
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        if not _nhwc(g) or g.data_ptr() % 16:
            g = g.contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, H, W, C), dtype=g.dtype, device=g.device)
        _lib.call("mx_subsample2", g.data_ptr(), dx.data_ptr(), N, H, W, C, 1, _lib.stream())
        return dx.permute(0, 3, 1, 2)


def subsample2(x: torch.Tensor) -> torch.Tensor:
    """F.max_pool2d(x, 1, 2) (kernel 1: a plain stride-2 subsample)."""
    if (_lib.use_hip(x) and x.dtype == torch.bfloat16 and _nhwc(x) and x.shape[1] % 8 == 0
            and x.data_ptr() % 16 == 0):
        return Subsample2Fn.apply(x)
    return F.max_pool2d(x, 1, 2)


class MaxPool3s2Fn(torch.autograd.Function):
    """max_pool2d(x, 3, 2, 1) of an NHWC bf16 tensor (the ResNet stem's pool0) on csrc/pool.hip:
    a one-byte window argmax instead of torch's int64 indices, and a gathering backward (each
    input pixel sums the <= 4 windows that picked it: deterministic, no zero fill)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty((N, OH, OW, C), dtype=x.dtype, device=x.device)
        arg = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=x.device)
        _lib.call("mx_maxpool3s2_fwd", x.data_ptr(), y.data_ptr(), arg.data_ptr(), N, H, W, C, _lib.stream())
        ctx.save_for_backward(arg)
        ctx.shape = (N, C, H, W)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, g):
        (arg,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        if not _nhwc(g) or g.data_ptr() % 16:
            g = g.contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, H, W, C), dtype=g.dtype, device=g.device)
        _lib.call("mx_maxpool3s2_bwd", g.data_ptr(), arg.data_ptr(), dx.data_ptr(), N, H, W, C, _lib.stream())
        return dx.permute(0, 3, 1, 2)


def maxpool3s2(x: torch.Tensor) -> torch.Tensor:
    """F.max_pool2d(x, 3, 2, 1)."""
    if (_lib.use_hip(x) and x.dtype == torch.bfloat16 and _nhwc(x) and x.shape[1] % 8 == 0
            and x.data_ptr() % 16 == 0):
        return MaxPool3s2Fn.apply(x)
    return F.max_pool2d(x, 3, 2, 1)


class GlobalAvgPoolFn(torch.autograd.Function):
    """x.float().mean(dim=(2, 3)) of an NHWC bf16 tensor -> fp32 [N, C] in one launch each way
    (csrc/pool.hip mx_gap_fwd / mx_gap_bwd)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        y = torch.empty((N, C), dtype=torch.float32, device=x.device)
        _lib.call("mx_gap_fwd", x.data_ptr(), y.data_ptr(), N, H * W, C, _lib.stream())
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        g = g.float().contiguous()
        dx = torch.empty((N, H, W, C), dtype=torch.bfloat16, device=g.device)
        _lib.call("mx_gap_bwd", g.data_ptr(), dx.data_ptr(), N, H * W, C, _lib.stream())
        return dx.permute(0, 3, 1, 2)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """x.float().mean(dim=(2, 3)) (fp32 [N, C])."""
    if (_lib.use_hip(x) and x.dtype == torch.bfloat16 and _nhwc(x) and x.shape[1] % 8 == 0
            and x.data_ptr() % 16 == 0):
        return GlobalAvgPoolFn.apply(x)
    return x.float().mean(dim=(2, 3))


def down2_sum(g: torch.Tensor, add: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Gradient of the 2x nearest upsampling: each 2 x 2 block summed (+ ``add``, a second
    gradient of the same tensor), NHWC memory kept -- one pass (csrc/epilogue.hip
    mx_down2_add) on the GPU path."""
    N, C, H, W = g.shape
    if (_lib.use_hip(g) and g.dtype == torch.bfloat16 and _nhwc(g) and C % 8 == 0 and H % 2 == 0 and W % 2 == 0
            and (add is None or (add.dtype == torch.bfloat16 and _nhwc(add) and add.shape == (N, C, H // 2, W // 2)))):
        out = torch.empty((N, H // 2, W // 2, C), dtype=g.dtype, device=g.device)
        _lib.call("mx_down2_add", _lib.ptr(g), _lib.ptr(add), _lib.ptr(out), N, H // 2, W // 2, C, _lib.stream())
        return out.permute(0, 3, 1, 2)
    t = g.permute(0, 2, 3, 1).reshape(N, H // 2, 2, W // 2, 2, C).sum((2, 4), dtype=torch.float32)
    t = t.to(g.dtype).permute(0, 3, 1, 2)
    return t if add is None else t + add


def _fused_ok(y, b, residual) -> bool:
    return (_ENABLED and y.is_cuda and y.dtype == torch.bfloat16 and _nhwc(y) and _nhwc(residual)
            and y.shape[1] % 8 == 0 and y.shape[1] <= 2048
            and (b is None or (b.dtype == torch.bfloat16 and b.is_contiguous()))
            and (residual is None or (residual.dtype == torch.bfloat16 and residual.shape == y.shape)))


def bias_act(y: torch.Tensor, b: Optional[torch.Tensor], residual: Optional[torch.Tensor] = None,
             relu: bool = False) -> torch.Tensor:
    """act(y + b (+ residual)); in place on ``y`` when the fused kernel runs."""
    if _fused_ok(y, b, residual):
        if b is None and residual is None and not relu:
            return y
        return BiasActFn.apply(y, b, residual, relu)
    if b is not None:
        y = y + b.view(1, -1, 1, 1)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y

def _conv_in_ok(x, w, b, residual) -> bool:
    """conv_bias_act's input-side conditions for the fused epilogues (the residual has the
    OUTPUT's shape: convwg.fwd_supported / bias_act check it against the conv output)."""
    return (_ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and _nhwc(x) and _nhwc(residual)
            and x.shape[1] == w.shape[1] and w.shape[0] % 8 == 0 and w.shape[0] <= 2048
            and (b is None or (b.dtype == torch.bfloat16 and b.is_contiguous()))
            and (residual is None or residual.dtype == torch.bfloat16))

def fused_conv_ok(x, w, b=None, residual=None, stride=1, padding=0, dilation=1) -> bool:
    """True when conv_bias_act runs ConvBiasActFn (every direction on csrc/convwg.hip)."""
    return _conv_in_ok(x, w, b, residual) and convwg.fwd_supported(x, w, b, residual, stride, padding, dilation)

def conv_bias_act(x, w, b=None, stride=1, padding=0, dilation=1, relu: bool = False,
                  residual: Optional[torch.Tensor] = None, fuse=None, res_up: bool = False) -> torch.Tensor:
    """act(conv2d(x, w) + b (+ residual)) -- one conv (MIOpen forward and input gradient;
    the weight gradient from csrc/convwg.hip where it tiles) + one fused epilogue pass.
    ``fuse``: (BlockLink, index, roles) -- only honoured on the ConvBiasActFn path (the
    caller checks fused_conv_ok before promising a role to a neighbour).  ``res_up``: the
    residual is at half resolution and joins nearest-upsampled (FPN top-down pathway); the
    implicit-GEMM forward reads it in place, elsewhere it is upsampled first."""
    if _conv_in_ok(x, w, b, residual):
        if res_up and convwg.fwd_supported(x, w, b, residual, stride, padding, dilation, res_up=True):
            return ConvBiasActFn.apply(x, w, b, residual, relu, stride, padding, dilation, fuse, True)
        if res_up:
            residual, res_up = F.interpolate(residual, scale_factor=2, mode="nearest"), False
        if convwg.fwd_supported(x, w, b, residual, stride, padding, dilation):
            # forward, input and weight gradients all implicit GEMMs (ops/convwg.py)
            return ConvBiasActFn.apply(x, w, b, residual, relu, stride, padding, dilation, fuse, False)
        if convwg.supported(x, w, stride, padding, dilation):
            # MIOpen forward / input gradient, implicit-GEMM weight gradient (ops/convwg.py)
            return bias_act(convwg.conv2d_wg(x, w, stride, padding, dilation), b, residual, relu)
        return bias_act(F.conv2d(x, w, None, stride, padding, dilation), b, residual, relu)
    y = F.conv2d(x, w, b, stride, padding, dilation)
    if residual is not None:
        y = y + (F.interpolate(residual, scale_factor=2, mode="nearest") if res_up else residual)
    return F.relu(y, inplace=True) if relu else y

class ConvTransposeBiasActFn(torch.autograd.Function):
    """act(conv_transpose2d(x, w, stride=s) + b) for a filter within s x s (windows do not
    overlap: the mask head's 2x2 stride-2 upsampling, tensorpack
    examples/FasterRCNN/modeling/model_mrcnn.py maskrcnn_upXconv_head) on csrc/convwg.hip.
    A transposed convolution is the input gradient of conv2d(., w): forward = the
    stride-decomposed dgrad kernel (one GEMM per output parity class) with bias + ReLU in its
    store; backward = the ReLU-mask + bias-gradient pass, then dX = conv2d(dy, w, stride s)
    on the implicit-GEMM forward and dW = the implicit-GEMM weight gradient of that conv2d
    with x and dy in each other's roles."""

    @staticmethod
    def forward(ctx, x, w, b, stride: int, relu: bool):
        N, _, H, W = x.shape
        _, Co, KH, KW = w.shape
        convwg.note_use(w)
        convwg.note_use(b)
        ctx.wkey, ctx.bkey = w.data_ptr(), (b.data_ptr() if b is not None else None)
        w = w.contiguous(memory_format=torch.channels_last)
        y = convwg.conv_dgrad(x, w, (N, Co, (H - 1) * stride + KH, (W - 1) * stride + KW), stride, 0, 1,
                              bias=b, relu=relu)
        ctx.stride, ctx.relu = stride, relu
        ctx.bdtype = b.dtype if b is not None else None
        ctx.save_for_backward(x, w, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, out = ctx.saved_tensors
        st = ctx.stride
        dy, db = _bias_act_bwd(g, out, ctx.relu, ctx.needs_input_grad[2], getattr(ctx, "bdtype", torch.bfloat16),
                               ctx.bkey)
        if db is not None and db.dtype != ctx.bdtype:
            db = db.to(ctx.bdtype)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if convwg.fwd_supported(dy, w, None, None, st, 0, 1):
                dx = convwg.conv_fwd(dy, w, None, None, False, st, 0, 1)
            else:
                dx = F.conv2d(dy, w, None, st)
        if ctx.needs_input_grad[1]:
            dw = convwg.conv_wgrad(x, dy, tuple(w.shape), st, 0, 1, key=ctx.wkey)
        return dx, dw, db, None, None

def _deconv_ok(x, w, b, stride) -> bool:
    """ConvTransposeBiasActFn's conditions: NHWC bf16, non-overlapping windows, channel
    counts the weight-gradient tiles take (multiples of 128), enough output tiles."""
    if not (_ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and _nhwc(x)
            and x.dim() == 4 and w.dim() == 4 and x.shape[1] == w.shape[0] and x.data_ptr() % 16 == 0
            and isinstance(stride, int) and w.shape[0] % 128 == 0 and w.shape[1] % 128 == 0
            and (b is None or (b.dtype == torch.bfloat16 and b.is_contiguous() and b.data_ptr() % 8 == 0))
            and convwg.decomposed(w.shape[2], w.shape[3], stride, 0, 1)):
        return False
    N, _, H, W = x.shape
    out_shape = (N, w.shape[1], (H - 1) * stride + w.shape[2], (W - 1) * stride + w.shape[3])
    return convwg.dgrad_supported(w, out_shape, stride, 0, 1)

def conv_transpose_bias_act(x, w, b=None, stride=1, relu: bool = False) -> torch.Tensor:
    """act(conv_transpose2d(x, w, stride) + b); ConvTransposeBiasActFn where it applies."""
    if _deconv_ok(x, w, b, stride):
        return ConvTransposeBiasActFn.apply(x, w, b, stride, relu)
    if _fused_ok(x, b, None):
        return bias_act(F.conv_transpose2d(x, w, None, stride=stride), b, None, relu)
    y = F.conv_transpose2d(x, w, b, stride=stride)
    return F.relu(y, inplace=True) if relu else y
