"""Convolution weight gradients as implicit GEMMs (csrc/convwg.hip).

``conv2d_wg(x, w, stride, padding, dilation)`` is ``F.conv2d`` (MIOpen forward) whose
backward computes the weight gradient with the hand-written implicit-GEMM kernel -- one
launch per conv (every filter tap in it), split over the output pixels, written straight
into the channels_last bf16 gradient of the compute copy -- and the input gradient with
its implicit-GEMM counterpart (dY rows gathered per tap).
That replaces MIOpen's weight-gradient solvers and their fp32 workspace fill / cast
helpers, ~2.9 ms of the ~12 ms graphed Mask R-CNN step
(profiles/r2_maskrcnn_s3/census_1img_graph_948_kernels.txt).

Convs the kernel does not tile (Cout or Cin not a multiple of 128, groups, non-NHWC or
non-bf16 tensors, CPU) take plain ``F.conv2d`` -- part of the contract, not an error path.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Tuple

import torch
import torch.nn.functional as F

from . import _lib

ENABLED = True          # module switch (A/B runs: scripts/conv_wgrad_bench.py)
DGRAD = True            # input gradient from csrc/convwg.hip too (else MIOpen's backward-data)
FWD = True              # forward with the fused bias / residual / ReLU epilogue (else MIOpen)
FWD_MIN_TILES = 64
# forward convs with fewer 128 x 128 output tiles than this run 128 x 64 tiles (twice the
# workgroups, so a shallower K split or none)
FWD_HALF_TILES = 128
TARGET_WGS = 512        # two 128 x 128 workgroups per CU on 256 CUs; >= 16 K-steps per slice since
MIN_STEPS = 16          # the 32-bit gather made the slices cheaper than their fp32 partials
                        # (profiles/r4_s3/wgrad_split_ab*_{1,4}img.txt; before: r4_s2 sweep, 8)
_DESC_T = ctypes.c_int64 * 32
_WS: Dict[Tuple[torch.device, int], Tuple[torch.Tensor, torch.Tensor]] = {}
_RETIRED = []           # outgrown slabs stay alive: a captured hipGraph may still write them


def _pair(v) -> Tuple[int, int]:
    if isinstance(v, int):
        return v, v
    v = tuple(v)
    return (v[0], v[0]) if len(v) == 1 else (v[0], v[1])


def _sym(v):
    a, b = _pair(v)
    return a if a == b else None


def _cl(t: torch.Tensor) -> bool:
    return t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)


def supported(x: torch.Tensor, w: torch.Tensor, stride=1, padding=0, dilation=1, groups: int = 1) -> bool:
    return (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and groups == 1
            and x.dim() == 4 and w.dim() == 4 and w.requires_grad and w.shape[0] % 128 == 0
            and w.shape[1] % 128 == 0 and x.shape[1] == w.shape[1] and _cl(x)
            and None not in (_sym(stride), _sym(padding), _sym(dilation)) and isinstance(padding, (int, tuple, list))
            and x.data_ptr() % 16 == 0)


def plan_splits(T: int, ntiles: int) -> int:
    """Pixel slices per launch: enough workgroups to fill the chip (TARGET_WGS), each slice
    at least MIN_STEPS K-steps of 64 pixels (its 64-KiB fp32 partial tile is then small
    next to its MFMA work)."""
    bk = 64
    steps = (T + bk - 1) // bk
    s = max(1, min(TARGET_WGS // max(ntiles, 1), steps // MIN_STEPS))
    return int(_lib.query("mx_conv_wgrad_splits", T, max(s, 1)))


# split-K forward / input gradient: the last-arriving split of each tile sums the partials and
# runs the epilogue (csrc/convwg.hip split_last_arriver) instead of a reduction launch.  OFF:
# its agent-scope release is a whole-L2 write-back (buffer_wbl2) per workgroup, and the step
# ran 130.3 img/s with it vs 152.4 with the reduction launches at one image
# (profiles/r5_s1/mrcnn_ab_split_in_kernel_1img.txt)
SPLIT_IN_KERNEL = False
_TICKETS: Dict[torch.device, torch.Tensor] = {}


def _tickets(device) -> int:
    """Per-tile arrival counters (uint32, zero between launches: the last arriver resets its own)."""
    t = _TICKETS.get(device)
    if t is None:
        t = _TICKETS[device] = torch.zeros(1 << 16, dtype=torch.int32, device=device)
    return t.data_ptr()


def _workspace(device, slab_elems: int):
    """(fp32 split-K slab, 256 zero bf16): grown on demand, so the first (eager) steps size
    it before a hipGraph capture records its address."""
    key = (device, _lib.stream())   # per stream: kernels on two streams never share a workspace
    ws = _WS.get(key)
    if ws is None or ws[0].numel() < slab_elems:
        if ws is not None:
            _RETIRED.append(ws)
        s = max(slab_elems, ws[0].numel() if ws else 0, 1)
        ws = _WS[key] = (torch.empty(s, device=device, dtype=torch.float32),
                            torch.zeros(256, device=device, dtype=torch.bfloat16))
    return ws


# Deferred split-K reductions (FlatMaster, models/compute_weights.py): between
# ``defer_begin()`` (forward of a training step) and ``defer_flush()`` (right before the
# optimizer reads the gradients) every split weight gradient keeps its fp32 partials in its
# own region of a persistent arena and the reductions run as ONE launch
# (mx_conv_wgrad_reduce_batched) instead of one small launch per convolution (44 per 1-img
# Mask R-CNN step at ~5-7 us each, profiles/r5_s1/maskrcnn_1img_census_nms_par.txt).  The
# arena is sized by the eager steps; a capture that would outgrow it reduces immediately.
DEFER_WGRAD = True      # module switch (A/B)
_DEF = {"on": False, "jobs": [], "cjobs": [], "arena": None, "cursor": 0, "total": 0, "peak": 0,
        "uses": {}}
_DEF_RETIRED = []


def defer_begin(keys=()):
    """Start a deferring step.  ``keys`` are the data pointers of the FlatMaster compute
    copies: only a gradient of one of those, used by exactly ONE op of this forward
    (``note_use``), is deferred -- its unfinished dW / db then reaches _FlatCast.backward
    untouched.  A weight used twice (autograd would sum two unfinished gradients) or one
    outside the FlatMaster (AccumulateGrad, hooks) is reduced at once."""
    if _DEF["jobs"] or _DEF["cjobs"]:   # (a backward that never reached its flush)
        defer_flush(keep_on=False)
    _DEF["on"] = DEFER_WGRAD
    _DEF["uses"] = {int(k): 0 for k in keys}
    _DEF["jobs"] = []
    _DEF["cjobs"] = []
    _DEF["cursor"] = 0
    _DEF["total"] = 0


def note_use(t) -> None:
    """Forward of an op whose weight / bias gradient may be deferred: count the use."""
    if _DEF["on"] and t is not None:
        k = t.data_ptr()
        if k in _DEF["uses"]:
            _DEF["uses"][k] += 1


def _deferrable(key) -> bool:
    return (_DEF["on"] and key is not None and _DEF["uses"].get(key) == 1
            and torch._C._current_autograd_node() is not None)


def defer_flush(keep_on: bool = False):
    """Launch the pending reductions; deferral stays on only if ``keep_on`` (more gradient
    buckets of this backward still to come)."""
    _DEF["on"] = _DEF["on"] and keep_on
    for key, fn, width in (("jobs", "mx_conv_wgrad_reduce_batched", 10), ("cjobs", "mx_colsum_jobs", 5)):
        jobs = _DEF[key]
        if jobs:
            flat = [v for j in jobs for v in j]
            arr = (ctypes.c_int64 * len(flat))(*flat)
            _lib.call(fn, ctypes.addressof(arr), len(jobs), _lib.stream())
        _DEF[key] = []
    _DEF["cursor"] = 0
    # an arena outgrown mid-step held only the later jobs: size it for the whole step now
    # (eager), so the capture that follows this shape's eager step defers every reduction
    a = _DEF["arena"]
    _DEF["peak"] = max(_DEF["peak"], _DEF["total"])
    if a is not None and a.numel() < _DEF["peak"] and not torch.cuda.is_current_stream_capturing():
        _DEF_RETIRED.append(a)
        _DEF["arena"] = torch.empty(_DEF["peak"], device=a.device, dtype=torch.float32)


def deferring() -> bool:
    """Deferral is on and the caller runs inside an autograd backward."""
    return _DEF["on"] and torch._C._current_autograd_node() is not None


def defer_colsum(device, nparts: int, C: int, out: torch.Tensor, key=None):
    """fp32 [nparts * C] arena region for a bias gradient's column partials, reduced into the
    bf16 ``out`` at the flush; None when deferral is off or the bias (``key``: its data
    pointer) is not a single-use FlatMaster copy (reduce immediately)."""
    if not _deferrable(key):
        return None
    reg = _defer_slab(device, nparts * C)
    if reg is not None:
        _DEF["cjobs"].append([reg.data_ptr(), out.data_ptr(), nparts, C, 0])
    return reg


def _defer_slab(device, elems: int):
    """fp32 region of the deferral arena for one weight gradient's partials, or None."""
    need = (elems + 63) // 64 * 64
    _DEF["total"] += need
    a = _DEF["arena"]
    cur = _DEF["cursor"]
    if a is None or a.device != device or a.numel() < cur + need:
        if torch.cuda.is_current_stream_capturing():
            return None
        if a is not None:
            _DEF_RETIRED.append(a)   # earlier jobs of this step (and captured graphs) still use it
        a = _DEF["arena"] = torch.empty(max(2 * (a.numel() if a is not None else 0), need, 1 << 22),
                                        device=device, dtype=torch.float32)
        cur = 0
    _DEF["cursor"] = cur + need
    return a[cur:cur + need]


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, w_shape, stride, padding, dilation, out=None,
               beta: float = 0.0, splits: int = 0, key=None) -> torch.Tensor:
    """dW [Cout, Cin, KH, KW] (channels_last bf16) of conv2d(x, w) for the output gradient
    ``dy`` (NHWC bf16); ``out`` given: written (beta 0) or accumulated (beta 1) in place.
    ``key`` (the weight's data pointer, from a backward) allows a deferred split-K reduction."""
    Cout, Cin, KH, KW = w_shape
    N, _, IH, IW = x.shape
    _, _, OH, OW = dy.shape
    if not _fits(dy.numel(), x.numel()):
        # beyond the kernel's 32-bit offsets: MIOpen's weight gradient
        wz = torch.zeros((Cout, Cin, KH, KW), dtype=dy.dtype, device=dy.device)
        dw = torch.ops.aten.convolution_backward(dy, x, wz, None, list(_pair(stride)), list(_pair(padding)),
                                                 list(_pair(dilation)), False, [0, 0], 1,
                                                 [False, True, False])[1]
        if out is None:
            return dw.contiguous(memory_format=torch.channels_last)
        return out.add_(dw) if beta else out.copy_(dw)
    if not _cl(dy):
        dy = dy.contiguous(memory_format=torch.channels_last)
    if out is None:
        out = torch.empty((Cout, KH, KW, Cin), dtype=torch.bfloat16, device=x.device).permute(0, 3, 1, 2)
    assert tuple(out.shape) == (Cout, Cin, KH, KW) and out.stride(1) == 1 and out.stride(0) == KH * KW * Cin
    T = N * OH * OW
    ntiles = KH * KW * (-(-Cout // 128)) * (-(-Cin // 128))   # (narrow Cout / Cin: zero-padded tiles)
    if splits <= 0:
        splits = plan_splits(T, ntiles)
    splits = int(_lib.query("mx_conv_wgrad_splits", T, splits))
    slab, zero = _workspace(x.device, ntiles * splits * 128 * 128 if splits > 1 else 1)
    defer = 0
    # (only from inside an autograd backward, for a single-use FlatMaster weight: a direct
    # call never waits for a flush, and autograd must never sum an unfinished gradient)
    if splits > 1 and _deferrable(key):
        reg = _defer_slab(x.device, ntiles * splits * 128 * 128)
        if reg is not None:
            slab, defer = reg, 1
            _DEF["jobs"].append([reg.data_ptr(), out.data_ptr(), ntiles, splits, (-(-Cout // 128)) * (-(-Cin // 128)),
                                 -(-Cin // 128), KH * KW, Cin, 1 if beta else 0, Cout])
    d = _DESC_T()
    d[:20] = [dy.data_ptr(), x.data_ptr(), zero.data_ptr(), out.data_ptr(), slab.data_ptr(), defer,
            Cout, Cin, N, OH, OW, IH, IW, KH, KW, _sym(stride), _sym(padding), _sym(dilation), Cout, Cin]
    _lib.call("mx_conv_wgrad", d, float(beta), splits, _lib.stream())
    return out


def decomposed(KH: int, KW: int, stride, padding, dilation) -> bool:
    """Stride-decomposed dgrad (csrc/convwg.hip mx_conv_dgrad flags bit 1): stride > 1, no
    padding / dilation and a filter within s x s (1x1 stride 2, the 2x2 stride-2 transposed
    convolution) -- every input pixel takes at most one tap."""
    st, pd, dl = _sym(stride), _sym(padding), _sym(dilation)
    return st is not None and st > 1 and pd == 0 and dl == 1 and KH <= st and KW <= st


def conv_dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape, stride, padding, dilation, add=None,
               mask=None, bias=None, relu: bool = False, class_out: bool = False,
               add_class: bool = False) -> torch.Tensor:
    """dX [N, Cin, IH, IW] (channels_last bf16) of conv2d(x, w) for the output gradient
    ``dy``; ``w`` bf16 [Cout, Cin, KH, KW] (made channels_last if it is not).  In the same
    store (optional): ``+ bias`` ([Cin]), ``+ add`` (another gradient of X), ``relu`` and
    ``* (mask > 0)`` (X's ReLU; mask = X itself when X is a ReLU output); add / mask
    channels_last bf16 of X's shape.  With bias + relu this is conv_transpose2d's forward.
    A 1 x 1 stride-s filter (stride-decomposed, class_ok) reaches only the pixels
    (s i, s j): ``class_out`` returns just those, dX[:, :, ::s, ::s] as a compact
    [N, Cin, ceil(IH / s), ceil(IW / s)] tensor (no add / mask / bias / relu), and ``add_class``
    takes such a compact tensor as ``add`` (added to those pixels only)."""
    Cout, Cin, KH, KW = w.shape
    N, _, IH, IW = x_shape
    _, _, OH, OW = dy.shape
    if not _cl(dy):
        dy = dy.contiguous(memory_format=torch.channels_last)
    if not _cl(w):
        w = w.contiguous(memory_format=torch.channels_last)
    dec = decomposed(KH, KW, stride, padding, dilation)
    st = _sym(stride)
    if class_out or add_class:
        assert dec and KH == KW == 1, "class_out / add_class: a stride-decomposed 1 x 1 filter"
    cshape = (N, Cin, -(-IH // st), -(-IW // st))
    if class_out:
        assert add is None and mask is None and bias is None and not relu
        dx = torch.empty((N, cshape[2], cshape[3], Cin), dtype=torch.bfloat16, device=dy.device).permute(0, 3, 1, 2)
    else:
        dx = torch.empty((N, IH, IW, Cin), dtype=torch.bfloat16, device=dy.device).permute(0, 3, 1, 2)
    T = N * (-(-IH // st)) * (-(-IW // st)) if dec else N * IH * IW   # largest launch's pixels
    splits = dgrad_splits((T + 127) // 128 * -(-Cin // 128), (1 if dec else KH * KW) * -(-Cout // 64))
    slab, zero = _workspace(dy.device, splits * T * Cin if splits > 1 else 1)
    assert bias is None or (bias.dtype == torch.bfloat16 and bias.is_contiguous() and bias.numel() == Cin
                            and bias.data_ptr() % 8 == 0)
    for t, shp in ((add, cshape if add_class else (N, Cin, IH, IW)), (mask, (N, Cin, IH, IW))):
        assert t is None or (_cl(t) and tuple(t.shape) == shp and t.dtype == torch.bfloat16
                             and t.data_ptr() % 16 == 0), "dgrad add / mask: X's channels_last shape"
    assert not add_class or add is not None
    d = _DESC_T()
    d[:24] = [dy.data_ptr(), w.data_ptr(), zero.data_ptr(), dx.data_ptr(), _lib.ptr(add) or 0, _lib.ptr(mask) or 0,
              Cout, Cin, N, OH, OW, IH, IW, KH, KW, st, _sym(padding), _sym(dilation), Cout, Cin,
              splits, slab.data_ptr() if splits > 1 else 0, _lib.ptr(bias) or 0,
              int(relu) | (int(dec) << 1) | (int(class_out) << 2) | (int(add_class) << 3)]
    d[24] = _tickets(dy.device) if (splits > 1 and SPLIT_IN_KERNEL) else 0
    _lib.call("mx_conv_dgrad", d, _lib.stream())
    return dx


def class_ok(w: torch.Tensor, x_shape, stride, padding, dilation) -> bool:
    """conv_dgrad's class_out / add_class apply: the implicit-GEMM dgrad of a 1 x 1 filter
    with stride > 1 and no padding (stride-decomposed into a single parity class)."""
    return (tuple(w.shape[2:]) == (1, 1) and decomposed(1, 1, stride, padding, dilation)
            and dgrad_supported(w, x_shape, stride, padding, dilation))


DGRAD_MIN_TILES = 64


def dgrad_splits(tiles: int, nk: int) -> int:
    """Split-K of the input gradient (k_splits), the fp32 partials summed in order with the
    add / mask epilogue applied after."""
    return k_splits(tiles, nk)


# the kernels address x / dY / y / residual with 32-bit buffer offsets (csrc/convwg.hip:
# mx_conv_fwd / mx_conv_dgrad / mx_conv_wgrad reject larger tensors): bigger ones take MIOpen
_MAX_BYTES = 1 << 31


def _fits(*numels: int) -> bool:
    return all(2 * int(n) < _MAX_BYTES for n in numels)


def fwd_supported(x: torch.Tensor, w: torch.Tensor, b, residual, stride=1, padding=0, dilation=1,
                  res_up: bool = False) -> bool:
    """The implicit-GEMM forward: NHWC bf16, Cout a multiple of 64, Cin of 64, and at least
    FWD_MIN_TILES output tiles or a split reduction (any size unless SMALL_ON_MIOPEN).  ``res_up``: the
    residual is at half the output resolution, added nearest-upsampled."""
    # (Cout a multiple of 8: the narrow 1x1 heads -- RPN 16, mask logits 80 -- run zero-padded tiles)
    if not (FWD and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and w.dim() == 4 and cout_ok(w.shape[0]) and w.shape[1] % 64 == 0 and x.shape[1] == w.shape[1]
            and _cl(x) and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0
            and None not in (_sym(stride), _sym(padding), _sym(dilation))):
        return False
    if b is not None and not (b.dtype == torch.bfloat16 and b.is_contiguous() and b.numel() == w.shape[0]
                              and b.data_ptr() % 8 == 0):   # 8-B bias loads (4 channels per lane)
        return False
    st, pd, dl = _sym(stride), _sym(padding), _sym(dilation)
    N, _, IH, IW = x.shape
    OH = (IH + 2 * pd - dl * (w.shape[2] - 1) - 1) // st + 1
    OW = (IW + 2 * pd - dl * (w.shape[3] - 1) - 1) // st + 1
    rshape = (N, w.shape[0], OH // 2, OW // 2) if res_up else (N, w.shape[0], OH, OW)
    if res_up and (residual is None or OH % 2 or OW % 2):
        return False
    if OH <= 0 or OW <= 0 or not _fits(x.numel(), N * OH * OW * w.shape[0]):
        return False
    if residual is not None and not (residual.dtype == torch.bfloat16 and _cl(residual)
                                     and tuple(residual.shape) == rshape
                                     and residual.data_ptr() % 16 == 0):   # 16-B residual loads
        return False
    # 128 x 128 tiles, or 128 x 64 when Cout is an odd multiple of 64 (csrc/convwg.hip); fewer
    # than FWD_MIN_TILES tiles split the reduction (fwd_splits)
    tiles = (N * OH * OW + 127) // 128 * (w.shape[0] // 128 if w.shape[0] % 128 == 0 else -(-w.shape[0] // 64))
    if not SMALL_ON_MIOPEN:
        return True
    if w.shape[0] % 64:   # narrow Cout: no split-K (whole-tile partial planes)
        return tiles >= FWD_MIN_TILES
    return tiles >= FWD_MIN_TILES or fwd_splits(tiles, w.shape[2] * w.shape[3] * w.shape[1] // 64) > 1


# split-K below SPLIT_TILES output tiles (the chip holds 512 workgroups of the 128 x 128
# kernels: 256 CUs x 2) when the reduction is long (>= SPLIT_MIN_NK K-steps of 64): about
# SPLIT_WGS workgroups (rounded down: one more would start a second, mostly idle wave of
# workgroups -- 132 tiles x 4 splits = 528 ran 50 us where x 3 ran 39), at most SPLIT_MAX
# slices of >= 4 K-steps.  Short reductions lose
# more to the fp32 partial traffic than they gain (res3 3x3 at one image: 18 K-steps, 132
# tiles, 18.9 -> 26.9 us split in two); long ones on a part-empty chip gain (res5 3x3 at
# four images: 72 K-steps, 132 tiles, 60 -> 39 us in three) -- profiles/r4_s2/conv_split_ab_*.txt
SPLIT_TILES = 512       # 256 before the 32-bit gather (profiles/r4_s3/split_ab3_*: 512 best at 1 and 4 img)
SPLIT_WGS = 512
SPLIT_MAX = 8
SPLIT_MIN_NK = 32


# Convolutions with fewer than FWD_MIN_TILES / DGRAD_MIN_TILES output tiles once went to
# MIOpen unless their reduction was long enough to split.  MIOpen's split-K solvers for
# these (the coarse FPN levels and heads at small images) accumulate with atomics: two
# identical steps differed in the last bits even with cudnn.deterministic, so a graphed
# step could not reproduce the eager one (scripts/fpn_graph_probe.py).  Now every small
# convolution stays on the implicit GEMM, split when it has >= 8 K-steps (slices >= 4).
SMALL_ON_MIOPEN = False   # A/B switch (the former routing)

# Cout a multiple of 8 but not of 64 (the RPN head's 16 and the mask logits' 80 channels)
# runs zero-padded tiles; NARROW = False sends those convs back to MIOpen (A/B switch)
NARROW = True


def cout_ok(cout: int) -> bool:
    return cout % 64 == 0 or (NARROW and cout % 8 == 0)


def k_splits(tiles: int, nk: int) -> int:
    """Reduction slices of a conv forward / input gradient with ``tiles`` output tiles and
    ``nk`` 64-deep K-steps (res5 / P5 at one image: 9-36 tiles; at four images 66-132): the
    fp32 partials ([splits][pixels][channels]) are summed in order (deterministic) by the
    last-arriving slice of each tile (or the reduction kernel), which applies the epilogue."""
    small = tiles < FWD_MIN_TILES and not SMALL_ON_MIOPEN
    if tiles >= SPLIT_TILES or (nk < SPLIT_MIN_NK and not small):
        return 1
    return max(1, min(SPLIT_WGS // max(tiles, 1), nk // 4, SPLIT_MAX))


# the forward's own cap: at >= FWD_SPLIT_TILES tiles (128 x 64 ones included) an unsplit
# launch beat every split at the 1-img shapes (mask head 196 tiles: 28.5 us unsplit vs 35.4
# in two; res4 3x3 132 half tiles: 23.6 vs 25.0 -- profiles/r5_s1/conv_fwd_sweep_1img.txt)
FWD_SPLIT_TILES = 160


def fwd_splits(tiles: int, nk: int) -> int:
    return 1 if tiles >= FWD_SPLIT_TILES else k_splits(tiles, nk)


def conv_fwd(x: torch.Tensor, w: torch.Tensor, b=None, residual=None, relu: bool = False, stride=1, padding=0,
             dilation=1, res_up: bool = False, bn_stats: bool = False):
    """act(conv2d(x, w) + b (+ residual, nearest-upsampled 2x with ``res_up``)), NHWC bf16 in
    and out, one launch.  ``bn_stats``: returns (y, pre) where ``pre`` holds the per-64-row
    BatchNorm statistics of y from the epilogue (csrc/batchnorm.hip mx_bn_fwd's ``pre``), or
    None when the launch splits its reduction (the statistics pass then reads y)."""
    Cout, Cin, KH, KW = w.shape
    N, _, IH, IW = x.shape
    st, pd, dl = _sym(stride), _sym(padding), _sym(dilation)
    OH = (IH + 2 * pd - dl * (KH - 1) - 1) // st + 1
    OW = (IW + 2 * pd - dl * (KW - 1) - 1) // st + 1
    if not _cl(w):
        w = w.contiguous(memory_format=torch.channels_last)
    y = torch.empty((N, OH, OW, Cout), dtype=torch.bfloat16, device=x.device).permute(0, 3, 1, 2)
    T = N * OH * OW
    tiles = (T + 127) // 128 * (Cout // (128 if Cout % 128 == 0 else 64))
    half = Cout % 128 == 0 and tiles < FWD_HALF_TILES
    if half:
        tiles *= 2
    splits = 1 if Cout % 64 else fwd_splits(tiles, KH * KW * Cin // 64)
    slab, zero = _workspace(x.device, splits * T * Cout if splits > 1 else 1)
    d = _DESC_T()
    d[:24] = [x.data_ptr(), w.data_ptr(), zero.data_ptr(), y.data_ptr(), _lib.ptr(b) or 0,
              _lib.ptr(residual) or 0, Cin, Cout, N, OH, OW, IH, IW, KH, KW, st, pd, dl, Cout, Cin, int(relu),
              int(res_up), splits, slab.data_ptr() if splits > 1 else 0]
    d[24] = _tickets(x.device) if (splits > 1 and SPLIT_IN_KERNEL) else 0
    d[25] = int(half)
    pre = None
    if bn_stats and splits == 1 and Cout % 64 == 0:
        pre = torch.empty(_lib.query64("mx_bn_pre_size", T, Cout), dtype=torch.float32, device=x.device)
        d[26] = pre.data_ptr()
    _lib.call("mx_conv_fwd", d, _lib.stream())
    return (y, pre) if bn_stats else y


def dgrad_supported(w: torch.Tensor, x_shape, stride, padding=0, dilation=1) -> bool:
    """The implicit-GEMM input gradient where it beat MIOpen's backward-data solvers at the
    Mask R-CNN shapes (profiles/r3_s4/conv_dgrad_vs_miopen_graphed.txt): at least
    DGRAD_MIN_TILES 128 x 128 output tiles, or fewer with the reduction split (dgrad_splits;
    unsplit, a few tiles run long latency-bound K loops on a mostly idle chip -- res5 3x3
    65 vs 40 us), and stride 1, a stride-decomposed filter (1x1 stride 2: one GEMM over the
    pixels of one parity class) or at most 256 output channels (a strided 3x3's gathered dY
    has 3 of 4 rows zero, which costs MFMA time per K-step)."""
    # (the kernel also takes Cin = 64 -- half-padded 128-column tiles -- but at the ResNet res2
    # shapes that ran 1.4 ms per step vs MIOpen's 0.93 ms, profiles/r6/resnet50_census_cin64.txt)
    if not (DGRAD and cout_ok(w.shape[0]) and w.shape[1] % 128 == 0 and w.data_ptr() % 16 == 0):
        return False
    N, Cin, IH, IW = x_shape
    st = _sym(stride)
    if st is None or _sym(padding) is None or _sym(dilation) is None:
        return False
    pd, dl = _sym(padding), _sym(dilation)
    OH = (IH + 2 * pd - dl * (w.shape[2] - 1) - 1) // st + 1
    OW = (IW + 2 * pd - dl * (w.shape[3] - 1) - 1) // st + 1
    if OH <= 0 or OW <= 0 or not _fits(N * Cin * IH * IW, N * w.shape[0] * OH * OW):
        return False
    if decomposed(w.shape[2], w.shape[3], stride, padding, dilation):
        tiles = (N * (-(-IH // st)) * (-(-IW // st)) + 127) // 128 * -(-Cin // 128)
        return tiles >= DGRAD_MIN_TILES or dgrad_splits(tiles, -(-w.shape[0] // 64)) > 1 or not SMALL_ON_MIOPEN
    tiles = (N * IH * IW + 127) // 128 * -(-Cin // 128)
    nk = -(-(w.shape[2] * w.shape[3] * w.shape[0]) // 64)
    return ((tiles >= DGRAD_MIN_TILES or dgrad_splits(tiles, nk) > 1 or not SMALL_ON_MIOPEN)
            and (st == 1 or w.shape[0] <= 256))


class ConvWgFn(torch.autograd.Function):
    """conv2d(x, w): MIOpen forward, implicit-GEMM weight and input gradients."""

    @staticmethod
    def forward(ctx, x, w, stride, padding, dilation):
        ctx.conf = (list(_pair(stride)), list(_pair(padding)), list(_pair(dilation)))
        note_use(w)
        ctx.wkey = w.data_ptr()
        ctx.save_for_backward(x, w)
        return F.conv2d(x, w, None, stride, padding, dilation)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        st, pd, dl = ctx.conf
        if not _cl(g):
            g = g.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if dgrad_supported(w, tuple(x.shape), st, pd, dl):
                dx = conv_dgrad(g, w, tuple(x.shape), st, pd, dl)
            else:
                dx = torch.ops.aten.convolution_backward(g, x, w, None, st, pd, dl, False, [0, 0], 1,
                                                         [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            dw = conv_wgrad(g, x, tuple(w.shape), st, pd, dl, key=ctx.wkey)
        return dx, dw, None, None, None


def conv2d_wg(x, w, stride=1, padding=0, dilation=1):
    return ConvWgFn.apply(x, w, stride, padding, dilation)
