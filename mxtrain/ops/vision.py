"""Detection ops (``csrc/vision.hip``) + PyTorch references: multi-level RoIAlign
(fwd/bwd), batched bitmask NMS, anchor <-> ground-truth matching, box decode + clip.

Conventions: boxes are fp32 ``[x1, y1, x2, y2]`` in input-image pixels; RoIs are
``[R, 5]`` = (image index, box); FPN features are NHWC (channels_last) tensors.
"""
from __future__ import annotations

import ctypes
import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

BBOX_CLAMP = math.log(1000.0 / 16)


# ============================================================================ RoIAlign
def _levels_of(rois, n_levels, lvl_min, canon, canon_lvl):
    if n_levels == 1:
        return torch.zeros(rois.shape[0], dtype=torch.long, device=rois.device)
    w = (rois[:, 3] - rois[:, 1]).clamp(min=0)
    h = (rois[:, 4] - rois[:, 2]).clamp(min=0)
    k = torch.floor(canon_lvl + torch.log2(torch.sqrt(w * h) / canon + 1e-8))
    return (k.long() - lvl_min).clamp(0, n_levels - 1)


def _ref_roi_align(feats: Sequence[torch.Tensor], scales, rois, PH, PW, sr, aligned, lvl_min, canon, canon_lvl):
    """feats: NHWC tensors (any float dtype). Returns [R, PH, PW, C] fp32 (autograd-able)."""
    R = rois.shape[0]
    C = feats[0].shape[-1]
    out = feats[0].new_zeros((R, PH, PW, C), dtype=torch.float32)
    if R == 0:
        return out
    lv = _levels_of(rois, len(feats), lvl_min, canon, canon_lvl)
    off = 0.5 if aligned else 0.0
    iy = (torch.arange(PH, device=rois.device, dtype=torch.float32)[:, None] +
          (torch.arange(sr, device=rois.device, dtype=torch.float32)[None, :] + 0.5) / sr).reshape(-1)  # PH*sr
    ix = (torch.arange(PW, device=rois.device, dtype=torch.float32)[:, None] +
          (torch.arange(sr, device=rois.device, dtype=torch.float32)[None, :] + 0.5) / sr).reshape(-1)
    pieces = []
    for li, f in enumerate(feats):
        sel = (lv == li).nonzero().flatten()
        if sel.numel() == 0:
            continue
        r = rois[sel].float()
        s = scales[li]
        x0, y0 = r[:, 1] * s - off, r[:, 2] * s - off
        rw, rh = r[:, 3] * s - off - x0, r[:, 4] * s - off - y0
        if not aligned:
            rw, rh = rw.clamp(min=1.0), rh.clamp(min=1.0)
        ys = y0[:, None] + iy[None, :] * (rh / PH)[:, None]          # [n, PH*sr]
        xs = x0[:, None] + ix[None, :] * (rw / PW)[:, None]          # [n, PW*sr]
        B, H, W, _ = f.shape
        Y = ys[:, :, None].expand(-1, -1, xs.shape[1])
        X = xs[:, None, :].expand(-1, ys.shape[1], -1)
        valid = ~((Y < -1) | (Y > H) | (X < -1) | (X > W))
        Y = Y.clamp(min=0)
        X = X.clamp(min=0)
        yl = Y.floor().long()
        xl = X.floor().long()
        ytop = yl >= H - 1
        xtop = xl >= W - 1
        yl = torch.where(ytop, torch.full_like(yl, H - 1), yl)
        xl = torch.where(xtop, torch.full_like(xl, W - 1), xl)
        Y = torch.where(ytop, yl.float(), Y)
        X = torch.where(xtop, xl.float(), X)
        yh = torch.where(ytop, yl, yl + 1)
        xh = torch.where(xtop, xl, xl + 1)
        ly, lx = Y - yl, X - xl
        hy, hx = 1 - ly, 1 - lx
        bidx = r[:, 0].long()[:, None, None]
        ff = f.float()

        def g(yy, xx):
            return ff[bidx.expand_as(yy), yy, xx]                    # [n, PH*sr, PW*sr, C]
        v = (g(yl, xl) * (hy * hx)[..., None] + g(yl, xh) * (hy * lx)[..., None] +
             g(yh, xl) * (ly * hx)[..., None] + g(yh, xh) * (ly * lx)[..., None])
        v = v * valid[..., None]
        v = v.view(-1, PH, sr, PW, sr, C).mean(dim=(2, 4))
        pieces.append((sel, v))
    for sel, v in pieces:
        out = out.index_copy(0, sel, v)
    return out


def _ptr_array(ts, ctype=ctypes.c_void_p):
    arr = (ctype * 4)()
    for i, t in enumerate(ts):
        arr[i] = t.data_ptr() if t is not None else 0
    return arr


# the tiled backward (roi_align_bwd_tile_kernel) handles sr <= 2, C % 64 == 0, C <= 256; other
# shapes take the fp32-atomic one (roi_align_bwd_kernel).  Tests flip this to compare the two.
_TILED = True


_WS_CACHE = {}
_LAST_WS = None   # the last tiled-backward workspace (tests read its overflow word)


def _tiled_ws(shapes, B, items, C):
    """(int32 workspace entries, fp32 partial entries) of mx_roi_align_bwd_tiled."""
    key = (tuple(tuple(s) for s in shapes), B, items, C)
    v = _WS_CACHE.get(key)
    if v is None:
        n = len(shapes)
        H = (ctypes.c_int * 4)(*[s[1] for s in shapes] + [0] * (4 - n))
        W = (ctypes.c_int * 4)(*[s[2] for s in shapes] + [0] * (4 - n))
        fn = _lib.lib().mx_roi_align_bwd_tiled_ws
        fn.restype = ctypes.c_int64
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                       ctypes.POINTER(ctypes.c_int64)]
        part = ctypes.c_int64(0)
        nws = fn(ctypes.cast(H, ctypes.c_void_p), ctypes.cast(W, ctypes.c_void_p), n, B, items, C, ctypes.byref(part))
        v = _WS_CACHE[key] = (int(nws), int(part.value))
    return v


def tiled_overflow() -> int:
    """Overflow word of the last tiled RoIAlign backward (0 = every chunk was processed
    within the geometric bounds the workspace was sized for); synchronises."""
    if _LAST_WS is None:
        return 0
    ws, idx = _LAST_WS
    return int(ws[idx].item())


class RoIAlignFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rois, PH, PW, sr, aligned, lvl_min, canon, canon_lvl, scales, *feats):
        R = rois.shape[0]
        C = feats[0].shape[-1]
        ctx.meta = (PH, PW, sr, aligned, lvl_min, canon, canon_lvl, tuple(scales))
        ctx.shapes = [f.shape for f in feats]
        ctx.dtypes = [f.dtype for f in feats]
        ctx.save_for_backward(rois)
        fs = [f.contiguous() for f in feats]
        out = torch.empty((R, PH, PW, C), dtype=feats[0].dtype, device=rois.device)
        H = (ctypes.c_int * 4)(*[f.shape[1] for f in fs] + [0] * (4 - len(fs)))
        W = (ctypes.c_int * 4)(*[f.shape[2] for f in fs] + [0] * (4 - len(fs)))
        S = (ctypes.c_float * 4)(*list(scales) + [0.0] * (4 - len(fs)))
        _lib.call("mx_roi_align_fwd", ctypes.cast(_ptr_array(fs), ctypes.c_void_p), ctypes.cast(H, ctypes.c_void_p),
                  ctypes.cast(W, ctypes.c_void_p), ctypes.cast(S, ctypes.c_void_p), len(fs), lvl_min, float(canon),
                  canon_lvl, _lib.ptr(rois), R, C, PH, PW, sr, int(aligned), _lib.ptr(out), _lib.stream())
        return out

    @staticmethod
    def backward(ctx, dout):
        (rois,) = ctx.saved_tensors
        PH, PW, sr, aligned, lvl_min, canon, canon_lvl, scales = ctx.meta
        d = dout.contiguous().to(torch.bfloat16)
        n = len(ctx.shapes)
        C = ctx.shapes[0][-1]
        H = (ctypes.c_int * 4)(*[s[1] for s in ctx.shapes] + [0] * (4 - n))
        W = (ctypes.c_int * 4)(*[s[2] for s in ctx.shapes] + [0] * (4 - n))
        S = (ctypes.c_float * 4)(*list(scales) + [0.0] * (4 - n))
        R = rois.shape[0]
        if _TILED and sr <= 2 and C % 64 == 0 and C <= 256:
            # tiled, deterministic, float-atomics-free kernel straight into bf16 gradients
            B = ctx.shapes[0][0]
            grads = [torch.empty(s, dtype=torch.bfloat16, device=rois.device) for s in ctx.shapes]
            nws, npart = _tiled_ws(tuple(ctx.shapes), B, R * PH * PW, C)
            ws = torch.empty(nws, dtype=torch.int32, device=rois.device)
            part = torch.empty(npart, dtype=torch.float32, device=rois.device)
            _lib.call("mx_roi_align_bwd_tiled", ctypes.cast(_ptr_array(grads), ctypes.c_void_p),
                      ctypes.cast(H, ctypes.c_void_p), ctypes.cast(W, ctypes.c_void_p),
                      ctypes.cast(S, ctypes.c_void_p), n, lvl_min, float(canon), canon_lvl, B, _lib.ptr(rois), R, C,
                      PH, PW, sr, int(aligned), _lib.ptr(d), _lib.ptr(ws), _lib.ptr(part), _lib.stream())
            global _LAST_WS
            T = sum(B * (-(-s[1] // 8)) * (-(-s[2] // 8)) for s in ctx.shapes)
            _LAST_WS = (ws, R * PH * PW * 12 + 5 * T + 3)   # footprints, 5 tile arrays, overflow
            return (None,) * 9 + tuple(g if dt == torch.bfloat16 else g.to(dt) for g, dt in zip(grads, ctx.dtypes))
        grads = [torch.zeros(s, dtype=torch.float32, device=rois.device) for s in ctx.shapes]
        _lib.call("mx_roi_align_bwd", ctypes.cast(_ptr_array(grads), ctypes.c_void_p),
                  ctypes.cast(H, ctypes.c_void_p), ctypes.cast(W, ctypes.c_void_p), ctypes.cast(S, ctypes.c_void_p),
                  n, lvl_min, float(canon), canon_lvl, _lib.ptr(rois), rois.shape[0], ctx.shapes[0][-1], PH, PW, sr,
                  int(aligned), _lib.ptr(d), _lib.stream())
        return (None,) * 9 + tuple(g.to(dt) for g, dt in zip(grads, ctx.dtypes))


def roi_align(feats: List[torch.Tensor], rois: torch.Tensor, output_size: Tuple[int, int], scales: Sequence[float],
              sampling_ratio: int = 2, aligned: bool = True, lvl_min: int = 2, canon: float = 224.0,
              canon_lvl: int = 4) -> torch.Tensor:
    """Multi-level RoIAlign.  feats: NHWC [B, H, W, C] per level (P2..P5; a single level
    means no level assignment).  rois: fp32 [R, 5].  Returns [R, PH, PW, C] (NHWC)."""
    PH, PW = output_size
    rois = rois.float().contiguous()
    if _lib.use_hip(feats[0]):
        feats = [f if f.dtype == torch.bfloat16 else f.to(torch.bfloat16) for f in feats]
        return RoIAlignFn.apply(rois, PH, PW, sampling_ratio, aligned, lvl_min, canon, canon_lvl, list(scales),
                                *feats)
    return _ref_roi_align(feats, scales, rois, PH, PW, sampling_ratio, aligned, lvl_min, canon,
                          canon_lvl).to(feats[0].dtype)


# ============================================================================ box utils
def normalize_u8_nhwc(images: torch.Tensor, mean: Sequence[float], std: Sequence[float],
                      dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """(images - mean) / std of a uint8 NCHW RGB batch as a channels_last ``dtype`` tensor: one
    pass on the GPU (csrc/vision.hip normalize_u8_nhwc_kernel: uint8 in, bf16 NHWC out)
    instead of float / subtract / divide / layout-change / autocast-cast passes over fp32
    copies; the torch expression otherwise."""
    if (images.is_cuda and images.dtype == torch.uint8 and dtype == torch.bfloat16 and images.dim() == 4
            and images.shape[1] == 3 and images.is_contiguous() and (images.shape[2] * images.shape[3]) % 4 == 0
            and _lib.use_hip(images)):
        B, _, H, W = images.shape
        x = torch.empty(B, H, W, 3, dtype=dtype, device=images.device).permute(0, 3, 1, 2)
        _lib.call("mx_normalize_u8_nhwc", images.data_ptr(), x.data_ptr(), B, H, W,
                  ctypes.cast((ctypes.c_float * 3)(*[float(v) for v in mean]), ctypes.c_void_p),
                  ctypes.cast((ctypes.c_float * 3)(*[1.0 / float(v) for v in std]), ctypes.c_void_p),
                  _lib.stream())
        return x
    m = torch.tensor(list(mean), dtype=torch.float32, device=images.device).view(1, -1, 1, 1)
    sd = torch.tensor(list(std), dtype=torch.float32, device=images.device).view(1, -1, 1, 1)
    return ((images.float() - m) / sd).to(dtype).contiguous(memory_format=torch.channels_last)


def box_iou(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    area_a = (a[:, 2] - a[:, 0]).clamp(min=0) * (a[:, 3] - a[:, 1]).clamp(min=0)
    area_b = (b[:, 2] - b[:, 0]).clamp(min=0) * (b[:, 3] - b[:, 1]).clamp(min=0)
    lt = torch.max(a[:, None, :2], b[None, :, :2])
    rb = torch.min(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area_a[:, None] + area_b[None, :] - inter).clamp(min=1e-12)


# ============================================================================ NMS
def _ref_nms_one(boxes, thr, max_out):
    n = boxes.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.long)
    iou = box_iou(boxes.float().cpu(), boxes.float().cpu()).numpy()
    removed = np.zeros(n, dtype=bool)
    keep = []
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        if len(keep) >= max_out:
            break
        removed |= iou[i] > thr
    return torch.tensor(keep, dtype=torch.long)


def batched_nms_sorted(boxes: torch.Tensor, counts: Optional[torch.Tensor], thr: float, max_out: int,
                       raw: bool = False):
    """boxes [P, N, 4] sorted by descending score per problem (rows >= counts[p] ignored).
    Returns (keep [P, max_out] int64 row indices, -1 padded; nkeep [P]); ``raw``: the
    kernel's int32 tensors as they are (no conversion launches)."""
    P, N, _ = boxes.shape
    if _lib.use_hip(boxes) and N <= 4096:
        b = boxes.float().contiguous()
        cnt = counts.to(torch.int32).contiguous() if counts is not None else None
        nb = (N + 63) // 64 + 1   # mask words + the transposed diagonal word (mx_nms_workspace_words)
        ws = torch.empty(P * N * nb, dtype=torch.int64, device=boxes.device)
        keep = torch.empty(P, max_out, dtype=torch.int32, device=boxes.device)
        nk = torch.empty(P, dtype=torch.int32, device=boxes.device)
        _lib.call("mx_nms", _lib.ptr(b), _lib.ptr(cnt), P, N, float(thr), max_out, _lib.ptr(ws), _lib.ptr(keep),
                  _lib.ptr(nk), _lib.stream())
        return (keep, nk) if raw else (keep.long(), nk.long())
    keep = torch.full((P, max_out), -1, dtype=torch.long)
    nk = torch.zeros(P, dtype=torch.long)
    for p in range(P):
        n = int(counts[p]) if counts is not None else N
        k = _ref_nms_one(boxes[p, :n], thr, max_out)
        keep[p, :k.numel()] = k
        nk[p] = k.numel()
    return keep.to(boxes.device), nk.to(boxes.device)


def nms(boxes: torch.Tensor, scores: torch.Tensor, thr: float, max_out: Optional[int] = None) -> torch.Tensor:
    """Single-problem NMS; returns kept indices into boxes (score order)."""
    order = scores.argsort(descending=True)
    max_out = max_out or boxes.shape[0]
    keep, nk = batched_nms_sorted(boxes[order][None], None, thr, max_out)
    k = keep[0, : int(nk[0])]
    return order[k]


# ============================================================================ matching
def match_boxes(anchors: torch.Tensor, gt: torch.Tensor, gcount: torch.Tensor, low_quality: bool = True,
                int32: bool = False):
    """anchors [A, 4] (shared) or [B, A, 4]; gt [B, G, 4] (rows >= gcount[b] ignored).
    Returns (max_iou [B, A], argmax [B, A] (-1 if no gt), lowq [B, A] gt index forced by
    the low-quality rule or -1); ``int32``: the index tensors as the kernel writes them
    (GPU; no int64 conversion launches)."""
    per_image = anchors.dim() == 3
    B, G = gt.shape[0], gt.shape[1]
    A = anchors.shape[-2]
    if _lib.use_hip(anchors):
        an = anchors.float().contiguous()
        g = gt.float().contiguous()
        gc = gcount.to(torch.int32).contiguous()
        mi = torch.empty(B, A, dtype=torch.float32, device=anchors.device)
        am = torch.empty(B, A, dtype=torch.int32, device=anchors.device)
        gb = torch.empty(B, max(G, 1), dtype=torch.int32, device=anchors.device)
        lq = torch.empty(B, A, dtype=torch.int32, device=anchors.device) if low_quality else None
        _lib.call("mx_match", _lib.ptr(an), A, int(per_image), _lib.ptr(g), _lib.ptr(gc), B, G, _lib.ptr(mi),
                  _lib.ptr(am), _lib.ptr(gb), _lib.ptr(lq), _lib.stream())
        if int32:
            return mi, am, lq
        return mi, am.long(), (lq.long() if lq is not None else None)
    mis, ams, lqs = [], [], []
    for b in range(B):
        an = anchors[b] if per_image else anchors
        n = int(gcount[b])
        if n == 0:
            mis.append(torch.zeros(A, device=anchors.device))
            ams.append(torch.full((A,), -1, dtype=torch.long, device=anchors.device))
            lqs.append(torch.full((A,), -1, dtype=torch.long, device=anchors.device))
            continue
        iou = box_iou(an.float(), gt[b, :n].float())
        mi, am = iou.max(1)
        mis.append(mi)
        ams.append(am)
        best = iou.max(0).values
        hit = (iou >= best[None, :]) & (best[None, :] > 0)
        idx = torch.arange(n, device=anchors.device)[None, :].expand_as(hit)
        lq = torch.where(hit, idx, torch.full_like(idx, -1)).max(1).values
        lqs.append(lq)
    return torch.stack(mis), torch.stack(ams), (torch.stack(lqs) if low_quality else None)


# ============================================================================ encode/decode
def decode_boxes(ref: torch.Tensor, deltas: torch.Tensor, weights=(1.0, 1.0, 1.0, 1.0),
                 img_hw: Optional[torch.Tensor] = None, rows_per_img: int = 0) -> torch.Tensor:
    """ref [N, 4] (or [4] broadcast), deltas [N, 4] -> decoded (and clipped) boxes [N, 4]."""
    N = deltas.shape[0]
    wx, wy, ww, wh = weights
    if _lib.use_hip(deltas):
        r = ref.float().contiguous()
        d = deltas.float().contiguous()
        out = torch.empty(N, 4, dtype=torch.float32, device=deltas.device)
        hw = img_hw.float().contiguous() if img_hw is not None else None
        _lib.call("mx_decode_clip", _lib.ptr(r), _lib.ptr(d), N, int(r.dim() == 2 and r.shape[0] == N), wx, wy, ww,
                  wh, BBOX_CLAMP, _lib.ptr(hw), rows_per_img, _lib.ptr(out), _lib.stream())
        return out
    r = ref.float().reshape(-1, 4).expand(N, 4)
    d = deltas.float()
    w = r[:, 2] - r[:, 0]
    h = r[:, 3] - r[:, 1]
    cx = r[:, 0] + 0.5 * w
    cy = r[:, 1] + 0.5 * h
    dx, dy = d[:, 0] / wx, d[:, 1] / wy
    dw = (d[:, 2] / ww).clamp(max=BBOX_CLAMP)
    dh = (d[:, 3] / wh).clamp(max=BBOX_CLAMP)
    pcx, pcy = dx * w + cx, dy * h + cy
    pw, ph = torch.exp(dw) * w, torch.exp(dh) * h
    out = torch.stack([pcx - 0.5 * pw, pcy - 0.5 * ph, pcx + 0.5 * pw, pcy + 0.5 * ph], 1)
    if img_hw is not None:
        im = (torch.arange(N, device=out.device) // rows_per_img) if rows_per_img > 0 else torch.zeros(
            N, dtype=torch.long, device=out.device)
        H = img_hw.reshape(-1, 2)[im, 0].float()
        W = img_hw.reshape(-1, 2)[im, 1].float()
        out = torch.stack([torch.min(out[:, 0].clamp(min=0), W), torch.min(out[:, 1].clamp(min=0), H),
                           torch.min(out[:, 2].clamp(min=0), W), torch.min(out[:, 3].clamp(min=0), H)], 1)
    return out


def encode_boxes(ref: torch.Tensor, gt: torch.Tensor, weights=(1.0, 1.0, 1.0, 1.0)) -> torch.Tensor:
    """Box-regression targets of gt [N, 4] w.r.t. ref [N, 4] (fp32 [N, 4]); one launch on the
    GPU (csrc/dettarget.hip), the PyTorch formula below otherwise."""
    wx, wy, ww, wh = weights
    if (_lib.use_hip(gt) and gt.dim() == 2 and gt.shape[-1] == 4 and ref.dim() == 2 and ref.shape[-1] == 4
            and ref.shape[0] in (1, gt.shape[0]) and gt.shape[0] > 0):
        r = ref.float().contiguous()
        g = gt.float().contiguous()
        out = torch.empty(g.shape[0], 4, dtype=torch.float32, device=g.device)
        _lib.call("mx_encode_boxes", _lib.ptr(r), int(r.numel() == 4 and g.shape[0] != 1), _lib.ptr(g), g.shape[0],
                  float(wx), float(wy), float(ww), float(wh), _lib.ptr(out), _lib.stream())
        return out
    rw = (ref[:, 2] - ref[:, 0]).clamp(min=1e-6)
    rh = (ref[:, 3] - ref[:, 1]).clamp(min=1e-6)
    rcx = ref[:, 0] + 0.5 * rw
    rcy = ref[:, 1] + 0.5 * rh
    gw = (gt[:, 2] - gt[:, 0]).clamp(min=1e-6)
    gh = (gt[:, 3] - gt[:, 1]).clamp(min=1e-6)
    gcx = gt[:, 0] + 0.5 * gw
    gcy = gt[:, 1] + 0.5 * gh
    return torch.stack([wx * (gcx - rcx) / rw, wy * (gcy - rcy) / rh, ww * torch.log(gw / rw),
                        wh * torch.log(gh / rh)], 1)


# ============================================================================ mask targets
def crop_resize_masks(masks: torch.Tensor, boxes: torch.Tensor, gidx: torch.Tensor, M: int = 28) -> torch.Tensor:
    """masks uint8 [G, H, W]; boxes [R, 4] image px; gidx [R] -> fp32 [R, M, M] bilinear
    crops (pixel-center aligned), the Mask R-CNN mask-head targets."""
    R = boxes.shape[0]
    G, H, W = masks.shape
    if _lib.use_hip(masks):
        out = torch.empty(R, M, M, dtype=torch.float32, device=masks.device)
        _lib.call("mx_crop_resize_masks", _lib.ptr(masks.contiguous()), H, W, _lib.ptr(boxes.float().contiguous()),
                  _lib.ptr(gidx.to(torch.int32).contiguous()), R, M, _lib.ptr(out), _lib.stream())
        return out
    if R == 0:
        return torch.zeros(0, M, M)
    b = boxes.float()
    t = (torch.arange(M, dtype=torch.float32, device=boxes.device) + 0.5) / M
    ys = b[:, 1:2] + t[None] * (b[:, 3:4] - b[:, 1:2]) - 0.5      # [R, M]
    xs = b[:, 0:1] + t[None] * (b[:, 2:3] - b[:, 0:1]) - 0.5
    Y = ys[:, :, None].expand(-1, -1, M)
    X = xs[:, None, :].expand(-1, M, -1)
    valid = ~((Y < -1) | (Y > H) | (X < -1) | (X > W))
    Y, X = Y.clamp(min=0), X.clamp(min=0)
    yl, xl = Y.floor().long(), X.floor().long()
    ytop, xtop = yl >= H - 1, xl >= W - 1
    yl = torch.where(ytop, torch.full_like(yl, H - 1), yl)
    xl = torch.where(xtop, torch.full_like(xl, W - 1), xl)
    Y = torch.where(ytop, yl.float(), Y)
    X = torch.where(xtop, xl.float(), X)
    yh = torch.where(ytop, yl, yl + 1)
    xh = torch.where(xtop, xl, xl + 1)
    ly, lx = Y - yl, X - xl
    m = masks.float()
    gi = gidx.long()[:, None, None].expand_as(yl)
    v = ((1 - ly) * ((1 - lx) * m[gi, yl, xl] + lx * m[gi, yl, xh]) +
         ly * ((1 - lx) * m[gi, yh, xl] + lx * m[gi, yh, xh]))
    return v * valid


def crop_resize_mask_crops(flat: torch.Tensor, table: torch.Tensor, H: int, W: int, boxes: torch.Tensor,
                           gidx: torch.Tensor, M: int = 28) -> torch.Tensor:
    """``crop_resize_masks`` over packed per-instance crops (data/coco.py ``mask_crop``):
    flat uint8 crops, table int32 [G, 5] = (offset, x0, y0, w, h), H x W the padded
    image the full masks would cover.  Same result as unpacking to full masks."""
    R = boxes.shape[0]
    if _lib.use_hip(boxes):
        out = torch.empty(R, M, M, dtype=torch.float32, device=boxes.device)
        if flat.numel() == 0:
            flat = torch.zeros(1, dtype=torch.uint8, device=boxes.device)
        _lib.call("mx_crop_resize_mask_crops", _lib.ptr(flat), _lib.ptr(table.to(torch.int32).contiguous()), H, W,
                  _lib.ptr(boxes.float().contiguous()), _lib.ptr(gidx.to(torch.int32).contiguous()), R, M,
                  _lib.ptr(out), _lib.stream())
        return out
    from ..data.coco import unpack_mask_crops
    full = unpack_mask_crops(flat, table.reshape(1, -1, 5), H, W)[0].to(boxes.device)
    return crop_resize_masks(full, boxes, gidx, M)


# ------------------------------------------------------------------ RPN level top-k + decode
_TK_CACHE = {}


def nms_merge_topk(keep: torch.Tensor, scores: torch.Tensor, boxes: torch.Tensor, B: int, L: int, top: int):
    """The proposal tail after a batched NMS of B x L score-sorted problems: each image's
    top ``top`` survivors over its L levels, as (boxes [B, top, 4], scores [B, top]); padded
    survivors score -inf with the problem's first box.  ``keep`` int32 [B L, pre] (the
    kernel's raw NMS output, ``batched_nms_sorted(..., raw=True)``); one launch
    (csrc/vision.hip merge_keep_topk_kernel)."""
    P, pre = keep.shape
    if (_lib.use_hip(keep) and keep.dtype == torch.int32 and scores.dtype == torch.float32
            and boxes.dtype == torch.float32 and L * pre <= 16384 and top <= L * pre and P == B * L
            # (the kernel indexes scores / boxes with keep's row length: NMS inputs of
            # exactly [B L, pre]; any other width takes the gather path)
            and tuple(scores.shape) == tuple(keep.shape) and tuple(boxes.shape[:2]) == tuple(keep.shape)):
        k, sc, bx = keep.contiguous(), scores.contiguous(), boxes.contiguous()
        ov = torch.empty(B, top, dtype=torch.float32, device=keep.device)
        ob = torch.empty(B, top, 4, dtype=torch.float32, device=keep.device)
        _lib.call("mx_merge_keep_topk", _lib.ptr(k), _lib.ptr(sc), _lib.ptr(bx), B, L, pre, top, _lib.ptr(ov),
                  _lib.ptr(ob), _lib.stream())
        return ob, ov
    keep = keep.long()
    valid = keep >= 0
    ki = keep.clamp(min=0)
    kb = torch.gather(boxes, 1, ki[..., None].expand(-1, -1, 4)).view(B, L * pre, 4)
    ks = torch.where(valid, torch.gather(scores, 1, ki), torch.full_like(scores, -float("inf")))
    s, i = merge_sorted_topk(ks.view(B, L, pre), top)
    return torch.gather(kb, 1, i[..., None].expand(-1, -1, 4)), s


def merge_sorted_topk(ks: torch.Tensor, top: int):
    """topk_rows(ks.view(B, L * pre), top) for ks [B, L, pre] whose L lists are each sorted
    non-increasing (the per-level NMS survivors): one rank-by-binary-search pass
    (csrc/vision.hip merge_topk_kernel) instead of a radix select + sort."""
    B, L, pre = ks.shape
    if _lib.use_hip(ks) and ks.dtype == torch.float32 and L * pre <= 16384 and top <= L * pre:
        k = ks.contiguous()
        ov = torch.empty(B, top, dtype=torch.float32, device=ks.device)
        oi = torch.empty(B, top, dtype=torch.int64, device=ks.device)
        _lib.call("mx_merge_sorted_topk", _lib.ptr(k), B, L, pre, top, _lib.ptr(ov), _lib.ptr(oi), _lib.stream())
        return ov, oi
    return topk_rows(ks.reshape(B, L * pre), top)


def topk_rows(x: torch.Tensor, k: int, largest: bool = True):
    """(values, int64 indices) of the k largest / smallest entries of each row of a 2-D
    fp32 tensor, sorted, ties by lower index -- torch.topk(x, k, dim=1, largest) semantics
    in ONE launch (csrc/vision.hip topk_rows_kernel; capture-safe).  One workgroup per row
    suits rows up to ~32k entries (the proposal / RoI selections); longer rows (the ~270k RPN
    anchors) take two launches over <= 32k chunks; k > 2048, other dtypes / dims and CPU
    tensors go through torch.topk."""
    if (not _lib.use_hip(x) or x.dim() != 2 or x.dtype != torch.float32 or x.stride(1) != 1
            or k < 1 or k > x.shape[1] or k > 2048 or x.shape[0] == 0):
        return x.topk(k, dim=1, largest=largest)
    R, n = x.shape
    if n > 32768:
        # long rows (the ~270k RPN anchors of the sampling): the k best of each <= 32k chunk,
        # then the k best of those candidates -- two launches instead of torch.topk's radix
        # passes + device merge sort (~215 us per 1-img step).  Chunks are in index order and
        # each chunk's ties go to the lower index, so the merged ties do too.
        # chunk count ~ sqrt(n / k): both stages then scan rows of similar length (one
        # workgroup per row), each <= 32k
        nc = max(-(-n // 32768), min(int(math.sqrt(n / k)) + 1, 32768 // k))
        c = -(-n // nc)
        while nc > 1 and n - (nc - 1) * c < k:   # every chunk, the ragged last one too, >= k long
            nc -= 1
            c = -(-n // nc)
        if k > c or c > 32768 or nc * k > 32768:
            return x.topk(k, dim=1, largest=largest)
        cv = torch.empty((R * nc, k), dtype=torch.float32, device=x.device)
        ci = torch.empty((R * nc, k), dtype=torch.int64, device=x.device)
        ov = torch.empty((R, k), dtype=torch.float32, device=x.device)
        oi = torch.empty((R, k), dtype=torch.int64, device=x.device)
        _lib.call("mx_topk_rows_long", x.data_ptr(), R, n, x.stride(0), nc, c, k, int(largest), cv.data_ptr(),
                  ci.data_ptr(), ov.data_ptr(), oi.data_ptr(), _lib.stream())
        return ov, oi
    ov = torch.empty((R, k), dtype=torch.float32, device=x.device)
    oi = torch.empty((R, k), dtype=torch.int64, device=x.device)
    _lib.call("mx_topk_rows", x.data_ptr(), R, n, x.stride(0), k, int(largest), ov.data_ptr(), oi.data_ptr(),
              _lib.stream())
    return ov, oi


def _level_topk_decode_ref(logits_lv, deltas_lv, anchors_lv, img_hw, k):
    B = logits_lv[0].shape[0]
    boxes, scores, counts = [], [], []
    for lg, dl, an in zip(logits_lv, deltas_lv, anchors_lv):
        kk = min(k, lg.shape[1])
        sc, idx = lg.float().topk(kk, dim=1)                                 # sorted desc
        d = torch.gather(dl.float(), 1, idx[..., None].expand(-1, -1, 4))
        ref = an[idx.reshape(-1)]
        bx = decode_boxes(ref, d.reshape(-1, 4), (1.0, 1.0, 1.0, 1.0), img_hw, rows_per_img=kk).view(B, kk, 4)
        if kk < k:
            bx = torch.nn.functional.pad(bx, (0, 0, 0, k - kk))
            sc = torch.nn.functional.pad(sc, (0, k - kk), value=-float("inf"))
        boxes.append(bx)
        scores.append(sc)
        counts.append(kk)
    return torch.stack(boxes, 1), torch.stack(scores, 1), counts


def level_topk_decode(logits_lv: Sequence[torch.Tensor], deltas_lv: Sequence[torch.Tensor],
                      anchors_lv: Sequence[torch.Tensor], img_hw: torch.Tensor, k: int):
    """Per (image, level): the k highest objectness logits (sorted; ties -> lower anchor
    index), their anchors decoded with the level's deltas (weights 1, clamp, clipped to the
    image).  logits [B, n_l], deltas [B, n_l, 4], anchors [n_l, 4]; returns boxes
    [B, L, k, 4], scores [B, L, k] (-inf padded past n_l) and counts [min(k, n_l)].
    On the GPU: 6 launches for every row of the step (csrc/vision.hip tk_*)."""
    L = len(logits_lv)
    B = logits_lv[0].shape[0]
    lg0 = logits_lv[0]
    ok = (_lib.use_hip(lg0) and k <= 2048 and B * L <= _lib.query("mx_topk_max_rows")
          and all(t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1 for t in logits_lv)
          and all(t.dtype == torch.bfloat16 and t.dim() == 3 and t.stride(2) == 1 and t.stride(1) == 4
                  for t in deltas_lv)
          and all(t.dtype == torch.float32 and t.is_contiguous() for t in anchors_lv))
    if not ok:
        return _level_topk_decode_ref(logits_lv, deltas_lv, anchors_lv, img_hw, k)
    dev = lg0.device
    R = B * L
    rows = []
    for b in range(B):
        for lg, dl, an in zip(logits_lv, deltas_lv, anchors_lv):
            n = lg.shape[1]
            # (rows may be views of the flat all-level tensors: row stride, not n)
            rows += [lg.data_ptr() + 2 * b * lg.stride(0), dl.data_ptr() + 2 * b * dl.stride(0), an.data_ptr(), n, b, 0]
    chunk = _lib.query("mx_topk_chunk")
    nchunks = sum((lg.shape[1] + chunk - 1) // chunk for lg in logits_lv) * B
    key = (str(dev), R)
    bufs = _TK_CACHE.get(key)
    if bufs is None or bufs[2].numel() < 2 * nchunks:
        maxr = _lib.query("mx_topk_max_rows")
        tables = torch.empty(maxr * 6 * 8 + (maxr + 1) * 4, dtype=torch.uint8, device=dev)
        hist = torch.zeros(2, R, 256, dtype=torch.int32, device=dev)      # zero between calls
        bcnt = torch.empty(2 * max(nchunks, 1), dtype=torch.int32, device=dev)
        cand = torch.empty(R * 2048 * 2, dtype=torch.int32, device=dev)
        bufs = _TK_CACHE[key] = (tables, hist, bcnt, cand)
    tables, hist, bcnt, cand = bufs
    boxes = torch.empty(B, L, k, 4, dtype=torch.float32, device=dev)
    scores = torch.empty(B, L, k, dtype=torch.float32, device=dev)
    hw = img_hw.float().contiguous()
    arr = (ctypes.c_int64 * len(rows))(*rows)
    _lib.call("mx_level_topk_decode", ctypes.addressof(arr), R, k, _lib.ptr(hw), float(BBOX_CLAMP),
              _lib.ptr(tables), _lib.ptr(hist[0]), _lib.ptr(hist[1]), _lib.ptr(bcnt), bcnt.numel() // 2,
              _lib.ptr(cand), _lib.ptr(boxes), _lib.ptr(scores), _lib.stream())
    return boxes, scores, [min(k, lg.shape[1]) for lg in logits_lv]
