"""Fused Mask R-CNN losses (``csrc/detloss.hip``): RPN objectness + box, Fast R-CNN
classification + box, mask BCE -- each one autograd node (forward: partial sums +
finalize, backward: one gradient launch) instead of ~25 torch launches.  CPU tensors go
through the plain torch formulas (the reference definitions, models/maskrcnn.py)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def huber(x: torch.Tensor, delta: float) -> torch.Tensor:
    a = x.abs()
    return torch.where(a < delta, 0.5 * x * x, delta * (a - 0.5 * delta))


def _scratch(dev):
    return (torch.empty(4 * _lib.query("mx_detloss_max_blocks"), dtype=torch.float32, device=dev),
            torch.empty(4, dtype=torch.float32, device=dev))


def _gptr(g):
    return _lib.ptr(g.float().contiguous()) if g is not None else None


# ------------------------------------------------------------------------------ RPN
def rpn_loss_ref(logits, deltas, enc, sel_pos, sel_neg, box_norm):
    sel = sel_pos | sel_neg
    nsel = sel.sum().clamp(min=1).float()
    cls = (F.binary_cross_entropy_with_logits(logits.float(), sel_pos.float(), reduction="none") * sel).sum() / nsel
    box = (huber(deltas.float() - enc, 1.0 / 9).sum(-1) * sel_pos).sum() / box_norm
    return cls, box


class _RPNLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, deltas, enc, pos, neg, box_norm):
        partial, out = _scratch(logits.device)
        _lib.call("mx_rpn_loss_fwd", _lib.ptr(logits), _lib.ptr(deltas), _lib.ptr(enc), _lib.ptr(pos), _lib.ptr(neg),
                  logits.numel(), float(box_norm), _lib.ptr(partial), _lib.ptr(out), _lib.stream())
        ctx.save_for_backward(logits, deltas, enc, pos, neg, out)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_cls, g_box):
        logits, deltas, enc, pos, neg, out = ctx.saved_tensors
        dl, dd = torch.empty_like(logits), torch.empty_like(deltas)
        gc, gb = (g_cls.float().contiguous() if g_cls is not None else None,
                  g_box.float().contiguous() if g_box is not None else None)
        _lib.call("mx_rpn_loss_bwd", _lib.ptr(logits), _lib.ptr(deltas), _lib.ptr(enc), _lib.ptr(pos), _lib.ptr(neg),
                  logits.numel(), _lib.ptr(out), _lib.ptr(gc), _lib.ptr(gb), _lib.ptr(dl), _lib.ptr(dd), _lib.stream())
        return dl, dd, None, None, None, None


def rpn_loss(logits, deltas, enc, sel_pos, sel_neg, box_norm):
    """logits [B, A], deltas [B, A, 4] (bf16 on the GPU), enc fp32 [B, A, 4] targets,
    sel_pos / sel_neg bool [B, A]."""
    if (_lib.use_hip(logits) and logits.dtype == torch.bfloat16 and deltas.dtype == torch.bfloat16
            and logits.is_contiguous() and deltas.is_contiguous()):
        return _RPNLoss.apply(logits, deltas, enc.float().contiguous(), sel_pos.contiguous(), sel_neg.contiguous(),
                              box_norm)
    return rpn_loss_ref(logits, deltas, enc, sel_pos, sel_neg, box_norm)


# ------------------------------------------------------------------------------ Fast R-CNN
def frcnn_loss_ref(cls_logits, box_deltas, labels, tgt, fg, box_norm):
    cls_logits = cls_logits.float()
    box_deltas = box_deltas.float().view(cls_logits.shape[0], -1, 4)
    cls = F.cross_entropy(cls_logits, labels)
    pick = torch.gather(box_deltas, 1, labels[:, None, None].expand(-1, 1, 4)).squeeze(1)
    box = (huber(pick - tgt, 1.0).sum(-1) * fg).sum() / box_norm
    return cls, box


class _FRCNNLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, deltas, labels, tgt, fg, box_norm):
        partial, out = _scratch(logits.device)
        N, C = logits.shape
        _lib.call("mx_frcnn_loss_fwd", _lib.ptr(logits), _lib.ptr(deltas), _lib.ptr(labels), _lib.ptr(tgt),
                  _lib.ptr(fg), N, C, float(box_norm), _lib.ptr(partial), _lib.ptr(out), _lib.stream())
        ctx.save_for_backward(logits, deltas, labels, tgt, fg, out)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_cls, g_box):
        logits, deltas, labels, tgt, fg, out = ctx.saved_tensors
        N, C = logits.shape
        dl, dd = torch.empty_like(logits), torch.empty_like(deltas)
        gc, gb = (g_cls.float().contiguous() if g_cls is not None else None,
                  g_box.float().contiguous() if g_box is not None else None)
        _lib.call("mx_frcnn_loss_bwd", _lib.ptr(logits), _lib.ptr(deltas), _lib.ptr(labels), _lib.ptr(tgt),
                  _lib.ptr(fg), N, C, _lib.ptr(out), _lib.ptr(gc), _lib.ptr(gb), _lib.ptr(dl), _lib.ptr(dd),
                  _lib.stream())
        return dl, dd, None, None, None, None


def frcnn_loss(cls_logits, box_deltas, labels, tgt, fg, box_norm):
    """cls_logits [N, C], box_deltas [N, C * 4] (bf16 on the GPU), labels int64 [N],
    tgt fp32 [N, 4], fg bool [N]."""
    if (_lib.use_hip(cls_logits) and cls_logits.dtype == torch.bfloat16 and box_deltas.dtype == torch.bfloat16
            and cls_logits.is_contiguous() and box_deltas.is_contiguous()):
        return _FRCNNLoss.apply(cls_logits, box_deltas, labels.long().contiguous(), tgt.float().contiguous(),
                                fg.contiguous(), box_norm)
    return frcnn_loss_ref(cls_logits, box_deltas, labels, tgt, fg, box_norm)


# ------------------------------------------------------------------------------ mask
def mask_loss_ref(ml, labels, target, valid):
    """ml [R, K, H, W] logits, labels [R] in 1..K (0 = background row), target [R, H, W]
    (>= 0.5 = foreground), valid [R] float."""
    g = torch.gather(ml, 1, (labels - 1).clamp(min=0)[:, None, None, None].expand(-1, 1, *ml.shape[2:]))
    g = g.squeeze(1).float()
    bce = F.binary_cross_entropy_with_logits(g, (target >= 0.5).float(), reduction="none").mean(dim=(1, 2))
    return (bce * valid).sum() / valid.sum().clamp(min=1)


class _MaskLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ml, labels, target, valid):
        partial, out = _scratch(ml.device)
        R, K, H, W = ml.shape
        _lib.call("mx_mask_loss_fwd", _lib.ptr(ml), _lib.ptr(labels), _lib.ptr(target), _lib.ptr(valid), R, H * W, K,
                  _lib.ptr(partial), _lib.ptr(out), _lib.stream())
        ctx.save_for_backward(ml, labels, target, valid, out)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        ml, labels, target, valid, out = ctx.saved_tensors
        R, K, H, W = ml.shape
        dml = torch.empty_like(ml, memory_format=torch.channels_last)
        _lib.call("mx_mask_loss_bwd", _lib.ptr(ml), _lib.ptr(labels), _lib.ptr(target), _lib.ptr(valid), R, H * W, K,
                  _lib.ptr(out), _lib.ptr(g.float().contiguous()), _lib.ptr(dml), _lib.stream())
        return dml, None, None, None


def mask_loss(ml, labels, target, valid):
    if (_lib.use_hip(ml) and ml.dtype == torch.bfloat16 and ml.is_contiguous(memory_format=torch.channels_last)
            and ml.shape[1] % 8 == 0):
        return _MaskLoss.apply(ml, labels.long().contiguous(), target.float().contiguous(), valid.float().contiguous())
    return mask_loss_ref(ml, labels, target, valid)
