"""COCO-style bbox / segm AP without pycocotools (not installed on the node).

Same definition as COCOeval for the "all areas, maxDets=100" summary: per category,
detections sorted by score are greedily matched to unmatched ground truth at each IoU
threshold 0.50:0.05:0.95; precision is made monotone and sampled at 101 recall points;
AP is averaged over thresholds and over categories that have ground truth.
Reports AP, AP50, AP75 (what tensorpack writes into stats.json as
``mAP(bbox)/IoU=0.5:0.95`` etc.).
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

IOU_THRS = np.linspace(0.5, 0.95, 10)
REC_THRS = np.linspace(0.0, 1.0, 101)


def box_iou_np(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    if len(a) == 0 or len(b) == 0:
        return np.zeros((len(a), len(b)))
    lt = np.maximum(a[:, None, :2], b[None, :, :2])
    rb = np.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = np.clip(rb - lt, 0, None)
    inter = wh[..., 0] * wh[..., 1]
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    ab = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / np.maximum(aa[:, None] + ab[None] - inter, 1e-12)


def mask_iou_np(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    if len(a) == 0 or len(b) == 0:
        return np.zeros((len(a), len(b)))
    af = a.reshape(len(a), -1).astype(np.float32)
    bf = b.reshape(len(b), -1).astype(np.float32)
    inter = af @ bf.T
    return inter / np.maximum(af.sum(1)[:, None] + bf.sum(1)[None] - inter, 1e-12)


def evaluate(dets: List[dict], gts: List[dict], iou_type: str = "bbox") -> Dict[str, float]:
    """dets: [{image_id, category, score, box (x1y1x2y2) | mask (HxW bool)}];
    gts: [{image_id, category, box | mask}]."""
    key = "box" if iou_type == "bbox" else "mask"
    cats = sorted({g["category"] for g in gts})
    by_ic_g: Dict = {}
    for g in gts:
        by_ic_g.setdefault((g["image_id"], g["category"]), []).append(g[key])
    by_ic_d: Dict = {}
    for d in dets:
        by_ic_d.setdefault((d["image_id"], d["category"]), []).append((d["score"], d[key]))
    iou_fn = box_iou_np if iou_type == "bbox" else mask_iou_np
    aps = np.full((len(IOU_THRS), len(cats)), np.nan)
    for ci, c in enumerate(cats):
        scores, matches = [], [[] for _ in IOU_THRS]
        npos = 0
        images = {i for (i, cc) in list(by_ic_g) + list(by_ic_d) if cc == c}
        for im in images:
            g = by_ic_g.get((im, c), [])
            d = sorted(by_ic_d.get((im, c), []), key=lambda x: -x[0])[:100]
            npos += len(g)
            if not d:
                continue
            ious = iou_fn(np.stack([x[1] for x in d]), np.stack(g)) if g else np.zeros((len(d), 0))
            for ti, t in enumerate(IOU_THRS):
                used = np.zeros(len(g), dtype=bool)
                for di in range(len(d)):
                    best, bj = t, -1
                    for gj in range(len(g)):
                        if not used[gj] and ious[di, gj] >= best:
                            best, bj = ious[di, gj], gj
                    if bj >= 0:
                        used[bj] = True
                    matches[ti].append(bj >= 0)
            scores += [x[0] for x in d]
        if npos == 0:
            continue
        order = np.argsort(-np.asarray(scores), kind="mergesort")
        for ti in range(len(IOU_THRS)):
            tp = np.asarray(matches[ti], dtype=np.float64)[order] if scores else np.zeros(0)
            ctp = np.cumsum(tp)
            cfp = np.cumsum(1 - tp)
            rec = ctp / npos
            prec = ctp / np.maximum(ctp + cfp, 1e-12)
            for k in range(len(prec) - 2, -1, -1):
                prec[k] = max(prec[k], prec[k + 1])
            q = np.zeros(len(REC_THRS))
            inds = np.searchsorted(rec, REC_THRS, side="left")
            for ri, pi in enumerate(inds):
                if pi < len(prec):
                    q[ri] = prec[pi]
            aps[ti, ci] = q.mean()
    def m(x):
        x = x[~np.isnan(x)]
        return float(x.mean()) if x.size else 0.0
    return {"AP": m(aps), "AP50": m(aps[0]), "AP75": m(aps[5])}
