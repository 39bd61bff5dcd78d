"""COCO-style bbox / segm evaluation without pycocotools (not installed on the node).

Follows COCOeval's definition (evaluateImg / accumulate / summarize) for the standard
12-number summary that tensorpack's ``stats.json`` is derived from:

* per (image, category), detections sorted by score and cut to maxDets are greedily
  matched to ground truth at each IoU threshold 0.50:0.05:0.95, with ground truth that
  is not usable preferring usable ground truth first;
* for an area range, ground truth outside the range is *ignored* (a detection matched to
  it neither helps nor hurts) and so is an unmatched detection outside the range;
* precision is made monotone and sampled at 101 recall points, recall is the final
  recall of the sorted detection list; categories without usable ground truth count as
  missing (excluded from the means).

Area ranges (closed, as COCOeval): all [0, 1e10], small [0, 32^2], medium [32^2, 96^2],
large [96^2, 1e10].
GT area is the annotation's ``area`` when given (COCO: the segment area, used for both
bbox and segm), otherwise box area / mask pixel count.

Returns AP, AP50, AP75, APs, APm, APl, AR1, AR10, AR100, ARs, ARm, ARl.
tensorpack writes the first six as ``mAP(bbox)/IoU=0.5:0.95``, ``.../IoU=0.5``,
``.../IoU=0.75``, ``.../small``, ``.../medium``, ``.../large``
(reference: containers/tensorpack-maskrcnn notebooks read ``stats.json``).  Parity with
pycocotools is unpinned (not importable here); tests pin hand-checked cases.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

IOU_THRS = np.linspace(0.5, 0.95, 10)
REC_THRS = np.linspace(0.0, 1.0, 101)
AREA_RNG = {"all": (0.0, 1e10), "small": (0.0, 32.0 ** 2), "medium": (32.0 ** 2, 96.0 ** 2),
            "large": (96.0 ** 2, 1e10)}
MAX_DETS = (1, 10, 100)


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


def _area(x: np.ndarray, iou_type: str) -> float:
    if iou_type == "bbox":
        return float(max(x[2] - x[0], 0) * max(x[3] - x[1], 0))
    return float(np.count_nonzero(x))


def _match_image(d_area, g_area, ious, rng, max_det):
    """COCOeval.evaluateImg for one (image, category, area range, maxDet):
    -> (dt_matched [T, D], dt_ignored [T, D], n_usable_gt).  dets already score-sorted."""
    lo, hi = rng
    g_ign = np.array([not (lo <= a <= hi) for a in g_area], dtype=bool)
    gorder = np.argsort(g_ign, kind="mergesort")       # usable ground truth first
    g_ign_s = g_ign[gorder]
    nd = min(len(d_area), max_det)
    T = len(IOU_THRS)
    dtm = np.zeros((T, nd), dtype=bool)
    dt_ig = np.zeros((T, nd), dtype=bool)
    for ti, t in enumerate(IOU_THRS):
        gtm = np.zeros(len(gorder), dtype=bool)
        for di in range(nd):
            best, m = min(t, 1 - 1e-10), -1
            for gj in range(len(gorder)):
                if gtm[gj]:
                    continue
                if m > -1 and not g_ign_s[m] and g_ign_s[gj]:
                    break                                   # only ignored GT left
                iou = ious[di, gorder[gj]]
                if iou < best:
                    continue
                best, m = iou, gj
            if m == -1:
                continue
            gtm[m] = True
            dtm[ti, di] = True
            dt_ig[ti, di] = g_ign_s[m]
    # unmatched detections outside the area range are ignored
    d_out = np.array([not (lo <= a <= hi) for a in d_area[:nd]], dtype=bool)
    dt_ig |= (~dtm) & d_out[None, :]
    return dtm, dt_ig, int((~g_ign).sum())


def evaluate(dets: List[dict], gts: List[dict], iou_type: str = "bbox") -> Dict[str, float]:
    """dets: [{image_id, category, score, box (x1y1x2y2) | mask (HxW bool)}];
    gts: [{image_id, category, box | mask, optional area}]."""
    key = "box" if iou_type == "bbox" else "mask"
    cats = sorted({g["category"] for g in gts})
    by_ic_g: Dict = {}
    for g in gts:
        by_ic_g.setdefault((g["image_id"], g["category"]), []).append(
            (g[key], float(g["area"]) if g.get("area") is not None else _area(g[key], iou_type)))
    by_ic_d: Dict = {}
    for d in dets:
        by_ic_d.setdefault((d["image_id"], d["category"]), []).append((d["score"], d[key]))
    iou_fn = box_iou_np if iou_type == "bbox" else mask_iou_np
    T, R, K, A, M = len(IOU_THRS), len(REC_THRS), len(cats), len(AREA_RNG), len(MAX_DETS)
    precision = -np.ones((T, R, K, A, M))
    recall = -np.ones((T, K, A, M))
    for ci, c in enumerate(cats):
        images = sorted({i for (i, cc) in list(by_ic_g) + list(by_ic_d) if cc == c}, key=str)
        per_img = []
        for im in images:
            g = by_ic_g.get((im, c), [])
            d = sorted(by_ic_d.get((im, c), []), key=lambda x: -x[0])[:max(MAX_DETS)]
            ious = (iou_fn(np.stack([x[1] for x in d]), np.stack([x[0] for x in g]))
                    if d and g else np.zeros((len(d), len(g))))
            per_img.append((np.array([x[0] for x in d], dtype=np.float64),
                            np.array([_area(x[1], iou_type) for x in d]), [x[1] for x in g], ious))
        for ai, rng in enumerate(AREA_RNG.values()):
            for mi, md in enumerate(MAX_DETS):
                scores, tps, ign, npig = [], [], [], 0
                for sc, dar, gar, ious in per_img:
                    dtm, dig, ng = _match_image(dar, gar, ious, rng, md)
                    npig += ng
                    scores.append(sc[:md])
                    tps.append(dtm)
                    ign.append(dig)
                if npig == 0:
                    continue
                sc = np.concatenate(scores) if scores else np.zeros(0)
                order = np.argsort(-sc, kind="mergesort")
                dtm = np.concatenate(tps, axis=1)[:, order] if sc.size else np.zeros((T, 0), bool)
                dig = np.concatenate(ign, axis=1)[:, order] if sc.size else np.zeros((T, 0), bool)
                tp = np.cumsum(dtm & ~dig, axis=1).astype(np.float64)
                fp = np.cumsum(~dtm & ~dig, axis=1).astype(np.float64)
                for ti in range(T):
                    rc = tp[ti] / npig
                    pr = tp[ti] / np.maximum(tp[ti] + fp[ti], np.spacing(1))
                    recall[ti, ci, ai, mi] = rc[-1] if rc.size else 0.0
                    pr = pr.tolist()
                    for k in range(len(pr) - 1, 0, -1):
                        if pr[k] > pr[k - 1]:
                            pr[k - 1] = pr[k]
                    q = np.zeros(R)
                    inds = np.searchsorted(rc, REC_THRS, side="left")
                    for ri, pi in enumerate(inds):
                        if pi < len(pr):
                            q[ri] = pr[pi]
                    precision[ti, :, ci, ai, mi] = q

    def mean(x):
        x = x[x > -1]
        return float(x.mean()) if x.size else -1.0

    a = {n: i for i, n in enumerate(AREA_RNG)}
    m100 = MAX_DETS.index(100)
    out = {
        "AP": mean(precision[:, :, :, a["all"], m100]),
        "AP50": mean(precision[0, :, :, a["all"], m100]),
        "AP75": mean(precision[5, :, :, a["all"], m100]),
        "APs": mean(precision[:, :, :, a["small"], m100]),
        "APm": mean(precision[:, :, :, a["medium"], m100]),
        "APl": mean(precision[:, :, :, a["large"], m100]),
    }
    for mi, md in enumerate(MAX_DETS):
        out[f"AR{md}"] = mean(recall[:, :, a["all"], mi])
    out.update({"ARs": mean(recall[:, :, a["small"], m100]), "ARm": mean(recall[:, :, a["medium"], m100]),
                "ARl": mean(recall[:, :, a["large"], m100])})
    # COCOeval prints -1 for an empty summary; the AP keys keep 0.0 as before for callers
    for k in ("AP", "AP50", "AP75"):
        out[k] = max(out[k], 0.0)
    return out


# tensorpack stats.json key suffixes for the first six numbers
TP_KEYS = (("AP", "IoU=0.5:0.95"), ("AP50", "IoU=0.5"), ("AP75", "IoU=0.75"), ("APs", "small"),
           ("APm", "medium"), ("APl", "large"))


def tensorpack_stats(r: Dict[str, float], iou_type: str) -> Dict[str, float]:
    """``evaluate`` output -> tensorpack's stats.json keys (``mAP(bbox)/IoU=0.5:0.95`` ...)."""
    return {f"mAP({iou_type})/{suffix}": r[k] for k, suffix in TP_KEYS}
