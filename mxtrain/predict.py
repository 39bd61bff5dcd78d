"""Mask R-CNN offline predictor (the reference's Jupyter visualisation notebooks,
SURVEY §2.1 C15/C16 and §3.8 "Serving": newest `model-*.index` under
`$LOGDIR/train_log/maskrcnn`, `predict_image`, draw boxes + masks with score >= 0.7 and
mask >= 0.5).

    python -m mxtrain.predict --logdir /fsx/logs/<rel>-<date> [--image a.jpg ...] \\
        [--data-dir /fsx/data/coco2017] [--out predictions/]

Without --image a random test2017 image from --data-dir is used, as the notebooks do.
Writes <out>/<name>.png overlays and prints one JSON line per image (boxes, scores,
class names, mask pixel counts).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import random
import sys

import numpy as np
import torch


def _find_ckpt_dir(logdir: str) -> str:
    for d in (logdir, os.path.join(logdir, "train_log", "maskrcnn")):
        if glob.glob(os.path.join(d, "model-*.index")):
            return d
    raise FileNotFoundError(f"no model-*.index under {logdir} or {logdir}/train_log/maskrcnn")


@torch.no_grad()
def predict_images(model, paths, device, out_dir, short=800, max_size=1333, score_thresh=0.7, mask_thresh=0.5):
    from PIL import Image, ImageDraw
    from .data.coco import CLASS_NAMES, resize_shape
    from .workloads.maskrcnn.train import paste_mask
    model.eval()
    os.makedirs(out_dir, exist_ok=True)
    results = []
    for p in paths:
        img0 = Image.open(p).convert("RGB")
        w0, h0 = img0.size
        h, w, s = resize_shape(h0, w0, short, max_size)
        img = img0.resize((w, h), Image.BILINEAR)
        H, W = (h + 31) // 32 * 32, (w + 31) // 32 * 32
        t = torch.zeros(1, 3, H, W, dtype=torch.uint8)
        t[0, :, :h, :w] = torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1)
        res = model(t.to(device), torch.tensor([[h, w]], dtype=torch.float32, device=device))
        valid = (res["scores"][0] >= score_thresh).cpu()
        boxes = (res["boxes"][0].cpu() / s)[valid].numpy()
        scores = res["scores"][0].cpu()[valid].numpy()
        labels = res["labels"][0].cpu()[valid].numpy()
        overlay = img0.copy()
        draw = ImageDraw.Draw(overlay)
        mask_px = []
        if "masks" in res:
            m28 = res["masks"][0].cpu()[valid].numpy()
            canvas = np.asarray(overlay).copy()
            for k in range(len(scores)):
                full = paste_mask(m28[k], boxes[k], h0, w0, mask_thresh)
                mask_px.append(int(full.sum()))
                col = np.array([(37 * int(labels[k])) % 255, (91 * int(labels[k])) % 255, 160])
                canvas[full] = (0.5 * canvas[full] + 0.5 * col).astype(np.uint8)
            overlay = Image.fromarray(canvas)
            draw = ImageDraw.Draw(overlay)
        for k in range(len(scores)):
            x0, y0, x1, y1 = boxes[k].tolist()
            draw.rectangle([x0, y0, x1, y1], outline=(255, 64, 64), width=2)
            draw.text((x0 + 2, y0 + 2), f"{CLASS_NAMES[int(labels[k])]} {scores[k]:.2f}", fill=(255, 255, 255))
        name = os.path.splitext(os.path.basename(p))[0]
        out = os.path.join(out_dir, f"{name}.png")
        overlay.save(out)
        rec = {"image": p, "output": out, "boxes": boxes.round(1).tolist(), "scores": scores.round(4).tolist(),
               "labels": [CLASS_NAMES[int(c)] for c in labels], "mask_pixels": mask_px}
        print(json.dumps(rec), flush=True)
        results.append(rec)
    return results


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--logdir", required=True)
    ap.add_argument("--image", nargs="*", default=None)
    ap.add_argument("--data-dir", default="/fsx/data/coco2017")
    ap.add_argument("--out", default=None)
    ap.add_argument("--score-thresh", type=float, default=0.7)
    ap.add_argument("--config", nargs="*", default=[])
    a = ap.parse_args(argv)
    from .models.maskrcnn import MaskRCNN
    from .workloads.maskrcnn import config as C
    from .workloads.maskrcnn.train import latest_ckpt, load_ckpt
    d = _find_ckpt_dir(a.logdir)
    overrides = list(a.config)
    cfg = C.make_config(overrides)
    C.finalize(cfg, 1)
    device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    model = MaskRCNN(C.model_config(cfg)).to(device)
    ck = latest_ckpt(d)
    load_ckpt(model, ck)
    images = a.image
    if not images:
        cands = sorted(glob.glob(os.path.join(a.data_dir, "test2017", "*.jpg")))
        if not cands:
            raise SystemExit(f"no --image given and no test2017 images under {a.data_dir}")
        images = [random.choice(cands)]
    predict_images(model, images, device, a.out or os.path.join(d, "predictions"), cfg.PREPROC.TRAIN_SHORT,
                   int(cfg.PREPROC.MAX_SIZE), a.score_thresh)
    return 0


if __name__ == "__main__":
    sys.exit(main())
