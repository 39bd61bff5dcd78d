"""Synthetic COCO-2017-shaped dataset (the node is offline).

Writes exactly the directory layout the reference's coco-data chart downloads
(charts/machine-learning/data-prep/coco-data/templates/coco-data.yaml):

    <data-dir>/train2017/<12-digit id>.jpg
    <data-dir>/val2017/...     <data-dir>/test2017/...
    <data-dir>/annotations/instances_{train,val}2017.json      (COCO format)
    <data-dir>/pretrained-models/ImageNet-R50-AlignPadding.npz  (random-init weights,
                                                                  tensorpack names)

Images are COCO-sized (longer side 640, random aspect) JPEGs with 1-12 filled
polygon/ellipse/rectangle objects over textured backgrounds; every object gets an
exact polygon segmentation, its bbox and area, and one of the 80 COCO category ids.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import random

import numpy as np

# the 80 COCO category ids (1..90 with gaps) and names
COCO_CATEGORIES = [
    (1, "person"), (2, "bicycle"), (3, "car"), (4, "motorcycle"), (5, "airplane"), (6, "bus"), (7, "train"),
    (8, "truck"), (9, "boat"), (10, "traffic light"), (11, "fire hydrant"), (13, "stop sign"),
    (14, "parking meter"), (15, "bench"), (16, "bird"), (17, "cat"), (18, "dog"), (19, "horse"), (20, "sheep"),
    (21, "cow"), (22, "elephant"), (23, "bear"), (24, "zebra"), (25, "giraffe"), (27, "backpack"),
    (28, "umbrella"), (31, "handbag"), (32, "tie"), (33, "suitcase"), (34, "frisbee"), (35, "skis"),
    (36, "snowboard"), (37, "sports ball"), (38, "kite"), (39, "baseball bat"), (40, "baseball glove"),
    (41, "skateboard"), (42, "surfboard"), (43, "tennis racket"), (44, "bottle"), (46, "wine glass"),
    (47, "cup"), (48, "fork"), (49, "knife"), (50, "spoon"), (51, "bowl"), (52, "banana"), (53, "apple"),
    (54, "sandwich"), (55, "orange"), (56, "broccoli"), (57, "carrot"), (58, "hot dog"), (59, "pizza"),
    (60, "donut"), (61, "cake"), (62, "chair"), (63, "couch"), (64, "potted plant"), (65, "bed"),
    (67, "dining table"), (70, "toilet"), (72, "tv"), (73, "laptop"), (74, "mouse"), (75, "remote"),
    (76, "keyboard"), (77, "cell phone"), (78, "microwave"), (79, "oven"), (80, "toaster"), (81, "sink"),
    (82, "refrigerator"), (84, "book"), (85, "clock"), (86, "vase"), (87, "scissors"), (88, "teddy bear"),
    (89, "hair drier"), (90, "toothbrush"),
]


def _polygon(r: random.Random, cx, cy, rx, ry, kind):
    if kind == "rect":
        return [cx - rx, cy - ry, cx + rx, cy - ry, cx + rx, cy + ry, cx - rx, cy + ry]
    n = 24 if kind == "ellipse" else r.randint(5, 9)
    pts = []
    rot = r.random() * math.pi
    for i in range(n):
        a = rot + 2 * math.pi * i / n
        s = 1.0 if kind == "ellipse" else r.uniform(0.55, 1.0)
        pts += [cx + rx * s * math.cos(a), cy + ry * s * math.sin(a)]
    return pts


def _image(r: random.Random, nr: np.random.RandomState, W, H, cats):
    from PIL import Image, ImageDraw
    base = nr.randint(40, 200, size=3)
    grad = np.linspace(0, 1, W)[None, :, None] * nr.randint(-40, 40, size=3)[None, None, :]
    noise = nr.randint(-12, 12, size=(H, W, 3))
    arr = np.clip(base[None, None, :] + grad + noise, 0, 255).astype(np.uint8)
    img = Image.fromarray(arr)
    d = ImageDraw.Draw(img)
    anns = []
    for _ in range(r.randint(1, 12)):
        cid = r.choice(cats)
        rx = r.uniform(0.03, 0.3) * W
        ry = r.uniform(0.03, 0.3) * H
        cx = r.uniform(rx, W - rx)
        cy = r.uniform(ry, H - ry)
        kind = r.choice(["rect", "ellipse", "poly"])
        poly = [round(min(max(v, 0.0), (W if i % 2 == 0 else H) - 1), 2) for i, v in enumerate(_polygon(r, cx, cy, rx, ry, kind))]
        col = tuple(int(c) for c in ((cid * 53) % 256, (cid * 97) % 256, (cid * 193) % 256))
        d.polygon(poly, fill=col)
        xs, ys = poly[0::2], poly[1::2]
        x0, y0, x1, y1 = min(xs), min(ys), max(xs), max(ys)
        # polygon area (shoelace)
        area = 0.5 * abs(sum(xs[i] * ys[(i + 1) % len(xs)] - xs[(i + 1) % len(xs)] * ys[i] for i in range(len(xs))))
        anns.append({"category_id": cid, "bbox": [round(x0, 2), round(y0, 2), round(x1 - x0, 2), round(y1 - y0, 2)],
                     "area": round(area, 2), "iscrowd": 0, "segmentation": [poly]})
    return img, anns


def write_split(data_dir: str, split: str, n: int, seed: int, start_id: int, with_anns=True):
    r = random.Random(seed)
    nr = np.random.RandomState(seed)
    cats = [c for c, _ in COCO_CATEGORIES]
    d = os.path.join(data_dir, split)
    os.makedirs(d, exist_ok=True)
    images, anns = [], []
    aid = start_id * 100
    for k in range(n):
        iid = start_id + k
        long_side = 640
        ar = r.uniform(0.6, 1.0)
        if r.random() < 0.75:      # landscape majority, like COCO
            W, H = long_side, int(long_side * ar)
        else:
            W, H = int(long_side * ar), long_side
        img, a = _image(r, nr, W, H, cats)
        fn = f"{iid:012d}.jpg"
        img.save(os.path.join(d, fn), quality=90)
        images.append({"id": iid, "file_name": fn, "height": H, "width": W})
        for x in a:
            aid += 1
            x.update({"id": aid, "image_id": iid})
            anns.append(x)
    if with_anns:
        os.makedirs(os.path.join(data_dir, "annotations"), exist_ok=True)
        with open(os.path.join(data_dir, "annotations", f"instances_{split}.json"), "w") as f:
            json.dump({"info": {"description": "mxtrain synthetic COCO-shaped data", "year": 2017},
                       "images": images, "annotations": anns,
                       "categories": [{"id": c, "name": nm, "supercategory": "synthetic"} for c, nm in COCO_CATEGORIES]},
                      f)
    return images, anns


def write_backbone_npz(path: str, seed: int = 0, calib_images=None):
    """Random-init ResNet-50 in tensorpack's variable naming (HWIO conv kernels +
    FrozenBN statistics), what BACKBONE.WEIGHTS points at.  The frozen statistics are
    calibrated on a few synthetic images so the random backbone is well conditioned."""
    from ..models.resnet import calibrate_frozen_bn, resnet50
    import torch
    torch.manual_seed(seed)
    m = resnet50(norm="frozen")
    if calib_images:
        from PIL import Image
        ims = []
        for p in calib_images[:4]:
            im = Image.open(p).convert("RGB").resize((320, 256))
            ims.append(torch.from_numpy(np.asarray(im, dtype=np.float32).copy()).permute(2, 0, 1))
        x = torch.stack(ims)
    else:
        x = torch.rand(2, 3, 256, 320) * 255
    mean = torch.tensor([123.675, 116.28, 103.53]).view(1, 3, 1, 1)
    std = torch.tensor([58.395, 57.12, 57.375]).view(1, 3, 1, 1)
    calibrate_frozen_bn(m, (x - mean) / std)
    from ..workloads.maskrcnn.weights import to_tensorpack_npz
    np.savez(path, **to_tensorpack_npz(m))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--data-dir", required=True)
    ap.add_argument("--num-train", type=int, default=256)
    ap.add_argument("--num-val", type=int, default=32)
    ap.add_argument("--num-test", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    write_split(a.data_dir, "train2017", a.num_train, a.seed, 1)
    write_split(a.data_dir, "val2017", a.num_val, a.seed + 1, 1_000_000)
    write_split(a.data_dir, "test2017", a.num_test, a.seed + 2, 2_000_000, with_anns=False)
    os.makedirs(os.path.join(a.data_dir, "pretrained-models"), exist_ok=True)
    import glob
    calib = sorted(glob.glob(os.path.join(a.data_dir, "train2017", "*.jpg")))[:4]
    write_backbone_npz(os.path.join(a.data_dir, "pretrained-models", "ImageNet-R50-AlignPadding.npz"), a.seed, calib)
    print(f"wrote synthetic COCO-2017 layout to {a.data_dir}: {a.num_train} train / {a.num_val} val / "
          f"{a.num_test} test images")


if __name__ == "__main__":
    main()
