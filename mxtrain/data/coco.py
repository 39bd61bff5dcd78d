"""COCO-format detection data pipeline for the Mask R-CNN workload (tensorpack
`DATA.BASEDIR` / `DATA.TRAIN=["coco_train2017"]` conventions).

* ``COCODetection`` parses ``annotations/instances_<split>.json`` (json only -- no
  pycocotools), maps the 80 COCO category ids to contiguous 1..80, drops crowd boxes
  for training and images without boxes;
* ``DetectionDataset`` decodes the JPEG (PIL), resizes the short edge to
  PREPROC.TRAIN_SHORT_EDGE_SIZE (max PREPROC.MAX_SIZE), random horizontal flip, and
  rasterises every instance polygon at the resized resolution;
* ``collate`` pads to a fixed canvas per orientation -- (S, M) landscape / (M, S)
  portrait with M = MAX_SIZE rounded up to 32 -- so the training step sees at most two
  static shapes (PREPROC.PREDEFINED_PADDING); ``AspectGroupedSampler`` batches images
  of the same orientation together.
"""
from __future__ import annotations

import json
import os
import random
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .coco_synth import COCO_CATEGORIES

CAT_IDS = [c for c, _ in COCO_CATEGORIES]
CAT_TO_CONTIG = {c: i + 1 for i, c in enumerate(CAT_IDS)}
CONTIG_TO_CAT = {v: k for k, v in CAT_TO_CONTIG.items()}
CLASS_NAMES = ["BG"] + [n for _, n in COCO_CATEGORIES]


def split_dir_and_json(basedir: str, name: str):
    """"coco_train2017" -> (<basedir>/train2017, <basedir>/annotations/instances_train2017.json)."""
    s = name[len("coco_"):] if name.startswith("coco_") else name
    return os.path.join(basedir, s), os.path.join(basedir, "annotations", f"instances_{s}.json")


class COCODetection:
    def __init__(self, basedir: str, name: str, training: bool = True):
        self.img_dir, ann_file = split_dir_and_json(basedir, name)
        with open(ann_file) as f:
            js = json.load(f)
        self.images = {im["id"]: im for im in js["images"]}
        anns: Dict[int, List[dict]] = {}
        for a in js.get("annotations", []):
            if training and a.get("iscrowd", 0):
                continue
            if a["bbox"][2] < 1 or a["bbox"][3] < 1:
                continue
            anns.setdefault(a["image_id"], []).append(a)
        ids = sorted(self.images)
        if training:
            ids = [i for i in ids if anns.get(i)]
        self.ids = ids
        self.anns = anns

    def __len__(self):
        return len(self.ids)

    def record(self, i: int) -> dict:
        iid = self.ids[i]
        im = self.images[iid]
        a = self.anns.get(iid, [])
        boxes = np.array([[x["bbox"][0], x["bbox"][1], x["bbox"][0] + x["bbox"][2], x["bbox"][1] + x["bbox"][3]]
                          for x in a], dtype=np.float32).reshape(-1, 4)
        cls = np.array([CAT_TO_CONTIG[x["category_id"]] for x in a], dtype=np.int64)
        segs = [x.get("segmentation") for x in a]
        return {"image_id": iid, "file": os.path.join(self.img_dir, im["file_name"]), "height": im["height"],
                "width": im["width"], "boxes": boxes, "classes": cls, "segmentation": segs}


def resize_shape(h: int, w: int, short: int, max_size: int):
    scale = short / min(h, w)
    if max(h, w) * scale > max_size:
        scale = max_size / max(h, w)
    return int(round(h * scale)), int(round(w * scale)), scale


class DetectionDataset(torch.utils.data.Dataset):
    def __init__(self, coco: COCODetection, short_edge: int = 800, max_size: int = 1333, training: bool = True,
                 with_masks: bool = True, seed: int = 0):
        self.coco, self.short, self.max, self.training, self.with_masks = coco, short_edge, max_size, training, with_masks
        self.seed = seed
        self.epoch = 0

    def __len__(self):
        return len(self.coco)

    def orientation(self, i: int) -> int:
        im = self.coco.images[self.coco.ids[i]]
        return 0 if im["width"] >= im["height"] else 1

    def __getitem__(self, i: int):
        from PIL import Image, ImageDraw
        rec = self.coco.record(i)
        img = Image.open(rec["file"]).convert("RGB")
        w0, h0 = img.size
        h, w, scale = resize_shape(h0, w0, self.short, self.max)
        img = img.resize((w, h), Image.BILINEAR)
        flip = self.training and random.Random(self.seed * 7919 + self.epoch * 1_000_003 + i).random() < 0.5
        if flip:
            img = img.transpose(Image.FLIP_LEFT_RIGHT)
        arr = torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1)     # [3, h, w]
        boxes = torch.from_numpy(rec["boxes"]) * scale
        if flip:
            boxes = torch.stack([w - boxes[:, 2], boxes[:, 1], w - boxes[:, 0], boxes[:, 3]], 1)
        out = {"image": arr, "boxes": boxes, "classes": torch.from_numpy(rec["classes"]),
               "hw": torch.tensor([h, w], dtype=torch.float32), "image_id": rec["image_id"], "scale": scale,
               "orig_hw": (h0, w0)}
        if self.with_masks:
            masks = np.zeros((len(rec["segmentation"]), h, w), dtype=np.uint8)
            for k, seg in enumerate(rec["segmentation"]):
                m = Image.new("L", (w, h), 0)
                dr = ImageDraw.Draw(m)
                for poly in (seg or []):
                    pts = np.asarray(poly, dtype=np.float32).reshape(-1, 2) * scale
                    if flip:
                        pts[:, 0] = w - pts[:, 0]
                    if len(pts) >= 3:
                        dr.polygon([tuple(p) for p in pts.tolist()], fill=1)
                masks[k] = np.asarray(m, dtype=np.uint8)
            out["masks"] = torch.from_numpy(masks)
        return out


def canvas(short: int, max_size: int, orientation: int):
    m = (max_size + 31) // 32 * 32
    s = (short + 31) // 32 * 32
    return (s, m) if orientation == 0 else (m, s)


def collate(batch: List[dict], short: int = 800, max_size: int = 1333, max_gt: int = 100) -> dict:
    B = len(batch)
    H = max(b["image"].shape[1] for b in batch)
    W = max(b["image"].shape[2] for b in batch)
    orient = 0 if W >= H else 1
    CH, CW = canvas(short, max_size, orient)
    CH, CW = max(CH, (H + 31) // 32 * 32), max(CW, (W + 31) // 32 * 32)
    img = torch.zeros(B, 3, CH, CW, dtype=torch.uint8)
    G = min(max_gt, max(1, max(b["boxes"].shape[0] for b in batch)))
    Gm = (G + 7) // 8 * 8
    boxes = torch.zeros(B, G, 4)
    cls = torch.zeros(B, G, dtype=torch.long)
    cnt = torch.zeros(B, dtype=torch.int32)
    masks = torch.zeros(B, Gm, CH, CW, dtype=torch.uint8) if "masks" in batch[0] else None
    for i, b in enumerate(batch):
        h, w = b["image"].shape[1:]
        img[i, :, :h, :w] = b["image"]
        n = min(G, b["boxes"].shape[0])
        boxes[i, :n] = b["boxes"][:n]
        cls[i, :n] = b["classes"][:n]
        cnt[i] = n
        if masks is not None:
            masks[i, :n, :h, :w] = b["masks"][:n]
    out = {"images": img, "hw": torch.stack([b["hw"] for b in batch]), "gt_boxes": boxes, "gt_labels": cls,
           "gt_count": cnt, "image_ids": [b["image_id"] for b in batch], "scales": [b["scale"] for b in batch]}
    if masks is not None:
        out["gt_masks"] = masks
    return out


class AspectGroupedSampler(torch.utils.data.Sampler):
    """Distributed, aspect-grouped, epoch-shuffled batch sampler: every batch holds
    images of one orientation; rank r takes every world-th batch."""

    def __init__(self, ds: DetectionDataset, batch_size: int, rank: int = 0, world: int = 1, seed: int = 0,
                 drop_last: bool = True):
        self.ds, self.bs, self.rank, self.world, self.seed, self.drop = ds, batch_size, rank, world, seed, drop_last
        self.epoch = 0
        self.groups = [[i for i in range(len(ds)) if ds.orientation(i) == o] for o in (0, 1)]

    def set_epoch(self, e: int):
        self.epoch = e
        self.ds.epoch = e

    def _batches(self):
        r = random.Random(self.seed + self.epoch)
        out = []
        for g in self.groups:
            g = list(g)
            r.shuffle(g)
            for k in range(0, len(g), self.bs):
                b = g[k:k + self.bs]
                if len(b) == self.bs or (b and not self.drop):
                    out.append(b)
        r.shuffle(out)
        n = len(out) // self.world * self.world
        return out[:n] if n else out

    def __iter__(self):
        bs = self._batches()
        return iter(bs[self.rank::self.world])

    def __len__(self):
        return max(1, len(self._batches()) // self.world)
