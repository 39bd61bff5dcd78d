"""COCO-format detection data pipeline for the Mask R-CNN workload (tensorpack
`DATA.BASEDIR` / `DATA.TRAIN=["coco_train2017"]` conventions).

* ``COCODetection`` parses ``annotations/instances_<split>.json`` (json only -- no
  pycocotools), maps the 80 COCO category ids to contiguous 1..80, drops crowd boxes
  for training and images without boxes;
* ``DetectionDataset`` decodes the JPEG (PIL), resizes the short edge to
  PREPROC.TRAIN_SHORT_EDGE_SIZE (max PREPROC.MAX_SIZE), random horizontal flip, and
  rasterises every instance polygon at the resized resolution -- either as full-image
  masks (``mask_format="full"``) or, for training, as tight per-instance crops
  (``mask_format="crops"``): a mask is zero outside its polygon's extent, so the crop is
  the same information at a few percent of the bytes, which keeps the loader workers,
  the pinned-memory copy and the H2D transfer small (an 800 x 1333 image with 20
  instances is 21 MB of full masks and typically < 1 MB of crops);
* ``collate`` pads to a fixed canvas per orientation -- (S, M) landscape / (M, S)
  portrait with M = MAX_SIZE rounded up to 32 -- so the training step sees at most two
  static shapes (PREPROC.PREDEFINED_PADDING); ``AspectGroupedSampler`` batches images
  of the same orientation together.  ``fixed_gt`` pads the ground truth to ``max_gt``
  slots so every batch of one orientation has identical shapes (graph replay); the mask
  crops are concatenated into one flat uint8 buffer with an int32 table
  ``[B, G, 5] = (offset, x0, y0, w, h)`` per slot (w = h = 0 for padding).
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
                 with_masks: bool = True, seed: int = 0, mask_format: str = "full"):
        self.coco, self.short, self.max, self.training, self.with_masks = coco, short_edge, max_size, training, with_masks
        assert mask_format in ("full", "crops"), mask_format
        self.mask_format = mask_format
        self.seed = seed
        self.epoch = 0

    def __len__(self):
        return len(self.coco)

    def orientation(self, i: int) -> int:
        im = self.coco.images[self.coco.ids[i]]
        return 0 if im["width"] >= im["height"] else 1

    def __getitem__(self, i: int):
        from PIL import Image
        # AspectGroupedSampler(repeat=True) folds the epoch into the index
        epoch, i = divmod(i, len(self.coco)) if i >= len(self.coco) else (self.epoch, i)
        rec = self.coco.record(i)
        img = Image.open(rec["file"]).convert("RGB")
        w0, h0 = img.size
        h, w, scale = resize_shape(h0, w0, self.short, self.max)
        img = img.resize((w, h), Image.BILINEAR)
        flip = self.training and random.Random(self.seed * 7919 + epoch * 1_000_003 + i).random() < 0.5
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
            polys = []
            for seg in rec["segmentation"]:
                ps = []
                for poly in (seg or []):
                    pts = np.asarray(poly, dtype=np.float32).reshape(-1, 2) * scale
                    if flip:
                        pts[:, 0] = w - pts[:, 0]
                    if len(pts) >= 3:
                        ps.append(pts)
                polys.append(ps)
            if self.mask_format == "full":
                masks = np.zeros((len(polys), h, w), dtype=np.uint8)
                for k, ps in enumerate(polys):
                    masks[k] = rasterize(ps, 0, 0, w, h)
                out["masks"] = torch.from_numpy(masks)
            else:
                out["mask_crops"] = [mask_crop(ps, h, w) for ps in polys]
        return out


def rasterize(polys, x0: int, y0: int, w: int, h: int) -> np.ndarray:
    """uint8 [h, w] 0/1 fill of the polygons, window origin (x0, y0) in image pixels."""
    from PIL import Image, ImageDraw
    m = Image.new("L", (max(w, 0), max(h, 0)), 0)
    if w > 0 and h > 0:
        dr = ImageDraw.Draw(m)
        for pts in polys:
            # integer translation: the fill is identical to the full-image rasterisation
            dr.polygon([(float(x) - x0, float(y) - y0) for x, y in pts.tolist()], fill=1)
    return np.asarray(m, dtype=np.uint8).reshape(max(h, 0), max(w, 0))


def mask_crop(polys, h: int, w: int):
    """(x0, y0, uint8 [ch, cw]) -- the instance mask restricted to its polygons' extent
    (+1 px margin, clipped to the image); an empty crop for an instance without polygons."""
    if not polys:
        return 0, 0, np.zeros((0, 0), dtype=np.uint8)
    allp = np.concatenate(polys, 0)
    x0 = int(max(0, np.floor(allp[:, 0].min()) - 1))
    y0 = int(max(0, np.floor(allp[:, 1].min()) - 1))
    x1 = int(min(w, np.ceil(allp[:, 0].max()) + 2))
    y1 = int(min(h, np.ceil(allp[:, 1].max()) + 2))
    return x0, y0, rasterize(polys, x0, y0, x1 - x0, y1 - y0)


def unpack_mask_crops(flat: torch.Tensor, table: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """Packed crops -> full masks uint8 [B, G, H, W] (reference / debugging)."""
    B, G, _ = table.shape
    out = torch.zeros(B, G, H, W, dtype=torch.uint8)
    fl, tb = flat.cpu(), table.cpu()
    for b in range(B):
        for g in range(G):
            off, x0, y0, cw, ch = [int(v) for v in tb[b, g]]
            if cw > 0 and ch > 0:
                out[b, g, y0:y0 + ch, x0:x0 + cw] = fl[off:off + ch * cw].view(ch, cw)
    return out


def canvas(short: int, max_size: int, orientation: int):
    m = (max_size + 31) // 32 * 32
    s = (short + 31) // 32 * 32
    return (s, m) if orientation == 0 else (m, s)


def collate(batch: List[dict], short: int = 800, max_size: int = 1333, max_gt: int = 100,
            fixed_gt: bool = False) -> dict:
    B = len(batch)
    H = max(b["image"].shape[1] for b in batch)
    W = max(b["image"].shape[2] for b in batch)
    orient = 0 if W >= H else 1
    CH, CW = canvas(short, max_size, orient)
    CH, CW = max(CH, (H + 31) // 32 * 32), max(CW, (W + 31) // 32 * 32)
    img = torch.zeros(B, 3, CH, CW, dtype=torch.uint8)
    G = max_gt if fixed_gt else min(max_gt, max(1, max(b["boxes"].shape[0] for b in batch)))
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
    crops = None
    if "mask_crops" in batch[0]:
        table = torch.zeros(B, G, 5, dtype=torch.int32)
        parts, off = [], 0
        for i, b in enumerate(batch):
            for g, (x0, y0, c) in enumerate(b["mask_crops"][:G]):
                ch, cw = c.shape
                table[i, g] = torch.tensor([off, x0, y0, cw, ch], dtype=torch.int32)
                parts.append(c.reshape(-1))
                off += ch * cw
        crops = (torch.from_numpy(np.concatenate(parts)) if parts else torch.zeros(0, dtype=torch.uint8), table)
    out = {"images": img, "hw": torch.stack([b["hw"] for b in batch]), "gt_boxes": boxes, "gt_labels": cls,
           "gt_count": cnt, "image_ids": [b["image_id"] for b in batch], "scales": [b["scale"] for b in batch]}
    if masks is not None:
        out["gt_masks"] = masks
    if crops is not None:
        out["gt_mask_flat"], out["gt_mask_table"] = crops
    return out


class AspectGroupedSampler(torch.utils.data.Sampler):
    """Distributed, aspect-grouped, epoch-shuffled batch sampler.

    Every batch holds images of one orientation, and every GLOBAL step has one
    orientation: batches are grouped ``world`` at a time within an orientation, the
    groups are shuffled (one shared seed), and rank r takes batch r of each group.  So
    all ranks meet the same canvas shape on the same step -- the whole-step hipGraph
    (workloads/maskrcnn/graphed.py) captures a new shape on every rank together, and the
    padded canvases of one step cost the same on every rank (no straggler from a mixed
    landscape / portrait step).

    ``repeat=True`` yields an endless stream of epochs (tensorpack's RepeatedData): the
    DataLoader iterator then lives for the whole run and its workers never drain at an
    epoch boundary.  The epoch is folded into the yielded indices (``e * len(ds) + i``;
    DetectionDataset maps them back), so flips differ per epoch inside worker processes
    too.
    """

    def __init__(self, ds: DetectionDataset, batch_size: int, rank: int = 0, world: int = 1, seed: int = 0,
                 drop_last: bool = True, repeat: bool = False):
        self.ds, self.bs, self.rank, self.world, self.seed, self.drop = ds, batch_size, rank, world, seed, drop_last
        self.repeat = repeat
        self.epoch = 0
        self.groups = [[i for i in range(len(ds)) if ds.orientation(i) == o] for o in (0, 1)]

    def set_epoch(self, e: int):
        self.epoch = e
        self.ds.epoch = e

    def _batches(self, epoch: int):
        r = random.Random(self.seed + epoch)
        steps, loose = [], []
        for g in self.groups:
            g = list(g)
            r.shuffle(g)
            bl = []
            for k in range(0, len(g), self.bs):
                b = g[k:k + self.bs]
                if len(b) == self.bs or (b and not self.drop):
                    bl.append(b)
            n = len(bl) // self.world * self.world
            steps += [bl[k:k + self.world] for k in range(0, n, self.world)]
            loose += bl[n:]
        r.shuffle(steps)
        out = [b for st in steps for b in st]
        if not out:
            # fewer than ``world`` batches per orientation (tiny sets): mixed-orientation
            # steps, which graphed.py's collective capture protocol also handles
            n = len(loose) // self.world * self.world
            out = loose[:n] if n else loose
        return out

    def _epoch_iter(self, epoch: int):
        off = epoch * len(self.ds) if self.repeat else 0
        for b in self._batches(epoch)[self.rank::self.world]:
            yield [off + i for i in b]

    def __iter__(self):
        if not self.repeat:
            return self._epoch_iter(self.epoch)

        def endless():
            e = self.epoch
            while True:
                yield from self._epoch_iter(e)
                e += 1
        return endless()

    def __len__(self):
        return max(1, len(self._batches(self.epoch)) // self.world)
