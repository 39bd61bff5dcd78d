"""tensorpack-style configuration tree for the Mask R-CNN workload.

Accepts the `--config KEY=VALUE ...` overrides of tensorpack's FasterRCNN/train.py and
the aws-samples mask-rcnn-tensorflow fork exactly as the reference passes them
(charts/machine-learning/training/maskrcnn*/templates/maskrcnn.yaml,
examples/maskrcnn/*.yaml; SURVEY §2.2 "C05/C06", §2.11).  Values are parsed as Python
literals when possible (`MODE_MASK=True`, `TRAIN.LR_SCHEDULE=[240000,320000,360000]`,
`TRAIN.LR_EPOCH_SCHEDULE=[(16, 0.1), (20, 0.01), (24, None)]`), otherwise kept as strings.
"""
from __future__ import annotations

import ast
import json
from typing import Any, List


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, AttrDict) else v) for k, v in self.items()}


def _tree(d):
    return AttrDict({k: _tree(v) if isinstance(v, dict) else v for k, v in d.items()})


DEFAULTS = {
    "MODE_MASK": True,
    "MODE_FPN": True,
    "TRAINER": "replicated",
    "DATA": {"BASEDIR": "/fsx/data/coco2017", "TRAIN": ["coco_train2017"], "VAL": ("coco_val2017",),
             "NUM_CATEGORY": 80, "NUM_WORKERS": 4},
    "BACKBONE": {"WEIGHTS": "", "NORM": "FreezeBN", "FREEZE_AT": 2, "RESNET_NUM_BLOCKS": [3, 4, 6, 3],
                 "STRIDE_1X1": True},
    "TRAIN": {"NUM_GPUS": None, "WEIGHT_DECAY": 1e-4, "BASE_LR": 0.01, "WARMUP": 1000, "WARMUP_INIT_LR": None,
              "STEPS_PER_EPOCH": 500, "STARTING_EPOCH": 1, "LR_SCHEDULE": [240000, 320000, 360000],
              "LR_EPOCH_SCHEDULE": None, "EVAL_PERIOD": 25, "CHECKPOINT_PERIOD": 20, "BATCH_SIZE_PER_GPU": 1,
              "GRADIENT_CLIP": 0.0, "MOMENTUM": 0.9},
    "PREPROC": {"TRAIN_SHORT_EDGE_SIZE": [800, 800], "TEST_SHORT_EDGE_SIZE": 800, "MAX_SIZE": 1333,
                "PIXEL_MEAN": [123.675, 116.28, 103.53], "PIXEL_STD": [58.395, 57.12, 57.375],
                "PREDEFINED_PADDING": False},
    "RPN": {"ANCHOR_STRIDE": 16, "ANCHOR_SIZES": [32, 64, 128, 256, 512], "ANCHOR_RATIOS": [0.5, 1.0, 2.0],
            "POSITIVE_ANCHOR_THRESH": 0.7, "NEGATIVE_ANCHOR_THRESH": 0.3, "FG_RATIO": 0.5, "BATCH_PER_IM": 256,
            "PROPOSAL_NMS_THRESH": 0.7, "TRAIN_PER_LEVEL_NMS_TOPK": 2000, "TEST_PER_LEVEL_NMS_TOPK": 1000,
            "TRAIN_POST_NMS_TOPK": 2000, "TEST_POST_NMS_TOPK": 1000},
    "FRCNN": {"BATCH_PER_IM": 512, "FG_THRESH": 0.5, "FG_RATIO": 0.25, "BBOX_REG_WEIGHTS": [10.0, 10.0, 5.0, 5.0]},
    "FPN": {"ANCHOR_STRIDES": [4, 8, 16, 32, 64], "NUM_CHANNEL": 256, "FRCNN_HEAD_FUNC": "fastrcnn_2fc_head",
            "FRCNN_FC_HEAD_DIM": 1024, "MRCNN_HEAD_FUNC": "maskrcnn_up4conv_head"},
    "MRCNN": {"HEAD_DIM": 256, "ACCURATE_PASTE": True},
    "TEST": {"FRCNN_NMS_THRESH": 0.5, "RESULT_SCORE_THRESH": 0.05, "RESULTS_PER_IM": 100},
}


def parse_value(s: str) -> Any:
    try:
        return ast.literal_eval(s)
    except (ValueError, SyntaxError):
        return s


def make_config(overrides: List[str]) -> AttrDict:
    cfg = _tree(json.loads(json.dumps(DEFAULTS)))
    cfg.DATA.VAL = tuple(cfg.DATA.VAL)
    for item in overrides:
        if "=" not in item:
            raise ValueError(f"--config expects KEY=VALUE, got {item!r}")
        k, v = item.split("=", 1)
        node = cfg
        parts = k.split(".")
        for p in parts[:-1]:
            if p not in node:
                node[p] = AttrDict()
            node = node[p]
        node[parts[-1]] = parse_value(v)
    return cfg


def finalize(cfg: AttrDict, num_gpus: int, images_per_epoch: int = None):
    """Derive the schedule for the actual world size (tensorpack's config finalize)."""
    cfg.TRAIN.NUM_GPUS = num_gpus
    bs = int(cfg.TRAIN.BATCH_SIZE_PER_GPU)
    total = num_gpus * bs
    if isinstance(cfg.DATA.TRAIN, str):
        cfg.DATA.TRAIN = [cfg.DATA.TRAIN]
    if isinstance(cfg.DATA.VAL, str):
        cfg.DATA.VAL = (cfg.DATA.VAL,)
    if cfg.TRAIN.LR_EPOCH_SCHEDULE or images_per_epoch:
        # aws-samples convention: BASE_LR is per image, schedule in epochs of images_per_epoch
        cfg.TRAIN.LR = float(cfg.TRAIN.BASE_LR) * total
        ipe = int(images_per_epoch or 120000)
        cfg.TRAIN.STEPS_PER_EPOCH = max(1, ipe // total)
        sched = cfg.TRAIN.LR_EPOCH_SCHEDULE or [(16, 0.1), (20, 0.01), (24, None)]
        cfg.TRAIN.MAX_EPOCH = int(sched[-1][0])
        cfg.TRAIN.LR_STEPS = [(int(e) * cfg.TRAIN.STEPS_PER_EPOCH, m) for e, m in sched if m is not None]
        cfg.TRAIN.WARMUP_STEPS = min(1000, cfg.TRAIN.STEPS_PER_EPOCH)
    else:
        # tensorpack convention: BASE_LR for a total batch of 8, LR_SCHEDULE in iterations
        # of that batch; scale both to the real total batch (linear scaling rule)
        factor = 8.0 / total
        cfg.TRAIN.LR = float(cfg.TRAIN.BASE_LR) * total / 8.0
        steps = [int(s * factor) for s in cfg.TRAIN.LR_SCHEDULE]
        cfg.TRAIN.LR_STEPS = [(s, 0.1 ** (i + 1)) for i, s in enumerate(steps[:-1])]
        cfg.TRAIN.MAX_EPOCH = max(1, steps[-1] // int(cfg.TRAIN.STEPS_PER_EPOCH))
        cfg.TRAIN.WARMUP_STEPS = int(cfg.TRAIN.WARMUP * factor)
    if cfg.TRAIN.WARMUP_INIT_LR is None:
        cfg.TRAIN.WARMUP_INIT_LR = cfg.TRAIN.LR * 0.33
    short = cfg.PREPROC.TRAIN_SHORT_EDGE_SIZE
    cfg.PREPROC.TRAIN_SHORT = int(short[0] if isinstance(short, (list, tuple)) else short)
    return cfg


def lr_at(cfg: AttrDict, step: int) -> float:
    t = cfg.TRAIN
    if step < t.WARMUP_STEPS:
        a = step / max(1, t.WARMUP_STEPS)
        return t.WARMUP_INIT_LR + a * (t.LR - t.WARMUP_INIT_LR)
    lr = t.LR
    for s, m in t.LR_STEPS:
        if step >= s:
            lr = t.LR * m
    return lr


def model_config(cfg: AttrDict):
    from ...models.maskrcnn import MaskRCNNConfig
    return MaskRCNNConfig(
        num_classes=int(cfg.DATA.NUM_CATEGORY) + 1, fpn_channels=int(cfg.FPN.NUM_CHANNEL),
        anchor_sizes=tuple(cfg.RPN.ANCHOR_SIZES), anchor_ratios=tuple(cfg.RPN.ANCHOR_RATIOS),
        anchor_strides=tuple(cfg.FPN.ANCHOR_STRIDES), rpn_fg_thresh=float(cfg.RPN.POSITIVE_ANCHOR_THRESH),
        rpn_bg_thresh=float(cfg.RPN.NEGATIVE_ANCHOR_THRESH), rpn_batch_per_im=int(cfg.RPN.BATCH_PER_IM),
        rpn_fg_ratio=float(cfg.RPN.FG_RATIO), rpn_nms_thresh=float(cfg.RPN.PROPOSAL_NMS_THRESH),
        train_per_level_topk=int(cfg.RPN.TRAIN_PER_LEVEL_NMS_TOPK),
        train_post_nms_topk=int(cfg.RPN.TRAIN_POST_NMS_TOPK), test_per_level_topk=int(cfg.RPN.TEST_PER_LEVEL_NMS_TOPK),
        test_post_nms_topk=int(cfg.RPN.TEST_POST_NMS_TOPK), frcnn_batch_per_im=int(cfg.FRCNN.BATCH_PER_IM),
        frcnn_fg_ratio=float(cfg.FRCNN.FG_RATIO), frcnn_fg_thresh=float(cfg.FRCNN.FG_THRESH),
        bbox_reg_weights=tuple(float(x) for x in cfg.FRCNN.BBOX_REG_WEIGHTS), fc_dim=int(cfg.FPN.FRCNN_FC_HEAD_DIM),
        mask=bool(cfg.MODE_MASK), mask_head_dim=int(cfg.MRCNN.HEAD_DIM),
        result_score_thresh=float(cfg.TEST.RESULT_SCORE_THRESH), test_nms_thresh=float(cfg.TEST.FRCNN_NMS_THRESH),
        results_per_im=int(cfg.TEST.RESULTS_PER_IM), pixel_mean=tuple(cfg.PREPROC.PIXEL_MEAN),
        pixel_std=tuple(cfg.PREPROC.PIXEL_STD))
