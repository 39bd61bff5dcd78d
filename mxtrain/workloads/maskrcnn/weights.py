"""ResNet backbone weights <-> tensorpack `.npz` naming (BACKBONE.WEIGHTS, e.g.
ImageNet-R50-AlignPadding.npz).  Loaded with numpy.load(allow_pickle=False)."""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch


def _pairs(resnet):
    """(tensorpack prefix, ConvNorm module) for every conv of the backbone."""
    out = [("conv0", resnet.stem)]
    for gi, stage in enumerate(resnet.stages):
        for bi, blk in enumerate(stage):
            p = f"group{gi}/block{bi}"
            out += [(f"{p}/conv1", blk.conv1), (f"{p}/conv2", blk.conv2), (f"{p}/conv3", blk.conv3)]
            if blk.shortcut is not None:
                out.append((f"{p}/convshortcut", blk.shortcut))
    return out


def to_tensorpack_npz(resnet) -> Dict[str, np.ndarray]:
    d = {}
    for name, cn in _pairs(resnet):
        d[f"{name}/W"] = cn.conv.weight.detach().permute(2, 3, 1, 0).contiguous().cpu().numpy()   # OIHW -> HWIO
        n = cn.norm
        d[f"{name}/bn/gamma"] = n.weight.detach().cpu().numpy()
        d[f"{name}/bn/beta"] = n.bias.detach().cpu().numpy()
        d[f"{name}/bn/mean/EMA"] = n.running_mean.detach().cpu().numpy()
        d[f"{name}/bn/variance/EMA"] = n.running_var.detach().cpu().numpy()
    return d


def load_tensorpack_npz(resnet, path: str, strict: bool = False) -> int:
    """Copy matching arrays into the backbone; returns the number of tensors loaded."""
    data = np.load(path, allow_pickle=False)
    n = 0
    with torch.no_grad():
        for name, cn in _pairs(resnet):
            k = f"{name}/W"
            if k in data:
                cn.conv.weight.copy_(torch.from_numpy(data[k]).permute(3, 2, 0, 1))
                n += 1
            elif strict:
                raise KeyError(k)
            for suf, attr in (("gamma", "weight"), ("beta", "bias"), ("mean/EMA", "running_mean"),
                              ("variance/EMA", "running_var")):
                k = f"{name}/bn/{suf}"
                if k in data:
                    getattr(cn.norm, attr).copy_(torch.from_numpy(data[k]))
                    n += 1
    return n
