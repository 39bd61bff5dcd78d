#!/usr/bin/env python3
"""BN ResNet-50 training step (BASELINE config 5 model: batch 256 at 224^2, channels_last,
bf16 autocast, SGD-Nesterov) A/B in one process, interleaved rounds on the same random data:
  fused   csrc/batchnorm.hip BN + residual + ReLU nodes and the implicit-GEMM convolutions
  bn      the fused BN nodes, convolutions on MIOpen (ops/convwg.py switched off)
  torch   nn.BatchNorm2d + add + ReLU on MIOpen (the round-3 path)
  any other arm: "name:module.attr=value,..." on top of fused (e.g.
  "noepi:mxtrain.models.resnet.BN_EPILOGUE_STATS=0")
Prints images/s per arm (median over rounds).
    python scripts/resnet_ab.py [--batch 256] [--steps 10] [--rounds 3] [--arms fused,bn,torch]"""
import importlib
import argparse
import os
import statistics
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.models import resnet as R  # noqa: E402
from mxtrain.ops import batchnorm as BN  # noqa: E402
from mxtrain.ops import convwg  # noqa: E402


_SAVED = {}


def set_arm(arm):
    for (mod, attr), v in _SAVED.items():
        setattr(mod, attr, v)
    name, _, spec = arm.partition(":")
    base = "fused" if spec else name
    convwg.ENABLED = convwg.FWD = convwg.DGRAD = base == "fused"
    BN.ENABLED = base in ("fused", "bn")
    for item in filter(None, spec.split(",")):
        path, val = item.split("=")
        modname, attr = path.rsplit(".", 1)
        try:
            mod = importlib.import_module(modname)
        except ModuleNotFoundError:   # a class attribute: module.Class.attr
            modname, cls = modname.rsplit(".", 1)
            mod = getattr(importlib.import_module(modname), cls)
        _SAVED.setdefault((mod, attr), getattr(mod, attr))
        cur = getattr(mod, attr)
        setattr(mod, attr, type(cur)(int(val)) if isinstance(cur, (bool, int)) else type(cur)(val))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--arms", default="fused,bn,torch")
    a = ap.parse_args()
    torch.manual_seed(0)
    net = R.resnet50(norm="bn", num_classes=1000).cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, nesterov=True, weight_decay=5e-5)
    x = torch.randn(a.batch, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(net(x).float(), y, label_smoothing=0.1)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    res = {arm: [] for arm in a.arms.split(";" if ":" in a.arms else ",")}
    for arm in res:   # warm-up (MIOpen immediate-mode solution lookups, allocator)
        set_arm(arm)
        for _ in range(3):
            step()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for arm in res:
            set_arm(arm)
            step()
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(a.steps):
                loss = step()
            torch.cuda.synchronize()
            res[arm].append(a.batch * a.steps / (time.time() - t0))
    for arm, v in res.items():
        print(f"{arm.partition(':')[0]:6s} {statistics.median(v):8.1f} images/s  (rounds {[round(t) for t in v]})  loss {float(loss):.3f}")


if __name__ == "__main__":
    main()
