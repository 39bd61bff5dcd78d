"""DARTS trial (Katib's ``darts`` suggestion runs the whole search inside one trial;
mxtrain/katib/suggest.py DARTS emits its parameters).

Differentiable architecture search (Liu et al. 2019), first-order variant: a supernet of
``num-layers`` cells, each edge a softmax(alpha)-weighted mixture of the primitives in
``search-space``; network weights step on the training split, architecture weights alpha
on the validation split, alternately.  The derived genotype is argmax(alpha) per edge.

    python -m mxtrain.workloads.nas.darts --algorithm-settings '{"num_epochs": "2"}' \
        --search-space '["separable_convolution_3x3", "max_pooling_3x3", "skip_connection"]' \
        --num-layers 3

Prints ``Best-Genotype=<json>`` and ``Validation-accuracy=<x>`` (Katib StdOut collector).
Data: synthetic 3x32x32 images labelled by a fixed random teacher network (no dataset
download on the node); ``--device cuda`` runs it on the GPU (bf16 autocast).
"""
from __future__ import annotations

import argparse
import json
import re
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F


def make_op(name: str, c: int) -> nn.Module:
    m = re.fullmatch(r"([a-z_]+?)(?:_(\d+)x\d+)?", name)
    kind, k = m.group(1), int(m.group(2) or 3)
    p = k // 2
    if kind == "separable_convolution":
        return nn.Sequential(nn.ReLU(), nn.Conv2d(c, c, k, 1, p, groups=c, bias=False), nn.Conv2d(c, c, 1, bias=False),
                             nn.BatchNorm2d(c, affine=False))
    if kind == "dilated_convolution":
        return nn.Sequential(nn.ReLU(), nn.Conv2d(c, c, k, 1, 2 * p, dilation=2, groups=c, bias=False),
                             nn.Conv2d(c, c, 1, bias=False), nn.BatchNorm2d(c, affine=False))
    if kind in ("convolution",):
        return nn.Sequential(nn.ReLU(), nn.Conv2d(c, c, k, 1, p, bias=False), nn.BatchNorm2d(c, affine=False))
    if kind == "max_pooling":
        return nn.MaxPool2d(k, 1, p)
    if kind == "avg_pooling":
        return nn.AvgPool2d(k, 1, p, count_include_pad=False)
    if kind == "skip_connection":
        return nn.Identity()
    raise ValueError(f"unknown DARTS primitive {name}")


class MixedOp(nn.Module):
    def __init__(self, prims, c):
        super().__init__()
        self.ops = nn.ModuleList(make_op(p, c) for p in prims)

    def forward(self, x, w):
        return sum(wi * op(x) for wi, op in zip(w, self.ops))


class Cell(nn.Module):
    """Two intermediate nodes over the cell input: n1 = op(x), n2 = op(x) + op(n1)."""
    EDGES = 3

    def __init__(self, prims, c):
        super().__init__()
        self.edges = nn.ModuleList(MixedOp(prims, c) for _ in range(self.EDGES))

    def forward(self, x, alphas):
        w = F.softmax(alphas, dim=-1)
        n1 = self.edges[0](x, w[0])
        n2 = self.edges[1](x, w[1]) + self.edges[2](n1, w[2])
        return n1 + n2


class SuperNet(nn.Module):
    def __init__(self, prims, layers, c=16, classes=10):
        super().__init__()
        self.prims = prims
        self.stem = nn.Sequential(nn.Conv2d(3, c, 3, 1, 1, bias=False), nn.BatchNorm2d(c))
        self.cells = nn.ModuleList(Cell(prims, c) for _ in range(layers))
        self.head = nn.Linear(c, classes)
        self.alphas = nn.Parameter(1e-3 * torch.randn(layers, Cell.EDGES, len(prims)))

    def weights(self):
        return [p for n, p in self.named_parameters() if n != "alphas"]

    def forward(self, x):
        x = self.stem(x)
        for i, cell in enumerate(self.cells):
            x = cell(x, self.alphas[i])
        return self.head(x.mean(dim=(2, 3)))

    def genotype(self):
        return [[self.prims[int(j)] for j in a.argmax(-1)] for a in self.alphas.detach()]


def synthetic(n, seed, device):
    g = torch.Generator().manual_seed(seed)
    teacher = nn.Sequential(nn.Conv2d(3, 8, 5, 2, 2), nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(8, 10))
    with torch.no_grad():
        for p in teacher.parameters():
            p.copy_(torch.randn(p.shape, generator=g))
        x = torch.randn(n, 3, 32, 32, generator=g)
        logits = teacher(x)
        y = (logits - logits.mean(0)).argmax(-1)   # centred: every class occurs
    return x.to(device), y.to(device)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--algorithm-settings", default="{}")
    ap.add_argument("--search-space", default='["separable_convolution_3x3", "max_pooling_3x3", "skip_connection"]')
    ap.add_argument("--num-layers", type=int, default=3)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--samples", type=int, default=512)
    a = ap.parse_args(argv)
    st = {k: str(v) for k, v in json.loads(a.algorithm_settings or "{}").items()}
    prims = json.loads(a.search_space)
    epochs = int(st.get("num_epochs", 2))
    w_lr = float(st.get("w_lr", 0.025))
    a_lr = float(st.get("alpha_lr", 3e-3))
    bs = int(st.get("batch_size", 64))
    torch.manual_seed(int(st.get("random_state", 0)))
    dev = torch.device(a.device)
    x, y = synthetic(a.samples * 2, 1, dev)
    xt, yt, xv, yv = x[:a.samples], y[:a.samples], x[a.samples:], y[a.samples:]
    net = SuperNet(prims, a.num_layers).to(dev)
    wopt = torch.optim.SGD(net.weights(), lr=w_lr, momentum=0.9, weight_decay=3e-4)
    aopt = torch.optim.Adam([net.alphas], lr=a_lr, betas=(0.5, 0.999), weight_decay=1e-3)
    amp = dict(device_type="cuda", dtype=torch.bfloat16) if dev.type == "cuda" else None
    for ep in range(epochs):
        perm = torch.randperm(a.samples, device=dev)
        for i in range(0, a.samples, bs):
            idx = perm[i:i + bs]
            # architecture step on validation data (first-order DARTS)
            aopt.zero_grad(set_to_none=True)
            with torch.autocast(**amp) if amp else torch.enable_grad():
                la = F.cross_entropy(net(xv[idx]).float(), yv[idx])
            la.backward()
            aopt.step()
            wopt.zero_grad(set_to_none=True)
            with torch.autocast(**amp) if amp else torch.enable_grad():
                lw = F.cross_entropy(net(xt[idx]).float(), yt[idx])
            lw.backward()
            nn.utils.clip_grad_norm_(net.weights(), 5.0)
            wopt.step()
        with torch.no_grad():
            acc = float((net(xv).argmax(-1) == yv).float().mean())
        print(f"epoch {ep} train-loss={float(lw):.4f} Validation-accuracy={acc:.4f}", flush=True)
    print(f"Best-Genotype={json.dumps(net.genotype())}", flush=True)
    print(f"Validation-accuracy={acc:.4f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
