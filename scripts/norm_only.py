#!/usr/bin/env python3
"""The GPT-2 345M BDA-LayerNorm kernels alone (for rocprofv3 kernel traces and PMC passes):
h = residual + dropout(x + bias); y = LN(h) forward and its fused backward (dx with the
dropout mask regenerated, dresidual, dgamma / dbeta / dbias column partials), [rows, cols]
bf16, N iterations.
    python scripts/norm_only.py [--rows 4096] [--cols 1024] [--iters 20] [--dropout 0.1]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops.norm import bda_norm_fwd, norm_bwd  # noqa: E402
from mxtrain.ops.rng import DropoutSeed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--cols", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dropout", type=float, default=0.1)
    a = ap.parse_args()
    dev = "cuda"
    bf = torch.bfloat16
    x = torch.randn(a.rows, a.cols, device=dev).to(bf)
    r = torch.randn(a.rows, a.cols, device=dev).to(bf)
    b = torch.randn(a.cols, device=dev).to(bf)
    g = (1 + 0.1 * torch.randn(a.cols, device=dev)).to(bf)
    be = (0.1 * torch.randn(a.cols, device=dev)).to(bf)
    dy = torch.randn(a.rows, a.cols, device=dev).to(bf)
    dres = torch.randn(a.rows, a.cols, device=dev).to(bf)
    seed = DropoutSeed(torch.device(dev), 1234)
    dg, db, dbias = (torch.zeros(a.cols, device=dev, dtype=bf) for _ in range(3))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for it in range(a.iters + 3):
        if it == 3:
            ev[0].record()
        h, y, mean, rstd = bda_norm_fwd(x, b, r, g, be, 1e-5, a.dropout, seed.t, 1001)
        if it == a.iters + 2:
            ev[1].record()
        norm_bwd(dy, dres, h, mean, rstd, g, want_dx=True, p=a.dropout, seed_t=seed.t, salt=1001,
                 dgamma=dg, dbeta=db, dbias=dbias, accumulate=True)
    ev[2].record()
    torch.cuda.synchronize()
    print(f"rows {a.rows} cols {a.cols} dropout {a.dropout}: {a.iters} iterations, "
          f"{ev[0].elapsed_time(ev[2]) * 1000 / a.iters:.1f} us per fwd+bwd")


if __name__ == "__main__":
    main()
