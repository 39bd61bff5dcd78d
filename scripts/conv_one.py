#!/usr/bin/env python3
"""One implicit-GEMM convolution shape, N calls of each direction (for rocprofv3 kernel
traces / PMC passes over csrc/convwg.hip).  Defaults: the RPN level canvas 3x3 at 4 images.
    python scripts/conv_one.py [--n 4 --cin 256 --cout 256 --h 301 --w 336 --k 3 --pad 1]
        [--iters 10] [--dirs fwd,dgrad,wgrad]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    for name, v in (("n", 4), ("cin", 256), ("cout", 256), ("h", 301), ("w", 336), ("k", 3), ("stride", 1),
                    ("pad", 1), ("iters", 10)):
        ap.add_argument(f"--{name}", type=int, default=v)
    ap.add_argument("--dirs", default="fwd,dgrad,wgrad")
    a = ap.parse_args()
    import torch
    from mxtrain.ops import convwg
    cl = torch.channels_last
    x = torch.randn(a.n, a.cin, a.h, a.w, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(a.cout, a.cin, a.k, a.k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    b = torch.randn(a.cout, device="cuda").to(torch.bfloat16)
    y = convwg.conv_fwd(x, w, b, None, True, a.stride, a.pad, 1)
    dy = torch.randn_like(y)
    dirs = a.dirs.split(",")
    for _ in range(a.iters):
        if "fwd" in dirs:
            convwg.conv_fwd(x, w, b, None, True, a.stride, a.pad, 1)
        if "dgrad" in dirs:
            convwg.conv_dgrad(dy, w, tuple(x.shape), a.stride, a.pad, 1)
        if "wgrad" in dirs:
            convwg.conv_wgrad(dy, x, tuple(w.shape), a.stride, a.pad, 1)
    torch.cuda.synchronize()
    print("ok", tuple(y.shape))


if __name__ == "__main__":
    main()
