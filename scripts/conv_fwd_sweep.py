#!/usr/bin/env python3
"""Implicit-GEMM forward at the 1-img Mask R-CNN shapes: time per call (graph replay) for
forced split counts x tile width (128 x 128 vs 128 x 64 tiles), to see where the small
convolutions lose time.  IMGS=1|4."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import convwg  # noqa: E402

# (the shape table and graph-replay timer of scripts/conv_wgrad_bench.py)
SHAPES = [
    ("res3.conv1 s2", 256, 128, 200, 336, 1, 2, 0, 1),
    ("res3.conv2", 128, 128, 100, 168, 3, 1, 1, 4),
    ("res3.conv3", 128, 512, 100, 168, 1, 1, 0, 4),
    ("res3.short s2", 256, 512, 200, 336, 1, 2, 0, 1),
    ("res3.conv1", 512, 128, 100, 168, 1, 1, 0, 3),
    ("res4.conv1 s2", 512, 256, 100, 168, 1, 2, 0, 1),
    ("res4.conv2", 256, 256, 50, 84, 3, 1, 1, 6),
    ("res4.conv3", 256, 1024, 50, 84, 1, 1, 0, 6),
    ("res4.short s2", 512, 1024, 100, 168, 1, 2, 0, 1),
    ("res4.conv1", 1024, 256, 50, 84, 1, 1, 0, 5),
    ("res5.conv1 s2", 1024, 512, 50, 84, 1, 2, 0, 1),
    ("res5.conv2", 512, 512, 25, 42, 3, 1, 1, 3),
    ("res5.conv3", 512, 2048, 25, 42, 1, 1, 0, 3),
    ("res5.short s2", 1024, 2048, 50, 84, 1, 2, 0, 1),
    ("res5.conv1", 2048, 512, 25, 42, 1, 1, 0, 2),
    ("fpn.lat2", 256, 256, 200, 336, 1, 1, 0, 1),
    ("fpn.lat3", 512, 256, 100, 168, 1, 1, 0, 1),
    ("fpn.lat4", 1024, 256, 50, 84, 1, 1, 0, 1),
    ("fpn.lat5", 2048, 256, 25, 42, 1, 1, 0, 1),
    ("fpn.out2 / rpn P2", 256, 256, 200, 336, 3, 1, 1, 2),
    ("fpn.out3 / rpn P3", 256, 256, 100, 168, 3, 1, 1, 2),
    ("fpn.out4 / rpn P4", 256, 256, 50, 84, 3, 1, 1, 2),
    ("fpn.out5 / rpn P5", 256, 256, 25, 42, 3, 1, 1, 2),
    ("rpn P6", 256, 256, 13, 21, 3, 1, 1, 1),
    ("mask head (64 rois)", 256, 256, 14, 14, 3, 1, 1, 4),
    ("rpn level canvas", 256, 256, 301, 336, 3, 1, 1, 1),
]


def timeit(fn, it=10, reps=5):
    """GPU time per call: `it` calls captured in one hipGraph, replayed `reps` times (the
    eager calls of the small convs are host-bound)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(it):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / (it * reps)


def main():
    N = int(os.environ.get("IMGS", "1"))
    dgrad = os.environ.get("DIR", "fwd") == "dgrad"
    cl = torch.channels_last
    splits_list = [1, 2, 4, 8]
    widths = ("128",) if dgrad else ("128", "64")
    print(f"{'dgrad' if dgrad else 'fwd'}: {'conv':22s} {'N':>3s} {'tiles':>5s} {'nk':>4s} "
          + " ".join(f"{'s%d/%s' % (s, h):>8s}" for h in widths for s in splits_list) + "   auto  GF")
    orig_f, orig_d = convwg.fwd_splits, convwg.dgrad_splits
    for name, Cin, Cout, H, W, k, s, p, cnt in SHAPES:
        n = 64 * N if name.startswith("mask") else N
        x = torch.randn(n, Cin, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(Cout, Cin, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
        b = torch.randn(Cout, device="cuda").to(torch.bfloat16)
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        dy = torch.randn(n, Cout, OH, OW, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        T = n * OH * OW
        if dgrad:
            if not convwg.dgrad_supported(w, tuple(x.shape), s, p, 1):
                continue
            tiles = (n * H * W + 127) // 128 * (Cin // 128)
            nk = k * k * Cout // 64
            fn = lambda: convwg.conv_dgrad(dy, w, tuple(x.shape), s, p, 1)
        else:
            tiles = (T + 127) // 128 * (Cout // 128)
            nk = k * k * Cin // 64
            fn = lambda: convwg.conv_fwd(x, w, b, None, True, s, p, 1)
        cols = []
        for half in ((0,) if dgrad else (0, 1 << 30)):
            convwg.FWD_HALF_TILES = half
            for sp in splits_list:
                if dgrad:
                    convwg.dgrad_splits = lambda t, kk, sp=sp: min(sp, kk)
                else:
                    convwg.fwd_splits = lambda t, kk, sp=sp: min(sp, kk)
                cols.append(timeit(fn))
        convwg.fwd_splits, convwg.dgrad_splits = orig_f, orig_d
        convwg.FWD_HALF_TILES = 128
        auto = timeit(fn)
        gf = 2.0 * T * Cout * Cin * k * k / 1e9
        print(f"{name:22s} {n:3d} {tiles:5d} {nk:4d} " + " ".join(f"{c:8.1f}" for c in cols) + f" {auto:6.1f} {gf:5.1f}",
              flush=True)


if __name__ == "__main__":
    main()
