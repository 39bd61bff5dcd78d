#!/usr/bin/env python3
"""ops/vision.py topk_rows at the Mask R-CNN step's shapes (post-NMS top 2000 of 5 x 2000
sorted level lists, RoI sampling's 128 / 512 of ~2100 uniform keys, the RPN sampling's 128 /
256 of ~270k keys), timed with events; --lib picks a kernel-library build (A/B), and each
result is checked against torch.topk.
    python scripts/topk_bench.py [--lib mxtrain/lib/ab/libmxkernels_a.so]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import torch
    from mxtrain.ops import _lib
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    from mxtrain.ops import vision as V
    g = torch.Generator().manual_seed(0)
    lv = torch.sort(torch.rand(1, 5, 2000, generator=g), dim=-1, descending=True)[0]
    lv[..., 1500:] = -float("inf")
    cases = {
        "post-NMS 2000 of 10000 (B 1)": (lv.reshape(1, -1), 2000, True),
        "post-NMS 2000 of 10000 (B 4)": (lv.reshape(1, -1).repeat(4, 1), 2000, True),
        "RoI fg 128 of 2100": (torch.rand(1, 2100, generator=g), 128, False),
        "RoI order 512 of 2100": (torch.rand(1, 2100, generator=g) + 1.0, 512, True),
        "RPN pos 128 of 268569": (torch.rand(1, 268569, generator=g), 128, False),
        "RPN neg 256 of 268569": (torch.rand(1, 268569, generator=g), 256, False),
    }
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, (x, k, largest) in cases.items():
        x = x.cuda()
        v, i = V.topk_rows(x, k, largest=largest)
        rv, _ = x.topk(k, dim=1, largest=largest)
        assert torch.equal(v, rv), name
        for _ in range(5):
            V.topk_rows(x, k, largest=largest)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            V.topk_rows(x, k, largest=largest)
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:32s} {e0.elapsed_time(e1) * 1000 / a.iters:8.1f} us")


if __name__ == "__main__":
    main()
