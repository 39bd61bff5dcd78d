#!/usr/bin/env python3
"""Batched NMS (ops/vision.py batched_nms_sorted -> csrc/vision.hip nms_mask_kernel +
nms_keep_kernel) at the RPN shapes of a Mask R-CNN training step: P problems (images x 5 FPN
levels) of N score-sorted boxes clustered around objects, IoU 0.7, up to max_out kept.
Times the pair with events and checks the kept lists against a greedy CPU reference.
    python scripts/nms_bench.py [--p 5] [--n 2000] [--max-out 2000]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def problems(P, N, gen):
    ctr = torch.rand(P, 40, 2, generator=gen) * 1000                     # 40 objects per problem
    pick = torch.randint(0, 40, (P, N), generator=gen)
    c = torch.gather(ctr, 1, pick[..., None].expand(P, N, 2)) + torch.randn(P, N, 2, generator=gen) * 12
    wh = 20 + torch.rand(P, N, 2, generator=gen) * 120
    return torch.cat([c - wh / 2, c + wh / 2], -1)


def greedy(boxes, thr, max_out):
    x1, y1, x2, y2 = boxes.unbind(1)
    area = (x2 - x1) * (y2 - y1)
    alive = torch.ones(len(boxes), dtype=torch.bool)
    keep = []
    for i in range(len(boxes)):
        if not alive[i]:
            continue
        keep.append(i)
        if len(keep) == max_out:
            break
        iw = (torch.minimum(x2[i], x2) - torch.maximum(x1[i], x1)).clamp(min=0)
        ih = (torch.minimum(y2[i], y2) - torch.maximum(y1[i], y1)).clamp(min=0)
        inter = iw * ih
        iou = inter / (area[i] + area - inter).clamp(min=1e-12)
        sup = iou > thr
        sup[: i + 1] = False
        alive &= ~sup
    return keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, default=5)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--max-out", type=int, default=2000)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--par", type=int, default=-1, help="mx_nms_par setting (-1: library default)")
    a = ap.parse_args()
    from mxtrain.ops import _lib
    from mxtrain.ops import vision as V
    _lib._fn("mx_nms_par")(a.par)
    par = _lib._fn("mx_nms_par")(-1)
    gen = torch.Generator().manual_seed(0)
    b = problems(a.p, a.n, gen)
    bd = b.cuda()
    keep, nkeep = V.batched_nms_sorted(bd, None, 0.7, a.max_out)
    torch.cuda.synchronize()
    for p in range(min(a.p, 2)):
        ref = greedy(b[p], 0.7, a.max_out)
        got = keep[p, : int(nkeep[p])].cpu().tolist()
        assert got == ref, (p, len(got), len(ref))
    for _ in range(5):
        V.batched_nms_sorted(bd, None, 0.7, a.max_out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        V.batched_nms_sorted(bd, None, 0.7, a.max_out)
    e1.record()
    torch.cuda.synchronize()
    print(f"nms par {par} P {a.p} N {a.n} max_out {a.max_out}: {e0.elapsed_time(e1) * 1000 / a.iters:.1f} us per call "
          f"(kept {nkeep.float().mean().item():.0f} per problem; matches greedy)")


if __name__ == "__main__":
    main()
