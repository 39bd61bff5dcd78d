#!/usr/bin/env python3
"""HBM roofline of this MI355X for streaming kernels (csrc/membw.hip): achieved TB/s per
access mix (R read streams, W write streams of fp32 float4), default vs non-temporal
access, over grid sizes; then the step's memory-bound kernels at their real sizes against
it: AdamW (28 B/element at GPT-2 345M) and torch's copy_ for reference.
    python scripts/hbm_probe.py [--mib 1024]"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import _lib  # noqa: E402


def timed(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024, help="MiB per stream")
    a = ap.parse_args()
    dev = "cuda"
    n4 = a.mib * (1 << 20) // 16
    bufs = [torch.ones(n4 * 4, device=dev) for _ in range(8)]
    best = {}
    print(f"# membw: {a.mib} MiB per stream, fp32 float4 vectors, 4 in flight per stream per thread")
    print(f"{'mix':>6} {'nt':>3} {'blocks':>7} {'us':>9} {'TB/s':>6}")
    for R, W in ((1, 0), (2, 0), (0, 1), (1, 1), (2, 1), (3, 3), (4, 4)):
        src = torch.tensor([b.data_ptr() for b in bufs[:max(R, 1)]], dtype=torch.int64, device=dev)
        dst = torch.tensor([b.data_ptr() for b in bufs[4:4 + max(W, 1)]], dtype=torch.int64, device=dev)
        for nt in (0, 1):
            for blocks in (2048, 8192, 32768, 131072):
                fn = lambda: _lib.call("mx_membw", R, W, nt, src.data_ptr(), dst.data_ptr(), n4, blocks,  # noqa: E731
                                       _lib.stream())
                us = timed(fn)
                tbs = (R + W) * n4 * 16 / (us * 1e-6) / 1e12
                best[(R, W)] = max(best.get((R, W), 0.0), tbs)
                print(f"{R}r{W}w {nt:>4} {blocks:>7} {us:9.1f} {tbs:6.2f}", flush=True)
    print("\n# best per mix (TB/s): " + ", ".join(f"{r}r{w}w {v:.2f}" for (r, w), v in best.items()))
    del bufs
    torch.cuda.empty_cache()
    # torch copy_ (1r1w) for reference
    x = torch.empty(n4 * 4, device=dev)
    y = torch.empty_like(x)
    us = timed(lambda: y.copy_(x))
    print(f"torch copy_ fp32 {a.mib} MiB: {us:.1f} us, {2 * x.numel() * 4 / us / 1e6:.2f} TB/s")
    del x, y
    torch.cuda.empty_cache()
    # AdamW at GPT-2 345M (354.87 M elements, 28 B / element) through the shipping launch
    from mxtrain.ops import optim as O
    n = 354_871_296 // 64 * 64
    m = torch.randn(n, device=dev)
    e1 = torch.zeros(n, device=dev)
    e2 = torch.zeros(n, device=dev)
    g = torch.randn(n, device=dev, dtype=torch.bfloat16)
    p = torch.empty(n, device=dev, dtype=torch.bfloat16)
    h = torch.tensor([1e-4, 0.9, 0.999, 1e-8, 0.01, 0.1, 0.001, 1.0, 1.0], device=dev)
    ns = torch.ones(1, device=dev)
    us = timed(lambda: O.adamw_step(m, e1, e2, g, p, h, normsq=ns))
    print(f"adamw (shipping launch) n={n}: {us:.1f} us, {28 * n / us / 1e6:.2f} TB/s "
          f"(3r3w-mix roofline {best[(3, 3)]:.2f} TB/s -> {28 * n / best[(3, 3)] / 1e6:.0f} us)")


if __name__ == "__main__":
    main()
