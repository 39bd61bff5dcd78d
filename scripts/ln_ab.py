#!/usr/bin/env python3
"""LN / BDA-LN kernels at the GPT-2 345M shape [4096, 1024] (dropout 0.1): us per call of
the forward and of the backward (+ its column reduction), each timed as a hipGraph of 20
calls, for the backward's rows-per-wave settings 2 and 4.
    python scripts/ln_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import _lib  # noqa: E402
from mxtrain.ops import norm as N  # noqa: E402


def graph_us(fn, n=20, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (n * reps)


def main():
    R, C, p = 4096, 1024, 0.1
    dev = "cuda"
    bf = lambda *s: torch.randn(*s, device=dev).to(torch.bfloat16)
    x, res, dy, dres = bf(R, C), bf(R, C), bf(R, C), bf(R, C)
    bias, g, b = bf(C) * 0.1, 1 + 0.1 * bf(C), 0.1 * bf(C)
    seed = torch.tensor([11], dtype=torch.int32, device=dev)
    h, y, mean, rstd = N.bda_norm_fwd(x, bias, res, g, b, p=p, seed_t=seed, salt=3)
    outs = [torch.zeros(C, dtype=torch.bfloat16, device=dev) for _ in range(3)]
    fwd = lambda: N.bda_norm_fwd(x, bias, res, g, b, p=p, seed_t=seed, salt=3)
    bwd = lambda: N.norm_bwd(dy, dres, h, mean, rstd, g, want_dx=True, p=p, seed_t=seed, salt=3,
                             dgamma=outs[0], dbeta=outs[1], dbias=outs[2])
    t = graph_us(fwd)
    print(f"bda_ln_fwd: {t:.2f} us  ({4 * R * C * 2 / 1e3 / t:.0f} GB/s)", flush=True)
    for rpw, mb in ((2, 512), (1, 512), (1, 1024), (2, 256), (4, 256), (2, 512), (1, 1024)):
        old = _lib._fn("mx_norm_bwd_rows_per_wave")(rpw)
        oldb = _lib._fn("mx_norm_bwd_max_blocks")(mb)
        t = graph_us(bwd)
        print(f"ln_bwd+colreduce rpw {rpw} max_blocks {mb}: {t:.2f} us  "
              f"({5 * R * C * 2 / 1e3 / t:.0f} GB/s of row traffic)", flush=True)
        _lib._fn("mx_norm_bwd_rows_per_wave")(old)
        _lib._fn("mx_norm_bwd_max_blocks")(oldb)


if __name__ == "__main__":
    main()
