#!/usr/bin/env python3
"""Do independent branches of a captured hipGraph run concurrently on this ROCm?  Times two
one-wave spin kernels (torch.cuda._sleep) and two half-GPU GEMM pairs, serial on one stream
vs forked onto a second stream, eager and inside a captured graph.  A fork that overlaps
shows ~1x the single-branch time for the spin pair; a graph that serialises branches shows 2x.
    python scripts/graph_branch_probe.py"""
import json

import torch


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    dev = torch.device("cuda")
    side = torch.cuda.Stream()
    cycles = 2_000_000
    a = torch.randn(4096, 1024, device=dev, dtype=torch.bfloat16)
    w1 = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
    w2 = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
    o1 = torch.empty(4096, 1024, device=dev, dtype=torch.bfloat16)
    o2 = torch.empty(4096, 1024, device=dev, dtype=torch.bfloat16)

    def work(kind, s1, s2):
        if kind == "spin":
            with torch.cuda.stream(s1):
                torch.cuda._sleep(cycles)
            with torch.cuda.stream(s2):
                torch.cuda._sleep(cycles)
        else:
            for _ in range(4):
                with torch.cuda.stream(s1):
                    torch.mm(a, w1, out=o1)
                with torch.cuda.stream(s2):
                    torch.mm(a, w2, out=o2)

    def serial(kind):
        cur = torch.cuda.current_stream()
        work(kind, cur, cur)

    def forked(kind):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        work(kind, cur, side)
        cur.wait_stream(side)

    res = {}
    for kind in ("spin", "gemm"):
        res[f"{kind}/eager_serial"] = timed(lambda: serial(kind))
        res[f"{kind}/eager_forked"] = timed(lambda: forked(kind))
        for mode, fn in (("serial", serial), ("forked", forked)):
            g = torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream()
            cs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cs):
                fn(kind)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=cs):
                fn(kind)
            res[f"{kind}/graph_{mode}"] = timed(g.replay)
    for k, v in res.items():
        print(f"{k:22s} {v:9.1f} us")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
