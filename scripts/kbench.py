#!/usr/bin/env python3
"""Per-op micro-benchmark of the HIP kernels (and the hipBLASLt GEMMs) at GPT-2 345M
shapes (b=4, s=1024, h=1024, 16 heads) -- interleaved rounds in one process, median of
N, with achieved bandwidth / TFLOP/s.  Usage: python scripts/kbench.py [--only attn]"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import attention as A  # noqa: E402
from mxtrain.ops import fused as Fu  # noqa: E402
from mxtrain.ops import norm as N  # noqa: E402
from mxtrain.ops import optim as O  # noqa: E402


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--D", type=int, default=64)
    args = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    B, S, H, D = args.B, args.S, args.H, args.D
    T, h = B * S, H * D
    bf = torch.bfloat16
    res = {}

    def rec(name, us, bytes_=None, flops=None):
        r = {"us": round(us, 2)}
        if bytes_:
            r["GB/s"] = round(bytes_ / us / 1e3, 1)
        if flops:
            r["TFLOP/s"] = round(flops / us / 1e6, 1)
        res[name] = r
        print(f"{name:28s} {us:9.2f} us  " + "  ".join(f"{k}={v}" for k, v in r.items() if k != "us"),
              flush=True)

    want = lambda k: (not args.only) or k in args.only.split(",")
    if want("attn"):
        qkv = torch.randn(T, 3 * h, device=dev).to(bf)
        q, k, v = qkv[:, :h], qkv[:, h:2 * h], qkv[:, 2 * h:]
        fl = 4 * B * H * S * S * D / 2
        o, lse, _ = A.attn_fwd(q, k, v, B, S, H, H, D, True)
        rec("attn_fwd causal", timeit(lambda: A.attn_fwd(q, k, v, B, S, H, H, D, True)), flops=fl)
        do = torch.randn(T, h, device=dev).to(bf)
        dqkv = torch.empty_like(qkv)
        rec("attn_bwd causal", timeit(lambda: A.attn_bwd(do, q, k, v, o, lse, B, S, H, H, D, True,
                                                         dq=dqkv[:, :h], dk=dqkv[:, h:2 * h],
                                                         dv=dqkv[:, 2 * h:])), flops=2.5 * fl)
        rec("attn_fwd full", timeit(lambda: A.attn_fwd(q, k, v, B, S, H, H, D, False)), flops=2 * fl)
        sd = torch.tensor([7], dtype=torch.int32, device=dev)
        o, lse, dm = A.attn_fwd(q, k, v, B, S, H, H, D, True, dropout_p=0.1, seed_t=sd)
        rec("attn_fwd causal drop0.1", timeit(lambda: A.attn_fwd(q, k, v, B, S, H, H, D, True, dropout_p=0.1,
                                                                 seed_t=sd)), flops=fl)
        rec("attn_bwd causal drop0.1", timeit(lambda: A.attn_bwd(do, q, k, v, o, lse, B, S, H, H, D, True,
                                                                 dq=dqkv[:, :h], dk=dqkv[:, h:2 * h],
                                                                 dv=dqkv[:, 2 * h:], dmask=dm, dropout_p=0.1)),
            flops=2.5 * fl)
    if want("attn128"):   # GPT-3 6.7B shapes: B=2, S=2048, H=32, D=128
        B2, S2, H2, D2 = 2, 2048, 32, 128
        T2, h2 = B2 * S2, H2 * D2
        qkv = torch.randn(T2, 3 * h2, device=dev).to(bf)
        q, k, v = qkv[:, :h2], qkv[:, h2:2 * h2], qkv[:, 2 * h2:]
        fl = 4 * B2 * H2 * S2 * S2 * D2 / 2
        o, lse, _ = A.attn_fwd(q, k, v, B2, S2, H2, H2, D2, True)
        rec("attn128_fwd causal", timeit(lambda: A.attn_fwd(q, k, v, B2, S2, H2, H2, D2, True)), flops=fl)
        do = torch.randn(T2, h2, device=dev).to(bf)
        dqkv = torch.empty_like(qkv)
        rec("attn128_bwd causal", timeit(lambda: A.attn_bwd(do, q, k, v, o, lse, B2, S2, H2, H2, D2, True,
                                                            dq=dqkv[:, :h2], dk=dqkv[:, h2:2 * h2],
                                                            dv=dqkv[:, 2 * h2:])), flops=2.5 * fl)
    if want("norm4096"):
        rows, cols = 4096, 4096
        x = torch.randn(rows, cols, device=dev).to(bf)
        g = torch.ones(cols, device=dev, dtype=bf)
        bb = torch.zeros(cols, device=dev, dtype=bf)
        seed = torch.tensor([1], dtype=torch.int32, device=dev)
        hh_, y_, mean_, rstd_ = N.bda_norm_fwd(x, bb, x, g, bb, p=0.1, seed_t=seed)
        dg, db, dbi = (torch.zeros(cols, device=dev, dtype=bf) for _ in range(3))
        rec("ln_bwd 4096x4096 (bda)", timeit(lambda: N.norm_bwd(x, x, hh_, mean_, rstd_, g, want_dx=True, p=0.1,
                                                                 seed_t=seed, dgamma=dg, dbeta=db, dbias=dbi,
                                                                 accumulate=True)), rows * cols * 2 * 5)
    if want("lnsplit"):   # GPT-2 345M LN backward (fused: register column partials) and BDA forward
        rows, cols = 4096, 1024
        x = torch.randn(rows, cols, device=dev).to(bf)
        g = torch.ones(cols, device=dev, dtype=bf)
        bb = torch.zeros(cols, device=dev, dtype=bf)
        seed = torch.tensor([1], dtype=torch.int32, device=dev)
        hh_, y_, mean_, rstd_ = N.bda_norm_fwd(x, bb, x, g, bb, p=0.1, seed_t=seed)
        dg, db, dbi = (torch.zeros(cols, device=dev, dtype=bf) for _ in range(3))
        rec("ln_bwd 4096x1024", timeit(lambda: N.norm_bwd(x, x, hh_, mean_, rstd_, g, want_dx=True, p=0.1,
                                                          seed_t=seed, dgamma=dg, dbeta=db, dbias=dbi,
                                                          accumulate=True)), rows * cols * 2 * 5)
        rec("bda_ln_fwd 4096x1024", timeit(lambda: N.bda_norm_fwd(x, bb, x, g, bb, p=0.1, seed_t=seed)),
            rows * cols * 2 * 4)
    if want("norm"):
        x = torch.randn(T, h, device=dev).to(bf)
        r_ = torch.randn(T, h, device=dev).to(bf)
        g = torch.ones(h, device=dev, dtype=bf)
        bb = torch.zeros(h, device=dev, dtype=bf)
        seed = torch.tensor([1], dtype=torch.int32, device=dev)
        nb = T * h * 2
        rec("ln_fwd", timeit(lambda: N.layernorm_fwd(x, g, bb)), 2 * nb)
        hh, y, mean, rstd = N.bda_norm_fwd(x, bb, r_, g, bb, p=0.1, seed_t=seed)
        rec("bda_ln_fwd p=0.1", timeit(lambda: N.bda_norm_fwd(x, bb, r_, g, bb, p=0.1, seed_t=seed)), 4 * nb)
        dg, db, dbi = (torch.zeros(h, device=dev, dtype=bf) for _ in range(3))
        rec("bda_ln_bwd p=0.1", timeit(lambda: N.norm_bwd(x, r_, hh, mean, rstd, g, want_dx=True, p=0.1,
                                                          seed_t=seed, dgamma=dg, dbeta=db, dbias=dbi,
                                                          accumulate=True)), 5 * nb)
        q3 = torch.randn(T, 3 * h, device=dev).to(bf)
        rec("colsum [T,3h]", timeit(lambda: N.colsum(q3, dbi[:h].clone().repeat(3), accumulate=True)), 3 * nb)
    if want("gelu"):
        x = torch.randn(T, 4 * h, device=dev).to(bf)
        b = torch.zeros(4 * h, device=dev, dtype=bf)
        nb = T * 4 * h * 2
        rec("bias_gelu_fwd", timeit(lambda: Fu.bias_gelu_fwd(x, b)), 2 * nb)
        dy = torch.randn(T, 4 * h, device=dev).to(bf)
        db = torch.zeros(4 * h, device=dev, dtype=bf)
        rec("bias_gelu_bwd", timeit(lambda: Fu.bias_gelu_bwd(dy, x, b, dbias=db, accumulate=True)), 3 * nb)
    if want("ce"):
        V = 50304
        logits = torch.randn(T, V, device=dev).to(bf)
        labels = torch.randint(0, V, (T,), device=dev)
        lg = logits.clone()
        rec("ce fwd+grad", timeit(lambda: Fu.cross_entropy_fwd_bwd(lg.copy_(logits), labels, 1.0 / T)),
            4 * T * V * 2)
    if want("adam"):
        n = 355_000_000 // 64 * 64
        master = torch.randn(n, device=dev)
        m, v_ = torch.zeros_like(master), torch.zeros_like(master)
        gg = torch.randn(n, device=dev).to(bf)
        p = torch.empty(n, device=dev, dtype=bf)
        hyper = torch.tensor([1e-4, 0.9, 0.999, 1e-8, 0.01, 0.1, 0.001, 1.0, 1.0, 0], device=dev)
        ns = O.sumsq_bf16(gg)
        rec("sumsq 355M", timeit(lambda: O.sumsq_bf16(gg, out=ns)), n * 2)
        rec("adamw 355M", timeit(lambda: O.adamw_step(master, m, v_, gg, p, hyper, ns)), n * 28)
    if want("gemm"):
        shapes = [("qkv fwd", T, 3 * h, h), ("proj fwd", T, h, h), ("fc1 fwd", T, 4 * h, h),
                  ("fc2 fwd", T, h, 4 * h), ("logits", T, 50304, h)]
        for name, M, Nn, K in shapes:
            a = torch.randn(M, K, device=dev).to(bf)
            w = torch.randn(Nn, K, device=dev).to(bf)
            rec(f"mm {name} {M}x{Nn}x{K}", timeit(lambda: torch.mm(a, w.t())), flops=2 * M * Nn * K)
            dy = torch.randn(M, Nn, device=dev).to(bf)
            rec(f"  dgrad {name}", timeit(lambda: torch.mm(dy, w)), flops=2 * M * Nn * K)
            gw = torch.zeros(Nn, K, device=dev, dtype=bf)
            rec(f"  wgrad {name}", timeit(lambda: gw.addmm_(dy.t(), a)), flops=2 * M * Nn * K)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/kbench.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
