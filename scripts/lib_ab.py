#!/usr/bin/env python3
"""Interleaved same-box A/B of two builds of the kernel library on the GPT-2 345M attention
shape (B 4, S 1024, 16 heads, D 64, causal, dropout 0.1): each round runs one child process
per library (A, B, A, B, ...), and each child times the forward and the backward over
200 calls after warm-up (events), so DVFS drift between the two builds averages out.
    python scripts/lib_ab.py --a mxtrain/lib/ab/libmxkernels_a.so [--b mxtrain/lib/libmxkernels.so]
        [--rounds 4]"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, REPO)
    import torch
    from mxtrain.ops import _lib
    _lib.LIB_PATH = os.path.abspath(lib)
    from mxtrain.ops import attention as A
    B, S, H, D, p = 4, 1024, 16, 64, 0.1
    dev = "cuda"
    torch.manual_seed(0)
    qkv = torch.randn(B * S, 3 * H * D, device=dev).to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    do = torch.randn(B * S, H * D, device=dev).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    sd = torch.tensor([7], dtype=torch.int32, device=dev)
    fwd = lambda: A.attn_fwd(q, k, v, B, S, H, H, D, True, dropout_p=p, seed_t=sd)
    o, lse, dm = fwd()
    bwd = lambda: A.attn_bwd(do, q, k, v, o, lse, B, S, H, H, D, True, dq=dqkv[:, :H * D],
                             dk=dqkv[:, H * D:2 * H * D], dv=dqkv[:, 2 * H * D:], dmask=dm, dropout_p=p)
    res = {}
    for name, fn in (("fwd", fwd), ("bwd", bwd)):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(200):
            fn()
        b.record()
        torch.cuda.synchronize()
        res[name] = a.elapsed_time(b) * 1000 / 200
    bwd()
    torch.cuda.synchronize()
    res["o_sum"] = float(o.float().abs().sum())
    res["g_sum"] = float(dqkv.float().abs().sum())
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default="")
    ap.add_argument("--b", default=os.path.join(REPO, "mxtrain", "lib", "libmxkernels.so"))
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--child", default="")
    a = ap.parse_args()
    if a.child:
        return child(a.child)
    runs = {"A": [], "B": []}
    for r in range(a.rounds):
        for tag, lib in (("A", a.a), ("B", a.b)):
            out = subprocess.run([sys.executable, __file__, "--child", lib], stdout=subprocess.PIPE, text=True,
                                 timeout=300, check=True).stdout.strip().splitlines()[-1]
            d = json.loads(out)
            runs[tag].append(d)
            print(f"round {r} {tag}: fwd {d['fwd']:.2f} us  bwd {d['bwd']:.2f} us  "
                  f"|o| {d['o_sum']:.6g}  |dqkv| {d['g_sum']:.6g}", flush=True)
    for tag in ("A", "B"):
        f = sorted(x["fwd"] for x in runs[tag])
        b = sorted(x["bwd"] for x in runs[tag])
        print(f"{tag}: fwd median {f[len(f) // 2]:.2f} us, bwd median {b[len(b) // 2]:.2f} us")


if __name__ == "__main__":
    main()
