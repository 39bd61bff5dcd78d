#!/usr/bin/env python3
"""Attention kernels alone at GPT-2 345M / GPT-3 6.7B shapes (for rocprofv3 kernel traces
and PMC passes): N iterations of fwd + bwd, optional dropout.
    python scripts/attn_only.py [--shape gpt2|gpt3] [--iters 20] [--dropout 0.1]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import attention as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="gpt2", choices=["gpt2", "gpt3"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dropout", type=float, default=0.0)
    ap.add_argument("--fwd-only", action="store_true")
    ap.add_argument("--qbk", default="", help="key-tile rows of the D 64 forward / dQ kernels, e.g. 64,128")
    ap.add_argument("--k128", type=int, default=-1,
                    help="D 128 dK/dV variant: 0 single pass, 1 two column-half passes")
    a = ap.parse_args()
    if a.k128 >= 0:
        from mxtrain.ops import _lib
        _lib._fn("mx_flash_kmajor128_variant")(a.k128)
    if a.qbk:
        from mxtrain.ops import _lib
        f, q = (int(x) for x in a.qbk.split(","))
        _lib._fn("mx_flash_qmajor_bk")(f, q)
    B, S, H, D = (4, 1024, 16, 64) if a.shape == "gpt2" else (2, 2048, 32, 128)
    dev = "cuda"
    torch.manual_seed(0)
    qkv = torch.randn(B * S, 3 * H * D, device=dev).to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    do = torch.randn(B * S, H * D, device=dev).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    sd = torch.tensor([7], dtype=torch.int32, device=dev)
    for _ in range(a.iters):
        o, lse, dm = A.attn_fwd(q, k, v, B, S, H, H, D, True, dropout_p=a.dropout, seed_t=sd)
        if not a.fwd_only:
            A.attn_bwd(do, q, k, v, o, lse, B, S, H, H, D, True, dq=dqkv[:, :H * D], dk=dqkv[:, H * D:2 * H * D],
                       dv=dqkv[:, 2 * H * D:], dmask=dm, dropout_p=a.dropout)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
