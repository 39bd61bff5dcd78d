#!/usr/bin/env python3
"""A/B of the D 64 query-major key-tile size (mx_flash_qmajor_bk) at the GPT-2 345M
attention shape (B 4, S 1024, 16 heads, causal, dropout 0.1): us per forward and per
backward call (event timing, 50 calls after warm-up), plus equality of the outputs.
    python scripts/attn_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import _lib  # noqa: E402
from mxtrain.ops import attention as A  # noqa: E402


def main():
    B, S, H, D, p = 4, 1024, 16, 64, 0.1
    dev = "cuda"
    torch.manual_seed(0)
    qkv = torch.randn(B * S, 3 * H * D, device=dev).to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    do = torch.randn(B * S, H * D, device=dev).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    sd = torch.tensor([7], dtype=torch.int32, device=dev)
    flops_f = 4 * B * H * S * S * D / 2
    ref = None
    for fbk, qbk in ((64, 64), (128, 128), (64, 64), (128, 128)):
        _lib._fn("mx_flash_qmajor_bk")(fbk, qbk)
        fwd = lambda: A.attn_fwd(q, k, v, B, S, H, H, D, True, dropout_p=p, seed_t=sd)
        o, lse, dm = fwd()
        bwd = lambda: A.attn_bwd(do, q, k, v, o, lse, B, S, H, H, D, True, dq=dqkv[:, :H * D],
                                 dk=dqkv[:, H * D:2 * H * D], dv=dqkv[:, 2 * H * D:], dmask=dm, dropout_p=p)
        bwd()
        out = (o.clone(), dqkv.clone())
        if ref is None:
            ref = out
        err_o = (out[0].float() - ref[0].float()).abs().max().item()
        err_g = (out[1].float() - ref[1].float()).abs().max().item()
        res = {}
        for name, fn in (("fwd", fwd), ("bwd", bwd)):
            for _ in range(10):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name] = e0.elapsed_time(e1) * 1000 / 50
        print(f"bk fwd {fbk} dq {qbk}: fwd {res['fwd']:.1f} us ({flops_f / res['fwd'] / 1e6:.0f} TF)  "
              f"bwd {res['bwd']:.1f} us ({2.5 * flops_f / res['bwd'] / 1e6:.0f} TF)  "
              f"fwd+bwd {3.5 * flops_f / (res['fwd'] + res['bwd']) / 1e6:.0f} TF  "
              f"max|dO| {err_o:.3g} max|dQKV| {err_g:.3g}", flush=True)


if __name__ == "__main__":
    main()
