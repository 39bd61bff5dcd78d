#!/usr/bin/env python3
"""In-kernel attention-dropout keep bits vs the pre-pass images, at the GPT-2 345M shapes
(B 4, S 1024, 16 heads, D 64, causal, p 0.1), same box, interleaved rounds:

  pre-pass arm: the step's 24-layer mask launch (mx_flash_dropmask_layers) / 24 + the
                shipping forward reading the image (mx_flash_fwd)
  in-kernel arm: the forward hashing its own bits (mx_flash_fwd_dgen), no pre-pass

Outputs must be bit-identical.  Only the forward is built in-kernel: the backward kernels
(dQ, dK/dV) would pay the same hashing again on the same VALU-bound loops, so if the forward
alone costs more than the whole pre-pass share, the in-kernel design loses.
    python scripts/attn_dropout_ab.py [--rounds 5] [--iters 50]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import _lib  # noqa: E402
from mxtrain.ops import attention as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    B, S, H, D, L, p, salt = 4, 1024, 16, 64, 24, 0.1, 50000
    dev = "cuda"
    qkv = torch.randn(B * S, 3 * H * D, device=dev).to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    seed = torch.tensor([123456], dtype=torch.int32, device=dev)
    o2 = torch.empty(B * S, H * D, dtype=torch.bfloat16, device=dev)
    lse2 = torch.empty(B, H, S, dtype=torch.float32, device=dev)

    def dgen():
        _lib.call("mx_flash_fwd_dgen", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), q.stride(0), k.stride(0), v.stride(0),
                  _lib.ptr(o2), o2.stride(0), _lib.ptr(lse2), B, S, H, H, D, 1, None, 1.0 / D ** 0.5,
                  _lib.ptr(seed), salt, p, 0, H, _lib.stream())

    masks = A.dropmask_layers(B, S, H, p, seed, salt, L)
    o1, lse1, _ = A.attn_fwd(q, k, v, B, S, H, H, D, True, dmask=masks[0])
    dgen()
    torch.cuda.synchronize()
    same = torch.equal(o1, o2) and torch.equal(lse1, lse2)
    print(f"bit-identical outputs: {same}")

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000 / n

    arms = {"prepass_24_layers": lambda: A.dropmask_layers(B, S, H, p, seed, salt, L),
            "fwd_with_image": lambda: A.attn_fwd(q, k, v, B, S, H, H, D, True, dmask=masks[0]),
            "fwd_inkernel_bits": dgen,
            "fwd_no_dropout": lambda: A.attn_fwd(q, k, v, B, S, H, H, D, True)}
    res = {n: [] for n in arms}
    for _ in range(a.rounds):
        for n, fn in arms.items():
            fn()
            res[n].append(timed(fn, a.iters))
    med = {n: statistics.median(v) for n, v in res.items()}
    for n, t in med.items():
        print(f"{n:22s} {t:8.2f} us  (rounds: {', '.join(f'{x:.2f}' for x in res[n])})")
    pre = med["prepass_24_layers"] / L
    print(f"per layer: pre-pass share {pre:.2f} + forward {med['fwd_with_image']:.2f} = "
          f"{pre + med['fwd_with_image']:.2f} us   vs   in-kernel forward {med['fwd_inkernel_bits']:.2f} us")
    print(f"in-kernel forward overhead over the image forward: {med['fwd_inkernel_bits'] - med['fwd_with_image']:+.2f} us "
          f"per layer (the pre-pass share it would remove: {pre:.2f} us; dQ and dK/dV would add their own hashing)")


if __name__ == "__main__":
    main()
