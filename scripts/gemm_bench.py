"""Time every GEMM of one GPT-2 345M training step (mbs 4, seq 1024) in the exact call
form the model uses (hipBLASLt through torch), report TFLOP/s per shape and the step total.

    python scripts/gemm_bench.py [--iters 50]
"""
import argparse
import json

import torch


def bench(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tokens", type=int, default=4096)
    a = ap.parse_args()
    torch.backends.cuda.preferred_blas_library("hipblaslt")
    T, h, f, V, L = a.tokens, 1024, 4096, 50304, 24
    dev = "cuda"
    bf = torch.bfloat16
    rows = []
    total = 0.0
    for name, n_out, k_in, per_step in (("qkv", 3 * h, h, L), ("proj", h, h, L), ("fc1", f, h, L), ("fc2", h, f, L),
                                         ("head", V, h, 1)):
        W = torch.randn(n_out, k_in, device=dev, dtype=bf) * 0.02
        b = torch.zeros(n_out, device=dev, dtype=bf)
        x = torch.randn(T, k_in, device=dev, dtype=bf)
        dy = torch.randn(T, n_out, device=dev, dtype=bf)
        g = torch.zeros(n_out, k_in, device=dev, dtype=bf)
        fl = 2.0 * T * n_out * k_in
        for kind, fn in (("fwd", lambda: torch.addmm(b, x, W.t())),
                         ("dgrad", lambda: torch.mm(dy, W)),
                         ("wgrad", lambda: g.addmm_(dy.t(), x))):
            if name == "head" and kind == "fwd":
                fn = lambda: torch.mm(x, W.t())  # noqa: E731
            ms = bench(fn, a.iters)
            tf = fl / ms / 1e9
            rows.append({"gemm": name, "kind": kind, "M": T if kind != "wgrad" else n_out,
                         "N": n_out if kind == "fwd" else (k_in if kind == "dgrad" else k_in),
                         "K": k_in if kind == "fwd" else (n_out if kind == "dgrad" else T),
                         "ms": round(ms, 4), "tflops": round(tf, 1), "ms_per_step": round(ms * per_step, 3)})
            total += ms * per_step
    for r in rows:
        print(json.dumps(r))
    print(json.dumps({"gemm_ms_per_step": round(total, 3)}))


if __name__ == "__main__":
    main()
