"""Compare GEMM implementations for the GPT-2 345M weight-gradient / small shapes:
hipBLASLt vs rocBLAS, and split-K (batched GEMM over K chunks + fp32 reduction)."""
import json
import torch


def bench(fn, iters=50):
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


T = 4096
bf = torch.bfloat16
for lib in ("hipblaslt", "rocblas"):
    torch.backends.cuda.preferred_blas_library(lib)
    for name, n_out, k_in in (("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096)):
        dy = torch.randn(T, n_out, device="cuda", dtype=bf)
        x = torch.randn(T, k_in, device="cuda", dtype=bf)
        g = torch.zeros(n_out, k_in, device="cuda", dtype=bf)
        W = torch.randn(n_out, k_in, device="cuda", dtype=bf)
        fl = 2.0 * T * n_out * k_in
        res = {"lib": lib, "gemm": name}
        res["wgrad"] = round(fl / bench(lambda: g.addmm_(dy.t(), x)) / 1e9, 1)
        res["fwd"] = round(fl / bench(lambda: torch.mm(x, W.t())) / 1e9, 1)
        res["dgrad"] = round(fl / bench(lambda: torch.mm(dy, W)) / 1e9, 1)
        for S in (2, 4, 8):
            dys = dy.view(S, T // S, n_out).transpose(1, 2)
            xs = x.view(S, T // S, k_in)
            def f():
                p = torch.bmm(dys, xs)
                g.add_(p.sum(0, dtype=torch.float32))
            res[f"wgrad_splitk{S}"] = round(fl / bench(f) / 1e9, 1)
        print(json.dumps(res), flush=True)
