"""Microbenchmark: the 1 x 1 stride-1 Cin = 64 convolutions of ResNet-50 res2 (batch 256,
56 x 56) -- MIOpen backward-data / backward-weights vs one plain GEMM on the NHWC views."""
import torch

cl = torch.channels_last
N, H, W = 256, 56, 56
M = N * H * W


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for Cin, Cout in [(64, 64), (64, 256)]:
    x = torch.randn(N, Cin, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(N, Cout, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = torch.randn(Cout, Cin, 1, 1, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    a = dy.permute(0, 2, 3, 1).reshape(M, Cout)
    xb = x.permute(0, 2, 3, 1).reshape(M, Cin)
    b = w.reshape(Cout, Cin)
    cb = lambda m: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, m)
    t_dg_mi = timeit(lambda: cb([True, False, False]))
    t_dg_mm = timeit(lambda: torch.mm(a, b))
    t_wg_mi = timeit(lambda: cb([False, True, False]))
    t_wg_mm = timeit(lambda: torch.mm(a.t(), xb))
    ref = cb([False, True, False])[1].float().reshape(Cout, Cin)
    err = (torch.mm(a.t(), xb).float() - ref).abs().max().item() / ref.abs().max().item()
    print(f"Cin {Cin} Cout {Cout}: dgrad MIOpen {t_dg_mi:7.1f} us  GEMM {t_dg_mm:7.1f} us | "
          f"wgrad MIOpen {t_wg_mi:7.1f} us  GEMM {t_wg_mm:7.1f} us (rel err {err:.1e})", flush=True)
