import sys, torch
sys.path.insert(0, "/root/repo")
from mxtrain.ops import stem as S
torch.manual_seed(0)
mean, std = (123.675, 116.28, 103.53), (58.395, 57.12, 57.375)
for (N, H, W) in [(4, 800, 1344), (4, 1344, 800), (1, 800, 1344)]:
    img = torch.randint(0, 256, (N, 3, H, W), dtype=torch.uint8, device="cuda")
    wf = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).to(torch.bfloat16)
    bf = (torch.randn(64, device="cuda") * 0.1).to(torch.bfloat16)
    y = S.stem_pool(img, wf, bf, mean, std)
    torch.cuda.synchronize()
    ref = S.stem_pool_ref(img, wf, bf, mean, std)
    print(N, H, W, "eager err", (y.float() - ref.float()).abs().max().item(), flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            y2 = S.stem_pool(img, wf, bf, mean, std)
    g.replay()
    torch.cuda.synchronize()
    print(N, H, W, "graph equal", torch.equal(y, y2), flush=True)

# timing: fused kernel vs normalise + conv (MIOpen) + bias/ReLU + max-pool
import torch.nn.functional as F
for (N, H, W) in [(1, 800, 1344), (4, 800, 1344)]:
    img = torch.randint(0, 256, (N, 3, H, W), dtype=torch.uint8, device="cuda")
    wf = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).to(torch.bfloat16)
    bf = (torch.randn(64, device="cuda") * 0.1).to(torch.bfloat16)
    def fused():
        return S.stem_pool(img, wf, bf, mean, std)
    wcl = wf.contiguous(memory_format=torch.channels_last)
    def unfused():
        x = torch.empty(N, H, W, 3, dtype=torch.bfloat16, device="cuda").permute(0, 3, 1, 2)
        from mxtrain.ops import _lib
        import ctypes
        _lib.call("mx_normalize_u8_nhwc", img.data_ptr(), x.data_ptr(), N, H, W,
                  ctypes.cast((ctypes.c_float * 3)(*mean), ctypes.c_void_p),
                  ctypes.cast((ctypes.c_float * 3)(*[1 / v for v in std]), ctypes.c_void_p), _lib.stream())
        y = F.relu(F.conv2d(x, wcl, bf, 2, 3))
        return F.max_pool2d(y, 3, 2, 1)
    from mxtrain.ops import _lib as L
    for gsz in (256, 512, 1024, 1 << 30):
        L._fn("mx_stem_grid")(gsz)
        for _ in range(3):
            fused()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fused()
        e1.record()
        torch.cuda.synchronize()
        print(f"N={N} fused grid {gsz}: {e0.elapsed_time(e1) * 1000 / 20:.1f} us", flush=True)
    L._fn("mx_stem_grid")(512)
    for name, fn in (("fused", fused), ("unfused", unfused)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"N={N} {name}: {e0.elapsed_time(e1) * 1000 / 20:.1f} us", flush=True)
