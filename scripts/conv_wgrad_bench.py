"""Mask R-CNN (1 img, 800 x 1344) convolution weight gradients: MIOpen (torch
convolution_backward, weight only) vs csrc/convwg.hip, per shape, with TFLOP/s."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mxtrain.ops import convwg

N = int(os.environ.get("IMGS", "1"))
WGRAD_ONLY = os.environ.get("WGRAD_ONLY", "0") == "1"   # split sweeps: skip the dgrad / fwd columns
# split-K planning A/B (ops/convwg.py k_splits): SPLIT_AB="TILES:WGS:MAX[:MIN_NK] ..." times
# the forward and the input gradient under each setting of SPLIT_TILES / WGS / MAX / MIN_NK
SPLIT_AB = [tuple(int(t) for t in c.split(":")) for c in os.environ.get("SPLIT_AB", "").split()]
# name, Cin, Cout, H_in, W_in, k, stride, pad, count per step
SHAPES = [
    ("res3.conv1 s2", 256, 128, 200, 336, 1, 2, 0, 1),
    ("res3.conv2", 128, 128, 100, 168, 3, 1, 1, 4),
    ("res3.conv3", 128, 512, 100, 168, 1, 1, 0, 4),
    ("res3.short s2", 256, 512, 200, 336, 1, 2, 0, 1),
    ("res3.conv1", 512, 128, 100, 168, 1, 1, 0, 3),
    ("res4.conv1 s2", 512, 256, 100, 168, 1, 2, 0, 1),
    ("res4.conv2", 256, 256, 50, 84, 3, 1, 1, 6),
    ("res4.conv3", 256, 1024, 50, 84, 1, 1, 0, 6),
    ("res4.short s2", 512, 1024, 100, 168, 1, 2, 0, 1),
    ("res4.conv1", 1024, 256, 50, 84, 1, 1, 0, 5),
    ("res5.conv1 s2", 1024, 512, 50, 84, 1, 2, 0, 1),
    ("res5.conv2", 512, 512, 25, 42, 3, 1, 1, 3),
    ("res5.conv3", 512, 2048, 25, 42, 1, 1, 0, 3),
    ("res5.short s2", 1024, 2048, 50, 84, 1, 2, 0, 1),
    ("res5.conv1", 2048, 512, 25, 42, 1, 1, 0, 2),
    ("fpn.lat2", 256, 256, 200, 336, 1, 1, 0, 1),
    ("fpn.lat3", 512, 256, 100, 168, 1, 1, 0, 1),
    ("fpn.lat4", 1024, 256, 50, 84, 1, 1, 0, 1),
    ("fpn.lat5", 2048, 256, 25, 42, 1, 1, 0, 1),
    ("fpn.out2 / rpn P2", 256, 256, 200, 336, 3, 1, 1, 2),
    ("fpn.out3 / rpn P3", 256, 256, 100, 168, 3, 1, 1, 2),
    ("fpn.out4 / rpn P4", 256, 256, 50, 84, 3, 1, 1, 2),
    ("fpn.out5 / rpn P5", 256, 256, 25, 42, 3, 1, 1, 2),
    ("rpn P6", 256, 256, 13, 21, 3, 1, 1, 1),
    ("mask head (64 rois)", 256, 256, 14, 14, 3, 1, 1, 4),
    ("rpn level canvas", 256, 256, 301, 336, 3, 1, 1, 1),
]


def timeit(fn, it=10, reps=5):
    """GPU time per call: `it` calls captured in one hipGraph, replayed `reps` times (the
    eager calls of the small convs are host-bound)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(it):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / (it * reps)


tot_m = tot_h = tot_dm = tot_dh = tot_fm = tot_fh = 0.0
cl = torch.channels_last
# weight-gradient split planning A/B (ops/convwg.py plan_splits): WG_AB="TARGET_WGS:MIN_STEPS ..."
WG_AB = [tuple(int(t) for t in c.split(":")) for c in os.environ.get("WG_AB", "").split()]
if WG_AB:
    tot = [0.0] * len(WG_AB)
    print(f"{'wgrad split A/B (us)':24s} {'N':>3s} " + " ".join(f"{'%d:%d' % c:>9s}" for c in WG_AB))
    for name, Cin, Cout, H, W, k, s, p, cnt in SHAPES:
        n = 64 * N if name.startswith("mask") else N
        x = torch.randn(n, Cin, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        dy = torch.randn(n, Cout, OH, OW, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        cols = []
        for i, (tw, ms) in enumerate(WG_AB):
            convwg.TARGET_WGS, convwg.MIN_STEPS = tw, ms
            t = timeit(lambda: convwg.conv_wgrad(dy, x, (Cout, Cin, k, k), s, p, 1))
            tot[i] += cnt * t
            cols.append(f"{t:9.1f}")
        print(f"{name:24s} {n:3d} " + " ".join(cols), flush=True)
    print("per step (counts): " + ", ".join(f"{'%d:%d' % c} {t:.0f} us" for c, t in zip(WG_AB, tot)))
    sys.exit(0)
if SPLIT_AB:
    tot = [[0.0, 0.0] for _ in SPLIT_AB]
    print(f"{'split-K A/B (fwd | dgrad us)':26s} {'N':>3s} " + " ".join(f"{':'.join(map(str, c)):>17s}" for c in SPLIT_AB))
    for name, Cin, Cout, H, W, k, s, p, cnt in SHAPES:
        if name.startswith("rpn P") or name in ("res3.conv1 s2", "res3.short s2", "fpn.lat2"):
            continue
        n = 64 * N if name.startswith("mask") else N
        x = torch.randn(n, Cin, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(Cout, Cin, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
        bias = torch.randn(Cout, device="cuda").to(torch.bfloat16)
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        dy = torch.randn(n, Cout, OH, OW, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        dg_ok = convwg.dgrad_supported(w, tuple(x.shape), s, p, 1)
        cols = []
        for i, c in enumerate(SPLIT_AB):
            convwg.SPLIT_TILES, convwg.SPLIT_WGS, convwg.SPLIT_MAX = c[:3]
            convwg.SPLIT_MIN_NK = c[3] if len(c) > 3 else 0
            tf = timeit(lambda: convwg.conv_fwd(x, w, bias, None, True, s, p, 1))
            td = timeit(lambda: convwg.conv_dgrad(dy, w, tuple(x.shape), s, p, 1)) if dg_ok else 0.0
            tot[i][0] += cnt * tf
            tot[i][1] += cnt * td
            cols.append(f"{tf:8.1f} {td:8.1f}")
        print(f"{name:26s} {n:3d} " + " ".join(cols), flush=True)
    print("per step (counts, fwd / dgrad): " + ", ".join(f"{':'.join(map(str, c))} {a:.0f} / {b:.0f} us"
                                                        for c, (a, b) in zip(SPLIT_AB, tot)))
    sys.exit(0)
print(f"{'conv':22s} {'N':>3s} {'MIOpen us':>10s} {'convwg us':>10s} {'TF/s mi':>8s} {'TF/s wg':>8s}  splits  maxrel"
      f"   | dgrad: MIOpen us  convdg us  maxrel   | fwd+bias: MIOpen us  convfw us  maxrel")
for name, Cin, Cout, H, W, k, s, p, cnt in SHAPES:
    n = 64 * N if name.startswith("mask") else N
    x = torch.randn(n, Cin, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(Cout, Cin, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(n, Cout, OH, OW, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    mi = lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                     [False, True, False])
    wg = lambda: convwg.conv_wgrad(dy, x, (Cout, Cin, k, k), s, p, 1)
    tm, th = timeit(mi), timeit(wg)
    ref = mi()[1].float()
    got = wg().float()
    rel = ((got - ref).abs().max() / ref.abs().max()).item()
    fl = 2.0 * n * OH * OW * Cout * Cin * k * k
    T = n * OH * OW
    ntiles = k * k * (Cout // 128) * (Cin // 128)
    if WGRAD_ONLY:
        print(f"{name:22s} {n:3d} {tm:10.1f} {th:10.1f} {fl / tm / 1e6:8.1f} {fl / th / 1e6:8.1f}  "
              f"{convwg.plan_splits(T, ntiles):6d}  {rel:.2e}  x{cnt}", flush=True)
        tot_m += cnt * tm
        tot_h += cnt * th
        continue
    dmi = lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                      [True, False, False])
    dwg = lambda: convwg.conv_dgrad(dy, w, tuple(x.shape), s, p, 1)
    dtm, dth = timeit(dmi), timeit(dwg)
    dref = dmi()[0].float()
    drel = ((dwg().float() - dref).abs().max() / dref.abs().max()).item()
    bias = torch.randn(Cout, device="cuda").to(torch.bfloat16)
    from mxtrain.ops.epilogue import bias_act
    fmi = lambda: bias_act(torch.nn.functional.conv2d(x, w, None, s, p), bias, None, True)
    ffw = lambda: convwg.conv_fwd(x, w, bias, None, True, s, p, 1)
    ftm, fth = timeit(fmi), timeit(ffw)
    fref = fmi().float()
    frel = ((ffw().float() - fref).abs().max() / fref.abs().max()).item()
    tot_fm += cnt * ftm
    tot_fh += cnt * fth
    print(f"{name:22s} {n:3d} {tm:10.1f} {th:10.1f} {fl / tm / 1e6:8.1f} {fl / th / 1e6:8.1f}  {convwg.plan_splits(T, ntiles):6d}  {rel:.2e}"
          f"   | {dtm:8.1f} {dth:9.1f}  {drel:.2e}   | {ftm:8.1f} {fth:9.1f}  {frel:.2e}  x{cnt}", flush=True)
    tot_m += cnt * tm
    tot_h += cnt * th
    if not name.startswith(("res3.conv1 s2", "res3.short", "fpn.lat2")):   # inputs without a gradient
        tot_dm += cnt * dtm
        tot_dh += cnt * dth
print(f"per step (counts): wgrad MIOpen {tot_m:.0f} us, convwg {tot_h:.0f} us; "
      f"dgrad MIOpen {tot_dm:.0f} us, convdg {tot_dh:.0f} us; fwd+bias MIOpen {tot_fm:.0f} us, convfw {tot_fh:.0f} us")
