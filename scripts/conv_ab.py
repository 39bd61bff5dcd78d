#!/usr/bin/env python3
"""Interleaved same-box A/B of two builds of the kernel library on the implicit-GEMM
convolutions (csrc/convwg.hip) at the Mask R-CNN shapes that dominate the step (the
rpn level canvas, the FPN 3x3 outputs, the res2-res5 3x3 / 1x1 convs): one child process
per library per round (A, B, A, B, ...); each child times forward, input gradient and
weight gradient of every shape over ITERS calls after warm-up (events), and checks both
builds produce the same outputs (max relative difference printed).
    python scripts/conv_ab.py --a mxtrain/lib/ab/libmxkernels_a.so [--b mxtrain/lib/libmxkernels.so]
        [--rounds 3] [--imgs 4]
    python scripts/conv_ab.py --toggle SETTER     # one library, A = setter(0), B = setter(1)"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# name, Cin, Cout, H, W, k, stride, pad  (input resolution at IMGS images of 800 x 1344)
SHAPES = [
    ("rpn canvas 3x3", 256, 256, 301, 336, 3, 1, 1),
    ("fpn.out2 3x3", 256, 256, 200, 336, 3, 1, 1),
    ("fpn.out3 3x3", 256, 256, 100, 168, 3, 1, 1),
    ("res3.conv2 3x3", 128, 128, 100, 168, 3, 1, 1),
    ("res4.conv2 3x3", 256, 256, 50, 84, 3, 1, 1),
    ("res3.conv3 1x1", 128, 512, 100, 168, 1, 1, 0),
    ("res4.conv3 1x1", 256, 1024, 50, 84, 1, 1, 0),
    ("fpn.lat2 1x1", 256, 256, 200, 336, 1, 1, 0),
    ("res2.conv2 3x3 (64)", 64, 64, 200, 336, 3, 1, 1),
]


def child(lib, imgs, iters, out_path, setting=None):
    sys.path.insert(0, REPO)
    import torch
    from mxtrain.ops import _lib
    _lib.LIB_PATH = os.path.abspath(lib)
    from mxtrain.ops import convwg
    if setting:
        fn, val = setting.split("=")
        _lib._fn(fn)(*[int(v) for v in val.split(":")])   # setter arguments, ':'-separated
    cl = torch.channels_last
    torch.manual_seed(0)
    res = {}
    outs = {}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, ci, co, h, w, k, st, pd in SHAPES:
        x = torch.randn(imgs, ci, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        wt = (torch.randn(co, ci, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
        b = torch.randn(co, device="cuda").to(torch.bfloat16)
        y = convwg.conv_fwd(x, wt, b, None, True, st, pd, 1) if convwg.fwd_supported(x, wt, b, None, st, pd, 1) \
            else None
        if y is None:
            continue
        dy = torch.randn_like(y)
        fns = {"fwd": lambda: convwg.conv_fwd(x, wt, b, None, True, st, pd, 1)}
        if co % 128 == 0 and ci % 128 == 0:
            fns["wgrad"] = lambda: convwg.conv_wgrad(dy, x, tuple(wt.shape), st, pd, 1)
        if convwg.dgrad_supported(wt, tuple(x.shape), st, pd, 1):
            fns["dgrad"] = lambda: convwg.conv_dgrad(dy, wt, tuple(x.shape), st, pd, 1)
        for d, fn in fns.items():
            o = fn()
            outs[f"{name}/{d}"] = o.float().flatten()[:: max(1, o.numel() // 65536)].cpu()
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(iters):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            res[f"{name}/{d}"] = ev[0].elapsed_time(ev[1]) * 1000 / iters
    torch.save(outs, out_path + ".pt")
    with open(out_path, "w") as f:
        json.dump(res, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default=None)
    ap.add_argument("--toggle", default=None, help="exported setter: A runs it with 0, B with 1 (same library)")
    ap.add_argument("--vals", default="0,1", help="setter arguments of A and B with --toggle")
    ap.add_argument("--set", default=None)
    ap.add_argument("--b", default=os.path.join(REPO, "mxtrain", "lib", "libmxkernels.so"))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--imgs", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--child", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.child:
        child(a.child, a.imgs, a.iters, a.out, a.set)
        return
    if a.toggle:
        a.a = a.b
    import statistics
    import tempfile
    times = {"A": {}, "B": {}}
    outs = {}
    for r in range(a.rounds):
        for tag, lib in (("A", a.a), ("B", a.b)):
            out = tempfile.mktemp(suffix=".json")
            va, vb = a.vals.split(",")
            extra = ["--set", f"{a.toggle}={va if tag == 'A' else vb}"] if a.toggle else []
            subprocess.run([sys.executable, __file__, "--child", lib, "--out", out, "--imgs",
                            str(a.imgs), "--iters", str(a.iters)] + extra, check=True)
            for k, v in json.load(open(out)).items():
                times[tag].setdefault(k, []).append(v)
            if r == 0:
                import torch
                outs[tag] = torch.load(out + ".pt", weights_only=True)
            os.remove(out)
            os.remove(out + ".pt")
    what = f"{a.toggle} {a.vals.replace(',', ' / ')}" if a.toggle else f"A = {a.a}, B = {a.b}"
    print(f"conv A/B at {a.imgs} images: {what}; median us over {a.rounds} rounds")
    ta = tb = 0.0
    for k in times["A"]:
        ma, mb = statistics.median(times["A"][k]), statistics.median(times["B"].get(k, [float("nan")]))
        oa, ob = outs["A"][k], outs["B"][k]
        diff = float((oa - ob).abs().max() / oa.abs().max().clamp_min(1e-6))
        ta += ma
        tb += mb
        print(f"  {k:32s} A {ma:8.1f}  B {mb:8.1f}  B/A {mb / ma:5.3f}  max rel diff {diff:.2e}")
    print(f"  total A {ta:.1f} us  B {tb:.1f} us  B/A {tb / ta:.3f}")


if __name__ == "__main__":
    main()
