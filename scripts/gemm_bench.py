#!/usr/bin/env python3
"""Weight-gradient GEMMs of GPT-2 345M (T = 4096 tokens): hipBLASLt (torch.addmm, with the
checked-in TunableOp table) vs csrc/gemm.hip grouped launches.  Interleaved rounds in one
process; prints per-group median microseconds and PF/s."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops.gemm import wgrad_group  # noqa: E402
from mxtrain.runtime.gemm_tuning import use_tuned_gemms  # noqa: E402


def main():
    use_tuned_gemms()
    T, h = 4096, 1024
    dev = "cuda"
    groups = {"fc2+fc1": [(h, 4 * h), (4 * h, h)], "proj+qkv": [(h, h), (3 * h, h)],
              "proj": [(h, h)], "qkv": [(3 * h, h)], "fc1": [(4 * h, h)], "fc2": [(h, 4 * h)]}
    data = {}
    for name, shapes in groups.items():
        items = []
        for M, N in shapes:
            dy = torch.randn(T, M, device=dev).to(torch.bfloat16)
            x = torch.randn(T, N, device=dev).to(torch.bfloat16)
            gb = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
            items.append((gb, dy, x))
        data[name] = items
    # numerics
    for name, items in data.items():
        wgrad_group(items, accumulate=False)
        for gb, dy, x in items:
            ref = dy.float().t() @ x.float()
            err = ((gb.float() - ref).abs().max() / ref.abs().max()).item()
            print(f"check {name} {tuple(gb.shape)} rel-max-err {err:.2e}")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def t_once(fn, reps=20):
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) * 1000 / reps

    from mxtrain.ops.gemm import plan
    cfgs = {}
    for name, items in data.items():
        cfgs[name] = [("auto", -1, 0)]
        for v, bm, bn in ((0, 128, 128), (3, 128, 128), (5, 128, 128), (6, 128, 128)):
            if any(dy.shape[1] % bm or x.shape[1] % bn for _, dy, x in items):
                continue
            for sp in (1, 2) if v in (0, 5) else (1,):
                cfgs[name].append((f"v{v}s{sp}", v, sp))
        print(name, "auto plan:", plan(items, T))
    for name, items in data.items():
        for label, v, sp in cfgs[name]:
            wgrad_group(items, accumulate=False, variant=v, splits=sp)
            for gb, dy, x in items:
                ref = dy.float().t() @ x.float()
                err = ((gb.float() - ref).abs().max() / ref.abs().max()).item()
                assert err < 1e-2, (name, label, err)
    res = {n: {"torch": [], **{c[0]: [] for c in cfgs[n]}} for n in groups}
    for _ in range(7):
        for name, items in data.items():
            res[name]["torch"].append(t_once(lambda: [gb.addmm_(dy.t(), x) for gb, dy, x in items]))
            for label, v, sp in cfgs[name]:
                res[name][label].append(t_once(lambda: wgrad_group(items, accumulate=True, variant=v, splits=sp)))
    for name, items in data.items():
        fl = sum(2 * T * gb.shape[0] * gb.shape[1] for gb, _, _ in items)
        print(f"== {name} ({fl / 1e9:.1f} GFLOP)")
        for k, vals in res[name].items():
            if vals:
                tm = statistics.median(vals)
                print(f"   {k:8s} {tm:7.1f} us {fl / tm / 1e9:5.3f} PF/s")


if __name__ == "__main__":
    main()
