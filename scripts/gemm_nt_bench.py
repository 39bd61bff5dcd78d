#!/usr/bin/env python3
"""Forward / dgrad GEMMs of a GPT-2 345M layer (T = 4096 tokens): hipBLASLt (torch, with the
checked-in TunableOp table, plus the separate bias-GeLU kernels where the layer has them)
vs csrc/gemm_nt.hip variants with fused epilogues.  Interleaved rounds in one process on
random data; prints per-shape median microseconds and PF/s."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import gemm as Gm  # noqa: E402
from mxtrain.ops.fused import bias_gelu_bwd, bias_gelu_fwd  # noqa: E402
from mxtrain.runtime.gemm_tuning import use_tuned_gemms  # noqa: E402


def main():
    use_tuned_gemms()
    T = int(os.environ.get("T", 4096))
    h = int(os.environ.get("H", 1024))
    dev = "cuda"
    bf = torch.bfloat16
    r = lambda *s, sc=1.0: (torch.randn(*s, device=dev) * sc).to(bf)  # noqa: E731
    probs = {
        # name: (kind, M, N, K)
        "qkv_fwd+bias": ("fwd1", T, 3 * h, h),
        "proj_fwd": ("fwd0", T, h, h),
        "fc1_fwd+bias_gelu": ("fwd2", T, 4 * h, h),
        "fc2_fwd": ("fwd0", T, h, 4 * h),
        "fc2_dgrad+dgelu": ("dg3", T, 4 * h, h),
        "fc1_dgrad": ("dg0", T, h, 4 * h),
        "proj_dgrad": ("dg0", T, h, h),
        "qkv_dgrad": ("dg0", T, h, 3 * h),
    }
    if os.environ.get("LMHEAD"):   # tied LM head: logits = X E^T, dX = dlogits E
        V = int(os.environ.get("V", 50304))
        probs = {"lm_fwd": ("fwd0", T, V, h), "lm_dgrad": ("dg0", T, h, V)}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def t_once(fn, reps=int(os.environ.get("REPS", 20))):
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) * 1000 / reps

    fns = {}
    for name, (kind, M, N, K) in probs.items():
        a = r(M, K)
        if kind.startswith("fwd"):
            w = r(N, K, sc=0.05)
            b = r(N) if kind != "fwd0" else None
            gelu = kind == "fwd2"
            if gelu:
                base = lambda a=a, w=w, b=b: bias_gelu_fwd(torch.mm(a, w.t()), b)  # noqa: E731
            elif b is not None:
                base = lambda a=a, w=w, b=b: torch.addmm(b, a, w.t())  # noqa: E731
            else:
                base = lambda a=a, w=w: torch.mm(a, w.t())  # noqa: E731
            mk = lambda v, a=a, w=w, b=b, gelu=gelu: (lambda: Gm.linear_fwd(a, w, b, gelu=gelu, variant=v))  # noqa: E731
            ref = (a.float() @ w.float().t() + (b.float() if b is not None else 0))
            if gelu:
                ref = Gm._gelu_ref(ref)
        else:
            w = r(K, N, sc=0.05)
            gelu = kind == "dg3"
            hh = r(M, N) if gelu else None
            db = torch.zeros(N, device=dev, dtype=bf) if gelu else None
            if gelu:
                base = lambda a=a, w=w, hh=hh, db=db: bias_gelu_bwd(torch.mm(a, w), hh, db, dbias=db,  # noqa: E731
                                                                     accumulate=True, inplace=True)
            else:
                base = lambda a=a, w=w: torch.mm(a, w)  # noqa: E731
            mk = lambda v, a=a, w=w, hh=hh, db=db: (lambda: Gm.linear_dgrad(a, w, gelu_aux=hh, dbias=db, variant=v))  # noqa: E731
            ref = a.float() @ w.float()
            if gelu:
                ref = ref * Gm._gelu_grad_ref(hh.float())
        variants = []
        for v in ([int(x) for x in os.environ["VARIANTS"].split(",")] if os.environ.get("VARIANTS") else range(9)):
            bm, bn, _, kok = Gm._nt_tile(v)
            if M % bm or N % bn or (kind.startswith("dg") and not kok):
                continue
            out = mk(v)()
            out = out[0] if isinstance(out, tuple) else out
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            print(f"check {name} v{v} rel-max-err {err:.2e}", flush=True)
            assert err < 2e-2, (name, v, err)
            variants.append(v)
        fns[name] = {"torch": base, **{f"v{v}": mk(v) for v in variants}}
        print(name, "plan:", Gm.nt_plan(M, N, K, kind.startswith("dg")), flush=True)
    res = {n: {k: [] for k in fs} for n, fs in fns.items()}
    rounds = int(os.environ.get("ROUNDS", 7))
    for _ in range(rounds):
        for name, fs in fns.items():
            for k, fn in fs.items():
                res[name][k].append(t_once(fn))
    tot = {"torch": 0.0, "best": 0.0, "plan": 0.0}
    for name, (kind, M, N, K) in probs.items():
        fl = 2 * M * N * K
        print(f"== {name} M{M} N{N} K{K} ({fl / 1e9:.1f} GFLOP)")
        meds = {k: statistics.median(v) for k, v in res[name].items()}
        for k, tm in meds.items():
            print(f"   {k:6s} {tm:7.1f} us {fl / tm / 1e9:5.3f} PF/s")
        tot["torch"] += meds["torch"]
        tot["best"] += min(v for k, v in meds.items() if k != "torch")
        pv = f"v{Gm.nt_plan(M, N, K, kind.startswith('dg'))}"
        tot["plan"] += meds.get(pv, meds["torch"])
    print("per-layer total us:", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
