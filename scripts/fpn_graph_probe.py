#!/usr/bin/env python3
"""FPN forward+backward: eager vs hipGraph replay, per-tensor differences, under switches
(JOIN=0/1 FPN.join_backward, SPLIT=0/1 convwg.SPLIT_IN_KERNEL).  Diagnostic for the
graphed-step mismatch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(join, split, batch=2):
    from mxtrain.models.maskrcnn import FPN
    from mxtrain.ops import convwg
    FPN.join_backward = bool(join)
    convwg.SPLIT_IN_KERNEL = bool(split)
    torch.manual_seed(0)
    chans = [256, 512, 1024, 2048]
    shapes = [(96, 128), (48, 64), (24, 32), (12, 16)]
    fpn = FPN(chans, 256).cuda().to(torch.bfloat16)
    names = [f"feat{i}" for i in range(4)] + [n for n, _ in fpn.named_parameters()]
    params = list(fpn.parameters())
    feats = [torch.randn(batch, c, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
             .requires_grad_(True) for c, (h, w) in zip(chans, shapes)]
    with torch.no_grad():
        gouts = [torch.randn_like(o) for o in fpn(feats)]

    def step():
        for p in params + feats:
            p.grad = None
        outs = fpn(feats)
        torch.autograd.backward(outs, gouts)
        return [t.grad for t in feats + params]

    ref = [g.clone() for g in step()]
    ref2 = [g.clone() for g in step()]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    for p in params + feats:
        p.grad = None
    with torch.cuda.graph(g):
        outs = fpn(feats)
        torch.autograd.backward(outs, gouts)
    grads = [t.grad for t in feats + params]
    res = []
    for rep in range(2):
        g.replay()
        torch.cuda.synchronize()
        res.append([x.clone() for x in grads])
    bad = []
    for n, a, a2, b0, b1 in zip(names, ref, ref2, res[0], res[1]):
        e = "" if torch.equal(a, a2) else " eager-vs-eager DIFFER"
        d0 = (a.float() - b0.float()).abs()
        d1 = (b0.float() - b1.float()).abs()
        if d0.max() > 0 or d1.max() > 0 or e:
            nz = (d0 > 0).nonzero()
            bad.append(f"  {n:28s} {tuple(a.shape)} eager-vs-replay max {d0.max().item():.3g} "
                       f"({int((d0 > 0).sum())} elems, first {nz[:3].tolist()}) replay-vs-replay max {d1.max().item():.3g}{e}")
    print(f"join={join} split={split}: {len(bad)} tensors differ", flush=True)
    for line in bad:
        print(line, flush=True)


def fwd_and_wgrad_repeat():
    """Forward outputs of two identical eager FPN forwards, and one 3x3 wgrad run twice."""
    from mxtrain.models.maskrcnn import FPN
    from mxtrain.ops import convwg
    torch.manual_seed(0)
    chans = [256, 512, 1024, 2048]
    shapes = [(96, 128), (48, 64), (24, 32), (12, 16)]
    fpn = FPN(chans, 256).cuda().to(torch.bfloat16)
    feats = [torch.randn(2, c, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
             for c, (h, w) in zip(chans, shapes)]
    with torch.no_grad():
        o1 = [o.clone() for o in fpn(feats)]
        junk = [torch.randn_like(o) for o in o1]   # disturb the allocator
        o2 = [o.clone() for o in fpn(feats)]
    for i, (a, b) in enumerate(zip(o1, o2)):
        d = (a.float() - b.float()).abs()
        print(f"fwd out {i}: max diff {d.max().item():.3g} ({int((d > 0).sum())} elems)", flush=True)
    for (h, w) in shapes[:3]:
        x = torch.randn(2, 256, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(2, 256, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r = [convwg.conv_wgrad(dy, x, (256, 256, 3, 3), 1, 1, 1).clone() for _ in range(4)]
        ref = torch.nn.grad.conv2d_weight(x.float(), (256, 256, 3, 3), dy.float(), 1, 1, 1)
        err = (r[0].float() - ref).abs().max().item() / ref.abs().max().item()
        print(f"wgrad 3x3 {h}x{w}: repeat diffs {[int((r[0] != q).sum()) for q in r[1:]]}, rel err vs fp32 {err:.3g}", flush=True)


def conv_repeat():
    """conv_fwd at the FPN shapes, run repeatedly with the allocator disturbed between runs."""
    from mxtrain.ops import convwg
    import torch.nn.functional as F
    shapes = [(96, 128), (48, 64), (24, 32), (12, 16)]
    chans = [256, 512, 1024, 2048]
    cl = lambda t: t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for lvl in range(3):
        h, w_ = shapes[lvl]
        for kind in ("lateral_res_up", "lateral_plain", "output3x3"):
            if kind == "output3x3":
                x = cl(torch.randn(2, 256, h, w_, device="cuda"))
                w = cl(torch.randn(256, 256, 3, 3, device="cuda") * 0.02)
                res, pad, up = None, 1, False
            else:
                x = cl(torch.randn(2, chans[lvl], h, w_, device="cuda"))
                w = cl(torch.randn(256, chans[lvl], 1, 1, device="cuda") * 0.02)
                res = cl(torch.randn(2, 256, h // 2, w_ // 2, device="cuda")) if kind == "lateral_res_up" else None
                pad, up = 0, kind == "lateral_res_up"
            b = (torch.randn(256, device="cuda") * 0.1).to(torch.bfloat16)
            for split in (1, 0):
                convwg.SPLIT_IN_KERNEL = bool(split)
                outs = []
                for k in range(4):
                    junk = torch.randn(1 << 20 + k, device="cuda")
                    outs.append(convwg.conv_fwd(x, w, b, res, False, 1, pad, 1, res_up=up).clone())
                    del junk
                ref = F.conv2d(x.float(), w.float(), b.float(), 1, pad)
                if res is not None:
                    ref = ref + F.interpolate(res.float(), scale_factor=2, mode="nearest")
                err = (outs[0].float() - ref).abs().max().item()
                print(f"level {lvl} {kind:15s} split_in_kernel={split}: repeat diffs "
                      f"{[int((outs[0] != q).sum()) for q in outs[1:]]}, max abs err vs fp32 {err:.3g}", flush=True)


def fpn_chain():
    """The FPN forward as explicit conv_fwd calls, twice: which intermediate differs."""
    from mxtrain.models.maskrcnn import FPN
    from mxtrain.ops import convwg
    from mxtrain.ops.epilogue import conv_bias_act
    torch.manual_seed(0)
    chans = [256, 512, 1024, 2048]
    shapes = [(96, 128), (48, 64), (24, 32), (12, 16)]
    fpn = FPN(chans, 256).cuda().to(torch.bfloat16)
    feats = [torch.randn(2, c, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
             for c, (h, w) in zip(chans, shapes)]
    for mode in ("conv_fwd_nchw_w", "conv_fwd_cl_w", "conv_bias_act"):
        runs = []
        for rep in range(3):
            junk = torch.randn((1 << 20) + 4096 * rep, device="cuda")
            lat = [None] * 4
            for i in range(3, -1, -1):
                m = fpn.lateral[i]
                wl = m.weight if mode != "conv_fwd_cl_w" else m.weight.contiguous(memory_format=torch.channels_last)
                res = lat[i + 1] if i < 3 else None
                if mode == "conv_bias_act":
                    lat[i] = conv_bias_act(feats[i], wl, m.bias, residual=res, res_up=res is not None)
                else:
                    lat[i] = convwg.conv_fwd(feats[i], wl, m.bias, res, False, 1, 0, 1, res_up=res is not None)
            outs = []
            for i in range(4):
                m = fpn.output[i]
                wo = m.weight if mode != "conv_fwd_cl_w" else m.weight.contiguous(memory_format=torch.channels_last)
                if mode == "conv_bias_act":
                    outs.append(conv_bias_act(lat[i], wo, m.bias, padding=1))
                else:
                    outs.append(convwg.conv_fwd(lat[i], wo, m.bias, None, False, 1, 1, 1))
            torch.cuda.synchronize()
            runs.append([t.clone() for t in lat + outs])
            del junk
        names = [f"lat{i}" for i in range(4)] + [f"out{i}" for i in range(4)]
        diffs = [f"{n}:{int((a != b).sum())}/{int((a != c).sum())}" for n, a, b, c in zip(names, *runs)]
        print(f"{mode}: " + " ".join(diffs), flush=True)


if __name__ == "__main__":
    fpn_chain()
    fwd_and_wgrad_repeat()
    for join in (0, 1):
        for split in (1, 0):
            run(join, split)
