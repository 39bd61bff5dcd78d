"""RoIAlign backward in isolation on the RoIs of a real Mask R-CNN training step (one
MI355X): records the box-head and mask-head RoIAlign calls of one eager step at the
training config, then times the tiled and the fp32-atomic backward kernels on exactly
those inputs and prints the tile-occupancy statistics of the tiled one.

    python scripts/roi_bwd_bench.py [--batch 4] [--iters 20]
"""
import argparse
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch
    from mxtrain.data.coco import COCODetection, DetectionDataset, collate
    from mxtrain.data.coco_synth import write_split
    from mxtrain.models.maskrcnn import MaskRCNN, MaskRCNNConfig
    from mxtrain.ops import vision as V
    d = tempfile.mkdtemp()
    write_split(d, "train2017", 16, 0, 1)
    ds = DetectionDataset(COCODetection(d, "coco_train2017"), 800, 1333, mask_format="crops")
    land = [i for i in range(len(ds)) if ds.orientation(i) == 0][:a.batch]
    b = collate([ds[i] for i in land], 800, 1333, fixed_gt=True, max_gt=100)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = MaskRCNN(MaskRCNNConfig()).to(dev).train()
    calls = []
    orig = V.RoIAlignFn.apply

    def rec(rois, PH, PW, sr, aligned, lvl_min, canon, canon_lvl, scales, *feats):
        calls.append((rois.detach().clone(), PH, PW, sr, aligned, lvl_min, canon, canon_lvl, list(scales),
                      [f.detach() for f in feats]))
        return orig(rois, PH, PW, sr, aligned, lvl_min, canon, canon_lvl, scales, *feats)
    V.RoIAlignFn.apply = rec
    x = {k: v.to(dev) for k, v in b.items() if torch.is_tensor(v)}
    losses = model(x["images"], x["hw"], x["gt_boxes"], x["gt_labels"], x["gt_count"], x["gt_mask_flat"],
                   x["gt_mask_table"])
    losses["total_loss"].backward()
    torch.cuda.synchronize()
    V.RoIAlignFn.apply = orig
    # plus a spread-out (trained-RPN-like) distribution: boxes of 2..~670 px anywhere
    g = torch.Generator().manual_seed(5)
    R = 2048
    x1 = torch.rand(R, generator=g) * 1344 * 0.8
    y1 = torch.rand(R, generator=g) * 800 * 0.8
    w = torch.rand(R, generator=g) * 1344 * 0.5 + 2
    h = torch.rand(R, generator=g) * 800 * 0.5 + 2
    bi = torch.randint(0, a.batch, (R,), generator=g).float()
    spread = torch.stack([bi, x1, y1, x1 + w, y1 + h], 1).to(dev)
    c0 = calls[0]
    calls.append((spread,) + tuple(c0[1:]))
    print(f"[roi] recorded {len(calls) - 1} RoIAlign calls (+1 spread-out RoI set)", flush=True)
    for ci, (rois, PH, PW, sr, aligned, lvl_min, canon, canon_lvl, scales, feats) in enumerate(calls):
        fs = [f.clone().requires_grad_(True) for f in feats]
        out = V.RoIAlignFn.apply(rois, PH, PW, sr, aligned, lvl_min, canon, canon_lvl, scales, *fs)
        dout = torch.randn_like(out)
        res = {}
        for tiled in (True, False):
            V._TILED = tiled
            for _ in range(3):
                g = torch.autograd.grad(out, fs, dout, retain_graph=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                g = torch.autograd.grad(out, fs, dout, retain_graph=True)
            e1.record()
            torch.cuda.synchronize()
            res[tiled] = (e0.elapsed_time(e1) * 1000 / a.iters, [t.float() for t in g])
        err = max(float((x - y).abs().max() / (y.abs().max() + 1e-6)) for x, y in zip(res[True][1], res[False][1]))
        V._TILED = True
        import ctypes
        fn = V._lib.lib().mx_roi_align_bwd_tiled_debug
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
        fn.restype = None
        # the scalar per-entry kernel (debug mode bit 2) against the MFMA one, same inputs
        fn2 = V._lib.lib().mx_roi_align_bwd_tiled_debug
        fn2.argtypes = [ctypes.c_void_p, ctypes.c_int]
        fn2.restype = None
        ab = {}
        for mode in (4, 0):
            fn2(None, mode)
            for _ in range(3):
                gg = torch.autograd.grad(out, fs, dout, retain_graph=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                gg = torch.autograd.grad(out, fs, dout, retain_graph=True)
            e1.record()
            torch.cuda.synchronize()
            ab[mode] = (e0.elapsed_time(e1) * 1000 / a.iters, [t.float() for t in gg])
        fn2(None, 0)
        d_ab = max(float((x - y).abs().max() / (y.abs().max() + 1e-6)) for x, y in zip(ab[0][1], ab[4][1]))
        print(f"[roi] call {ci}: tiled scalar-entry kernel {ab[4][0]:.1f} us, MFMA kernel {ab[0][0]:.1f} us, "
              f"max rel diff {d_ab:.2e}", flush=True)
        for mode in (0, 4):
            dbg = torch.full((200000, 4), -1, dtype=torch.int64, device=dev)
            fn(dbg.data_ptr(), mode)
            torch.autograd.grad(out, fs, dout, retain_graph=True)
            torch.cuda.synchronize()
            fn(None, 0)
            dd = dbg[dbg[:, 0] >= 0].cpu()
            t = dd[:, 3].float() / 100.0   # us
            top = torch.argsort(t, descending=True)[:4]
            print(f"[roi] call {ci} mode {mode}: {len(dd)} chunk records; per-WG us: mean {float(t.mean()):.1f} "
                  f"p50 {float(t.median()):.1f} max {float(t.max()):.1f}; slowest (chunk, tile, n, us): "
                  + ", ".join(f"({int(dd[i, 0])},{int(dd[i, 1])},{int(dd[i, 2])},{float(t[i]):.0f})" for i in top),
                  flush=True)
        ws, ovf_idx = V._LAST_WS
        R = rois.shape[0]
        items = R * PH * PW
        T = sum(feats[0].shape[0] * (-(-f.shape[1] // 8)) * (-(-f.shape[2] // 8)) for f in feats)
        counts = ws[items * 12: items * 12 + T].cpu()
        base = 0
        lv_stats = []
        for f in feats:
            nt = f.shape[0] * (-(-f.shape[1] // 8)) * (-(-f.shape[2] // 8))
            c = counts[base:base + nt]
            lv_stats.append(f"{int(c.sum())}e/{nt}t max {int(c.max())}")
            base += nt
        print(f"[roi] call {ci}: R={R} bins={PH}x{PW} items={items} entries={int(counts.sum())} "
              f"chunks={int(((counts + 255) // 256).clamp(min=1).sum())} overflow={int(ws[ovf_idx])} "
              f"levels: {' | '.join(lv_stats)}", flush=True)
        print(f"[roi] call {ci}: tiled {res[True][0]:.1f} us  atomic {res[False][0]:.1f} us  max rel diff {err:.2e}",
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
