"""Which Python-level ops launch the GPU kernels of a Mask R-CNN training step: one eager
step (after warm-up, FlatMaster optimizer as in training) under torch.profiler, aten ops
with their device-kernel counts, grouped by the top model frames of their call stacks.

    python scripts/op_census_maskrcnn.py [--batch 1] > gpurun_out/op_census.txt
"""
import argparse
import collections
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    a = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile
    from mxtrain.data.coco import COCODetection, DetectionDataset, collate
    from mxtrain.data.coco_synth import write_split
    from mxtrain.models.compute_weights import FlatMaster
    from mxtrain.models.maskrcnn import MaskRCNN, MaskRCNNConfig
    from mxtrain.workloads.maskrcnn.train import use_shipped_find_db
    os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
    use_shipped_find_db()
    torch.backends.cudnn.benchmark = True
    d = tempfile.mkdtemp()
    write_split(d, "train2017", 8, 0, 1)
    ds = DetectionDataset(COCODetection(d, "coco_train2017"), 800, 1333, mask_format="crops")
    land = [i for i in range(len(ds)) if ds.orientation(i) == 0]
    b = collate([ds[land[j % len(land)]] for j in range(a.batch)], 800, 1333, fixed_gt=True)
    dev = torch.device("cuda")
    x = {k: v.to(dev) for k, v in b.items() if torch.is_tensor(v)}
    model = MaskRCNN(MaskRCNNConfig()).to(dev).train()
    decay = [p for p in model.parameters() if p.requires_grad and p.ndim > 1]
    nod = [p for p in model.parameters() if p.requires_grad and p.ndim <= 1]
    opt = torch.optim.SGD([{"params": decay, "weight_decay": 1e-4}, {"params": nod, "weight_decay": 0.0}],
                          lr=1e-3, momentum=0.9)
    fm = FlatMaster(model, opt, 1.0)
    model.__dict__["_flat_master"] = fm

    def step():
        losses = model(x["images"], x["hw"], x["gt_boxes"], x["gt_labels"], x["gt_count"],
                       x.get("gt_mask_flat", x.get("gt_masks")), x.get("gt_mask_table"))
        opt.zero_grad(set_to_none=True)
        losses["total_loss"].backward()
        fm.step(1e-3)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    # kernels per aten op (direct children), attributed to the innermost repo frame
    evs = prof.events()
    agg = collections.Counter()
    for e in evs:
        if e.device_type.name != "CPU" or not e.name.startswith("aten::"):
            continue
        kids = [k for k in e.kernels] if hasattr(e, "kernels") else []
        nk = len(kids)
        if nk == 0:
            continue
        frames = [f for f in (e.stack or []) if "mxtrain" in f]
        where = frames[0].split("mxtrain/")[-1] if frames else "?"
        agg[(e.name, where)] += nk
    tot = sum(agg.values())
    print(f"kernels attributed to aten ops: {tot}")
    for (name, where), n in agg.most_common(150):
        print(f"{n:5d}  {name:40s} {where}")
    # which ops launch the kernels matching CENSUS_KERNELS (regex)
    import re
    pat = re.compile(os.environ.get("CENSUS_KERNELS", "rocprim|fillBuffer|SubTensorOp|CUDAFunctor_add"))
    sel = collections.Counter()
    for e in evs:
        if e.device_type.name != "CPU" or not e.name.startswith("aten::"):
            continue
        frames = [f for f in (e.stack or []) if "mxtrain" in f]
        where = frames[0].split("mxtrain/")[-1] if frames else "?"
        for k in getattr(e, "kernels", []) or []:
            if pat.search(k.name):
                sel[(k.name[:60], e.name, str(e.input_shapes)[:110])] += 1
    # gradient-accumulation / residual adds by operand shape (backward ops carry no stack)
    shp = collections.Counter()
    for e in evs:
        if e.device_type.name == "CPU" and e.name in ("aten::add", "aten::add_") and getattr(e, "kernels", None):
            shp[(e.name, str(e.input_shapes)[:90])] += len(e.kernels)
    print("\nadd kernels by operand shapes:")
    for (name, sh), n in shp.most_common(60):
        print(f"{n:5d}  {name:10s} {sh}")
    print("\nselected kernels by launching op:")
    for (kn, name, where), n in sel.most_common(80):
        print(f"{n:5d}  {kn:60s} {name:24s} {where}")
    # convolutions still on MIOpen, by operand shapes, with their kernels' device time
    conv = collections.defaultdict(lambda: [0, 0.0])
    for e in evs:
        if e.device_type.name == "CPU" and "convolution" in e.name and getattr(e, "kernels", None):
            c = conv[(e.name, str(e.input_shapes)[:120])]
            c[0] += 1
            c[1] += sum(getattr(k, "duration", 0.0) for k in e.kernels)
    print("\nMIOpen convolution ops by operand shapes (calls, kernel us):")
    for (name, sh), (n, us) in sorted(conv.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:4d} {us:9.1f}  {name:36s} {sh}")


if __name__ == "__main__":
    main()
