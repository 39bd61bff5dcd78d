"""Steady-state host-side (Python) profile of the eager Mask R-CNN training step on one
GPU: warm up, then cProfile a window of steps and print the top functions, to find what
the host spends its ~18 ms/step on at 1 img/GPU.

    python scripts/host_profile_maskrcnn.py [--batch 1] [--steps 20]
"""
import argparse
import cProfile
import os
import pstats
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from mxtrain.data.coco import COCODetection, DetectionDataset, collate
    from mxtrain.data.coco_synth import write_split
    from mxtrain.models.maskrcnn import MaskRCNN, MaskRCNNConfig
    d = tempfile.mkdtemp()
    write_split(d, "train2017", 8, 0, 1)
    ds = DetectionDataset(COCODetection(d, "coco_train2017"), 800, 1333, mask_format="crops")
    land = [i for i in range(len(ds)) if ds.orientation(i) == 0]
    b = collate([ds[land[j % len(land)]] for j in range(a.batch)], 800, 1333)
    dev = torch.device("cuda")
    x = {k: v.to(dev) for k, v in b.items() if torch.is_tensor(v)}
    model = MaskRCNN(MaskRCNNConfig()).to(dev).train()
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.SGD(params, lr=1e-3, momentum=0.9)

    def step():
        losses = model(x["images"], x["hw"], x["gt_boxes"], x["gt_labels"], x["gt_count"],
                       x.get("gt_mask_flat", x.get("gt_masks")), x.get("gt_mask_table"))
        opt.zero_grad(set_to_none=True)
        losses["total_loss"].backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()

    for _ in range(8):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host {1e3 * (t1 - t0) / a.steps:.2f} ms/step (profiled), wall incl. drain {1e3 * (t2 - t0) / a.steps:.2f}")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumtime").print_stats(45)


if __name__ == "__main__":
    main()
