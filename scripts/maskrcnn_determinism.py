"""Is one Mask R-CNN training step deterministic on the GPU?  Two model copies, the same
batch and RNG seed: forward losses (and, after backward + SGD, the parameters) compared
bitwise, step by step, at 2 images of 256 x 384 (the DP test's config) and at 800 x 1333.

    python scripts/maskrcnn_determinism.py
"""
import copy
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from mxtrain.data.coco import COCODetection, DetectionDataset, collate
    from mxtrain.data.coco_synth import write_split
    from mxtrain.models.compute_weights import FlatMaster
    from mxtrain.models.maskrcnn import MaskRCNN, MaskRCNNConfig
    if os.environ.get("MIOPEN_DET") == "1":   # MIOpen's deterministic solvers only
        torch.backends.cudnn.deterministic = True
        print("cudnn.deterministic = True")
    d = tempfile.mkdtemp()
    write_split(d, "train2017", 16, 0, 1)
    for (H, W, small) in ((256, 384, True), (800, 1333, False)):
        ds = DetectionDataset(COCODetection(d, "coco_train2017"), H, W, mask_format="crops")
        same = [i for i in range(len(ds)) if ds.orientation(i) == 0][:2]
        b = collate([ds[i] for i in same], H, W, fixed_gt=True, max_gt=16)
        x = {k: v.cuda() for k, v in b.items() if torch.is_tensor(v)}
        cfg = MaskRCNNConfig(train_per_level_topk=300, train_post_nms_topk=300, frcnn_batch_per_im=64) if small \
            else MaskRCNNConfig()
        torch.manual_seed(0)
        ma = MaskRCNN(cfg).cuda().train()
        mb = copy.deepcopy(ma)
        mw = copy.deepcopy(ma)   # warm-up copy: MIOpen's first call of a shape may run another solver
        hist = {}
        plain = os.environ.get("PLAIN") == "1"     # torch SGD + clip instead of FlatMaster
        side = torch.cuda.Stream()
        for tag, m in (("warm", mw), ("a", ma), ("b", mb)):
            ps = [p for p in m.parameters() if p.requires_grad]
            opt = torch.optim.SGD(ps, lr=0.01, momentum=0.9)
            fm = None if plain else FlatMaster(m, opt, 1.0)
            if fm is not None:
                m.__dict__["_flat_master"] = fm
            torch.cuda.manual_seed(7)
            out = []
            # SIDE=1: copy b runs on a side stream (as the graphed step's eager warm-up does)
            stream = side if (tag == "b" and os.environ.get("SIDE") == "1") else torch.cuda.current_stream()
            stream.wait_stream(torch.cuda.current_stream())
            for s in range(3):
                with torch.cuda.stream(stream):
                    opt.zero_grad(set_to_none=True)
                    losses = m(x["images"], x["hw"], x["gt_boxes"], x["gt_labels"], x["gt_count"], x["gt_mask_flat"],
                               x["gt_mask_table"])
                    losses["total_loss"].backward()
                    if fm is not None:
                        fm.step(0.01)
                    else:
                        torch.nn.utils.clip_grad_norm_(ps, 1.0)
                        opt.step()
                out.append({k: float(v.detach()) for k, v in losses.items()})
            torch.cuda.current_stream().wait_stream(stream)
            torch.cuda.synchronize()
            hist[tag] = (out, [p.detach().float().clone() for p in ps])
        print(f"== {H}x{W}")
        for s, (lw, la) in enumerate(zip(hist["warm"][0], hist["a"][0])):
            print(f"first-run copy vs a, step {s}: {'identical' if lw == la else 'differ'}")
        for s, (la, lb) in enumerate(zip(hist["a"][0], hist["b"][0])):
            diff = {k: (la[k], lb[k]) for k in la if la[k] != lb[k]}
            print(f"step {s}: {'identical' if not diff else 'DIFFER ' + str(diff)}")
        nd = sum(int(not torch.equal(p, q)) for p, q in zip(hist["a"][1], hist["b"][1]))
        print(f"parameters after 3 steps: {nd} of {len(hist['a'][1])} tensors differ", flush=True)


if __name__ == "__main__":
    main()
