"""Mask R-CNN training step on the MI355X: the whole-step hipGraph replay
(workloads/maskrcnn/graphed.py) against the eager step on the same batches, packed
mask crops in both."""
import copy

import pytest
import torch


def _eager_step(model, opt, params, batch, lr, clip):
    from mxtrain.workloads.maskrcnn.graphed import LOSS_NAMES, sgd_momentum_
    d = {k: v.cuda() for k, v in batch.items() if torch.is_tensor(v)}
    opt.zero_grad(set_to_none=True)
    losses = model(d["images"], d["hw"], d["gt_boxes"], d["gt_labels"], d["gt_count"], d["gt_mask_flat"],
                   d["gt_mask_table"])
    losses["total_loss"].backward()
    torch.nn.utils.clip_grad_norm_(params, clip)
    sgd_momentum_(opt, lr)
    return {k: losses[k].detach().float() for k in LOSS_NAMES}


def _sgd(model):
    decay = [p for p in model.parameters() if p.requires_grad and p.ndim > 1]
    nod = [p for p in model.parameters() if p.requires_grad and p.ndim <= 1]
    return torch.optim.SGD([{"params": decay, "weight_decay": 1e-4}, {"params": nod, "weight_decay": 0.0}],
                           lr=0.01, momentum=0.9), decay + nod


@pytest.mark.gpu
@pytest.mark.parametrize("join", [False, True])
def test_graphed_step_matches_eager(tmp_path, join, monkeypatch):
    from mxtrain.data.coco import COCODetection, DetectionDataset, collate
    from mxtrain.data.coco_synth import write_split
    from mxtrain.models.maskrcnn import FPN, MaskRCNN, MaskRCNNConfig
    monkeypatch.setattr(FPN, "join_backward", join)
    from mxtrain.workloads.maskrcnn.graphed import GraphedTrainStep
    write_split(str(tmp_path), "train2017", 24, 0, 1)
    ds = DetectionDataset(COCODetection(str(tmp_path), "coco_train2017"), 256, 384, mask_format="crops")
    same = [i for i in range(len(ds)) if ds.orientation(i) == 0]
    assert len(same) >= 4
    b1 = collate([ds[i] for i in same[:2]], 256, 384, fixed_gt=True, max_gt=16)
    b2 = collate([ds[i] for i in same[2:4]], 256, 384, fixed_gt=True, max_gt=16)
    b1 = {k: (v.pin_memory() if torch.is_tensor(v) else v) for k, v in b1.items()}
    b2 = {k: (v.pin_memory() if torch.is_tensor(v) else v) for k, v in b2.items()}
    cfg = MaskRCNNConfig(train_per_level_topk=300, train_post_nms_topk=300, frcnn_batch_per_im=64)
    # MIOpen's deterministic solvers: with its default (atomics-based) choices for the few
    # convolutions it still runs, two identical eager steps already differ in the last bits
    # and the random-init proposal sampling amplifies that (scripts/maskrcnn_determinism.py);
    # every in-repo kernel is deterministic, so the graph must then reproduce eager exactly
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    torch.manual_seed(0)
    ma = MaskRCNN(cfg).cuda().train()
    mb = copy.deepcopy(ma)
    oa, pa = _sgd(ma)
    ob, pb = _sgd(mb)
    gs = GraphedTrainStep(mb, ob, pb, 1.0, torch.device("cuda"))
    plan = [(b1, 0.01), (b2, 0.02), (b1, 0.02), (b2, 0.03)]
    torch.cuda.manual_seed(7)
    la = [_eager_step(ma, oa, pa, b, lr, 1.0) for b, lr in plan]
    torch.cuda.manual_seed(7)
    lb = [gs(b, lr) for b, lr in plan]
    torch.cuda.synchronize()
    torch.backends.cudnn.deterministic = det
    assert gs.captures == 1 and gs.replays == 3
    num = sum(float((p - q).float().norm() ** 2) for p, q in zip(pa, pb)) ** 0.5
    den = sum(float(p.float().norm() ** 2) for p in pa) ** 0.5
    rel = [max(abs(float(x[k]) - float(y[k])) / (abs(float(x[k])) + 1e-6) for k in x) for x, y in zip(la, lb)]
    print(f"graphed vs eager, max relative loss difference per step: {rel}; params {num / den:.2e}")
    for s, (x, y) in enumerate(zip(la, lb)):
        for k in x:
            assert torch.isfinite(y[k]), (s, k)
            assert abs(float(x[k]) - float(y[k])) <= 1e-5 * abs(float(x[k])), (s, k, float(x[k]), float(y[k]))
    assert num / den < 1e-6, num / den


@pytest.mark.gpu
def test_flat_master_gpu_matches_cpu():
    """csrc/multitensor.hip (gradient cast + fold scale + sumsq, clip + SGD + compute-copy
    refresh) against the FlatMaster's torch path on identical gradients: fp32 master and
    momentum to fp32 rounding, bf16 copies (channels_last for the convs) to one bf16 ulp."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_flat_master_cpu import Tiny, _opt
    from mxtrain.models.compute_weights import FlatMaster
    torch.manual_seed(3)
    cpu = Tiny()
    gpu = copy.deepcopy(cpu).cuda()
    fc = FlatMaster(cpu, _opt(cpu), 0.05, dt=torch.bfloat16)
    fg = FlatMaster(gpu, _opt(gpu), 0.05, dt=torch.bfloat16)
    fc.ensure_fresh()
    fg.ensure_fresh()
    for step in range(3):
        views = fc.compute_views()
        grads = [torch.randn(v.shape).to(torch.bfloat16) for v in views]
        # the GPU copies' grads in their layout (channels_last conv weights)
        ggrads = [g.cuda().contiguous(memory_format=torch.channels_last) if g.dim() == 4 else g.cuda()
                  for g in grads]
        fc.grads_in(grads)
        fg.grads_in(ggrads)
        torch.testing.assert_close(fg.normsq.cpu(), fc.normsq, rtol=1e-5, atol=0)
        fc.step(0.1 * (step + 1))
        fg.step(0.1 * (step + 1))
        torch.cuda.synchronize()
        torch.testing.assert_close(fg.P.cpu(), fc.P, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(fg.M.cpu(), fc.M, rtol=1e-6, atol=1e-6)
        for a, b in zip(fg.compute_views(), fc.compute_views()):
            assert a.shape == b.shape
            torch.testing.assert_close(a.float().cpu(), b.float(), rtol=8e-3, atol=1e-6)


@pytest.mark.gpu
def test_input_normalisation_kernel_matches_reference():
    """uint8 NCHW images -> normalised bf16 NHWC in one pass (csrc/vision.hip
    normalize_u8_nhwc_kernel, models/maskrcnn.py MaskRCNN.features) against the fp32 chain."""
    import ctypes
    from mxtrain.models.maskrcnn import MaskRCNNConfig
    from mxtrain.ops import _lib
    cfg = MaskRCNNConfig()
    g = torch.Generator().manual_seed(3)
    img = torch.randint(0, 256, (2, 3, 40, 36), generator=g, dtype=torch.uint8).cuda()
    x = torch.empty(2, 40, 36, 3, dtype=torch.bfloat16, device="cuda").permute(0, 3, 1, 2)
    _lib.call("mx_normalize_u8_nhwc", img.data_ptr(), x.data_ptr(), 2, 40, 36,
              ctypes.cast((ctypes.c_float * 3)(*cfg.pixel_mean), ctypes.c_void_p),
              ctypes.cast((ctypes.c_float * 3)(*[1.0 / v for v in cfg.pixel_std]), ctypes.c_void_p), _lib.stream())
    torch.cuda.synchronize()
    mean = torch.tensor(cfg.pixel_mean).view(1, 3, 1, 1)
    std = torch.tensor(cfg.pixel_std).view(1, 3, 1, 1)
    ref = (img.cpu().float() - mean) / std
    assert x.is_contiguous(memory_format=torch.channels_last)
    assert (x.float().cpu() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
