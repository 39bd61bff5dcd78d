"""Data-parallel Mask R-CNN step on the MI355X: 2 ranks (processes on the one GPU of the
test box; control plane gloo), FlatMaster bucketed gradient all-reduce through the direct
xGMI kernel, the whole step -- forward, backward, all-reduces, clip + SGD -- captured as
ONE hipGraph and replayed, against the same data-parallel step run eagerly.  Both paths
must stay bit-identical ACROSS ranks (every rank applies the same averaged gradient) and
agree with each other to the graphed single-GPU test's tolerance.

Modes: ``same`` -- every rank sees one orientation; ``mixed`` -- rank 0 sees landscape ->
portrait -> landscape -> portrait while rank 1 sees landscape -> landscape -> portrait ->
landscape, so ranks meet a new canvas shape on DIFFERENT steps (the capture decision must
be collective, graphed.py); ``grow`` -- the mask payload outgrows rank 1's buffer only
(every rank must regrow / recapture together)."""
import copy
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sgd(model):
    decay = [p for p in model.parameters() if p.requires_grad and p.ndim > 1]
    nod = [p for p in model.parameters() if p.requires_grad and p.ndim <= 1]
    return torch.optim.SGD([{"params": decay, "weight_decay": 1e-4}, {"params": nod, "weight_decay": 0.0}],
                           lr=0.01, momentum=0.9), decay + nod


def _worker(rank, world, port, data_dir, q, mode="same"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXTRAIN_XGMI="1",
                          MXTRAIN_XGMI_TIMEOUT_S="20", MXTRAIN_XGMI_MAX_MB="64")
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        torch.backends.cudnn.deterministic = True   # as workloads/maskrcnn/train.py
        from mxtrain.data.coco import COCODetection, DetectionDataset, collate
        from mxtrain.models.compute_weights import FlatMaster
        from mxtrain.models.maskrcnn import MaskRCNN, MaskRCNNConfig
        from mxtrain.workloads.maskrcnn.graphed import GraphedTrainStep
        ds = DetectionDataset(COCODetection(data_dir, "coco_train2017"), 256, 384, mask_format="crops")
        land = [i for i in range(len(ds)) if ds.orientation(i) == 0]
        port_ = [i for i in range(len(ds)) if ds.orientation(i) == 1]

        def mk(idx):
            b = collate([ds[i] for i in idx], 256, 384, fixed_gt=True, max_gt=16)
            return {k: (v.pin_memory() if torch.is_tensor(v) else v) for k, v in b.items()}
        mine = land[4 * rank:4 * rank + 4]   # each rank its own images
        b1, b2 = mk(mine[:2]), mk(mine[2:4])
        if mode == "mixed":
            assert len(port_) >= 4, "synthetic set without portrait images"
            pm = port_[2 * rank:2 * rank + 2]
            p1 = mk(pm)
            seq = [b1, p1, b2, p1] if rank == 0 else [b1, b2, p1, b2]
        else:
            seq = [b1, b2, b1, b2]
        cap = 16 << 20
        if mode == "grow":
            if rank == 1:   # rank 1's buffer is exactly its smaller payload: the larger one overflows it
                small, large = sorted((b1, b2), key=lambda b: b["gt_mask_flat"].numel())
                assert large["gt_mask_flat"].numel() > small["gt_mask_flat"].numel()
                cap = small["gt_mask_flat"].numel()
                seq = [small, large, small, large]
        cfg = MaskRCNNConfig(train_per_level_topk=300, train_post_nms_topk=300, frcnn_batch_per_im=64)
        torch.manual_seed(0)
        ma = MaskRCNN(cfg).cuda().train()
        mb = copy.deepcopy(ma)
        oa, pa = _sgd(ma)
        ob, pb = _sgd(mb)
        fa = FlatMaster(ma, oa, 1.0, bucket_bytes=8 << 20)
        fb = FlatMaster(mb, ob, 1.0, bucket_bytes=8 << 20)
        assert len(fa.buckets) >= 3
        ma.__dict__["_flat_master"] = fa
        mb.__dict__["_flat_master"] = fb
        gs = GraphedTrainStep(mb, ob, pb, 1.0, torch.device("cuda"), flat_master=fb, flat_capacity=cap)
        plan = list(zip(seq, [0.01, 0.02, 0.02, 0.03]))
        la = []
        torch.cuda.manual_seed(7)
        for b, lr in plan:   # eager data-parallel step
            d = {k: v.cuda() for k, v in b.items() if torch.is_tensor(v)}
            oa.zero_grad(set_to_none=True)
            losses = ma(d["images"], d["hw"], d["gt_boxes"], d["gt_labels"], d["gt_count"], d["gt_mask_flat"],
                        d["gt_mask_table"])
            losses["total_loss"].backward()
            fa.step(lr)
            la.append(float(losses["total_loss"].detach()))
        torch.cuda.manual_seed(7)
        lb = [float(gs(b, lr)["total_loss"]) for b, lr in plan]
        torch.cuda.synchronize()
        from mxtrain.parallel import xgmi
        for c in xgmi._COMMS.values():
            if c is not None:
                c.check()
        num = sum(float((p - r).float().norm() ** 2) for p, r in zip(pa, pb)) ** 0.5
        den = sum(float(p.float().norm() ** 2) for p in pa) ** 0.5
        # cross-rank agreement: hash of every parameter on both paths
        ha = torch.cat([p.detach().float().reshape(-1)[:4096].cpu() for p in pa])
        hb = torch.cat([p.detach().float().reshape(-1)[:4096].cpu() for p in pb])
        q.put((rank, dict(captures=gs.captures, replays=gs.replays, eager=gs.eager_steps, regrows=gs.regrows,
                          handshakes=gs.handshakes,
                          routes_a=sorted(fa.dp_routes), routes_b=sorted(fb.dp_routes), rel=num / den,
                          la=la, lb=lb), ha.numpy(), hb.numpy()))
        dist.barrier()
        xgmi.destroy_all()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc()[-3000:]}, None, None))
        raise


@pytest.mark.timeout(280)
@pytest.mark.parametrize("mode", ["same", "mixed", "grow"])
def test_dp_graphed_step_with_xgmi_allreduce_matches_eager(tmp_path, mode):
    from mxtrain.data.coco_synth import write_split
    write_split(str(tmp_path), "train2017", 40, 0, 1)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in procs], key=lambda t: t[0])
        for p in procs:
            p.join(timeout=30)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    for r, info, _, _ in res:
        assert "error" not in info, info.get("error")
    for p in procs:
        assert p.exitcode == 0
    import numpy as np
    for r, info, ha, hb in res:
        assert info["handshakes"] == 4, info
        if mode == "same":
            assert info["captures"] == 1 and info["replays"] == 3 and info["eager"] == 0, info
        elif mode == "mixed":
            # step 1 both capture landscape; step 2 rank 0 captures portrait (rank 1 eager);
            # step 3 rank 1 captures portrait (rank 0 eager); step 4 both replay
            assert info["captures"] == 2 and info["eager"] == 1 and info["replays"] == 1, info
        else:
            assert (info["regrows"] >= 1) if r == 1 else (info["regrows"] == 0), info
            assert info["captures"] + info["eager"] + info["replays"] == 4 and info["replays"] >= 1, info
        assert info["routes_a"] == ["xgmi"] and info["routes_b"] == ["xgmi"], info
        # MIOpen's deterministic solvers (set in the worker) + deterministic in-repo kernels and
        # xGMI reductions: the graphed step reproduces the eager one
        assert info["rel"] < 1e-6, info
        for s, (x, y) in enumerate(zip(info["la"], info["lb"])):
            assert abs(x - y) <= 1e-5 * abs(x), (r, s, info["la"], info["lb"])
    # every rank applied the same averaged gradients: identical parameters on both paths
    assert np.array_equal(res[0][2], res[1][2])
    assert np.array_equal(res[0][3], res[1][3])
