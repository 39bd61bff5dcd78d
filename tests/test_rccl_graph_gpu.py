"""The default N > 1 step route -- RCCL collectives captured inside the whole-step hipGraph
-- executed on the test box's one MI355X: a ONE-rank RCCL ("nccl") process group with the
data-parallel machinery forced on, so every collective the 8-GPU bench issues (the GPT
ZeRO-1 per-bucket reduce-scatter / all-gather, the Mask R-CNN FlatMaster per-bucket
all-reduce) is a real RCCL call, captured into the graph and replayed.  RCCL cannot put two
ranks on one GPU, so one rank is the most this box can run; with one rank RCCL still runs
its collective kernels (a copy), which is what the capture / replay machinery needs.

The replayed steps must be BIT-identical to the same steps run eagerly through the same
RCCL calls (and, for GPT, to the trainer without the forced collectives).
Reference: examples/maskrcnn/train-maskrcnn-tensorpack.yaml:34 (TRAINER=horovod) and
examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-zero1.yaml:7-8 (DP + ZeRO-1)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(num_layers=2, hidden_size=256, num_attention_heads=4, seq_length=256, max_position_embeddings=256,
           vocab_size=1024, hidden_dropout=0.1, attention_dropout=0.1)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init_rccl(port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      MXTRAIN_XGMI="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"


def _gpt_worker(port, q):
    try:
        _init_rccl(port)
        import torch.distributed as dist
        from mxtrain.models.gpt import GPTConfig
        from mxtrain.parallel import state as pstate
        from mxtrain.training import GPTTrainer, TrainConfig
        ps = pstate.initialize_model_parallel(device_type="cuda")
        cfg = GPTConfig(**CFG)
        g = torch.Generator().manual_seed(11)
        x = torch.randint(0, CFG["vocab_size"], (1, 4, CFG["seq_length"] + 1), generator=g)
        tok, lab = x[..., :-1].contiguous().cuda(), x[..., 1:].contiguous().cuda()
        out = {}
        for name, force, graph in (("plain", False, False), ("forced", True, False), ("graph", True, True)):
            tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=4, lr=1e-3, force_dp_collectives=force), ps)
            assert tr.opt.sharded == force
            if graph:
                losses = [float(tr.capture(tok, lab, warmup=1))]
                losses += [float(tr.train_step(tok, lab)) for _ in range(3)]
                census = tr.graph_census
            else:
                losses = [float(tr.train_step(tok, lab)) for _ in range(4)]
            tr.sync_params()
            torch.cuda.synchronize()
            out[name] = (losses, {n: p.detach().float().cpu().numpy() for n, p in tr.flat.params.items()})
            del tr
        q.put(("ok", out, census))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put(("error", traceback.format_exc()[-3000:], None))
        raise


def _maskrcnn_worker(port, data_dir, q):
    try:
        _init_rccl(port)
        import copy
        import torch.distributed as dist
        torch.backends.cudnn.deterministic = True
        from mxtrain.data.coco import COCODetection, DetectionDataset, collate
        from mxtrain.models.compute_weights import FlatMaster
        from mxtrain.models.maskrcnn import MaskRCNN, MaskRCNNConfig
        from mxtrain.workloads.maskrcnn.graphed import GraphedTrainStep
        ds = DetectionDataset(COCODetection(data_dir, "coco_train2017"), 256, 384, mask_format="crops")
        land = [i for i in range(len(ds)) if ds.orientation(i) == 0]

        def mk(idx):
            b = collate([ds[i] for i in idx], 256, 384, fixed_gt=True, max_gt=16)
            return {k: (v.pin_memory() if torch.is_tensor(v) else v) for k, v in b.items()}
        b1, b2 = mk(land[:2]), mk(land[2:4])
        cfg = MaskRCNNConfig(train_per_level_topk=300, train_post_nms_topk=300, frcnn_batch_per_im=64)
        torch.manual_seed(0)
        ma = MaskRCNN(cfg).cuda().train()
        mb = copy.deepcopy(ma)

        def sgd(m):
            decay = [p for p in m.parameters() if p.requires_grad and p.ndim > 1]
            nod = [p for p in m.parameters() if p.requires_grad and p.ndim <= 1]
            return torch.optim.SGD([{"params": decay, "weight_decay": 1e-4}, {"params": nod, "weight_decay": 0.0}],
                                   lr=0.01, momentum=0.9), decay + nod
        oa, pa = sgd(ma)
        ob, pb = sgd(mb)
        fa = FlatMaster(ma, oa, 1.0, bucket_bytes=8 << 20, force_dp=True)
        fb = FlatMaster(mb, ob, 1.0, bucket_bytes=8 << 20, force_dp=True)
        assert fa.dp and fb.dp and len(fa.buckets) >= 3
        ma.__dict__["_flat_master"] = fa
        mb.__dict__["_flat_master"] = fb
        gs = GraphedTrainStep(mb, ob, pb, 1.0, torch.device("cuda"), flat_master=fb)
        plan = [(b1, 0.01), (b2, 0.02), (b1, 0.02), (b2, 0.03)]
        la = []
        torch.cuda.manual_seed(7)
        for b, lr in plan:
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
        same = all(bool(torch.equal(x, y)) for x, y in zip(pa, pb))
        num = sum(float((x - y).float().norm() ** 2) for x, y in zip(pa, pb)) ** 0.5
        den = sum(float(x.float().norm() ** 2) for x in pa) ** 0.5
        q.put(("ok", dict(la=la, lb=lb, same=same, rel=num / den, captures=gs.captures, replays=gs.replays,
                          eager=gs.eager_steps, routes_a=sorted(fa.dp_routes), routes_b=sorted(fb.dp_routes),
                          nodes=[v for v in gs.graph_info.values()]), None))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put(("error", traceback.format_exc()[-3000:], None))
        raise


def _run(target, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=target, args=(_port(), *args, q))
    p.start()
    try:
        res = q.get(timeout=240)
        p.join(timeout=30)
    finally:
        if p.is_alive():
            p.kill()
    assert res[0] == "ok", res[1]
    assert p.exitcode == 0
    return res


@pytest.mark.timeout(280)
def test_gpt_zero1_rccl_in_graph_bit_identical():
    import numpy as np
    _, out, census = _run(_gpt_worker)
    assert census["kernel"] > 0, census
    lp, pp = out["plain"]
    lf, pf = out["forced"]
    lg, pg = out["graph"]
    # the RCCL reduce-scatter / all-gather of one rank move the same bytes: forced == plain
    assert lf == lp, (lf, lp)
    # the captured step (RCCL collectives inside the graph) replays the eager step exactly
    assert lg == lf, (lg, lf)
    for n in pf:
        assert np.array_equal(pf[n], pp[n]), n
        assert np.array_equal(pg[n], pf[n]), n


@pytest.mark.timeout(280)
def test_maskrcnn_flat_allreduce_rccl_in_graph_bit_identical(tmp_path):
    from mxtrain.data.coco_synth import write_split
    write_split(str(tmp_path), "train2017", 8, 0, 1)
    _, info, _ = _run(_maskrcnn_worker, str(tmp_path))
    assert info["routes_a"] == ["rccl"] and info["routes_b"] == ["rccl"], info
    assert info["captures"] == 1 and info["replays"] == 3 and info["eager"] == 0, info
    print(f"[rccl-graph] bit-identical parameters: {info['same']}, relative difference {info['rel']:.3g}")
    # the tolerance of the xGMI DP test (tests/test_maskrcnn_dp_gpu.py): deterministic MIOpen
    # solvers + deterministic in-repo kernels reproduce the eager step
    assert info["rel"] < 1e-6, info
    for x, y in zip(info["la"], info["lb"]):
        assert abs(x - y) <= 1e-5 * abs(x), info
