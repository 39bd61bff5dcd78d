"""Mask R-CNN R50-FPN training / evaluation / prediction, command-line compatible with
tensorpack `examples/FasterRCNN/train.py` and the aws-samples `MaskRCNN/train.py` as the
reference's MPIJob charts run them:

    mpirun ... python3 train.py --logdir $LOG_DIR [--images_per_epoch N] [--verbose] \\
        --config MODE_MASK=True MODE_FPN=True DATA.BASEDIR=/fsx/data/coco2017 \\
        DATA.TRAIN='["coco_train2017"]' DATA.VAL='("coco_val2017")' TRAIN.BASE_LR=0.01 \\
        BACKBONE.WEIGHTS=.../ImageNet-R50-AlignPadding.npz BACKBONE.NORM=FreezeBN TRAINER=horovod ...

One process per MI355X (ranks from mpirun / torchrun env), RCCL gradient all-reduce
(mxtrain.parallel.hvd), the MI355X Mask R-CNN (HIP RoIAlign / NMS / matching kernels,
MIOpen NHWC bf16 convs).  Checkpoints keep tensorpack's discovery contract:
`<logdir>/model-<step>.index` + `.data-00000-of-00001` (safetensors payload) + a
`checkpoint` file; COCO eval results go to `<logdir>/stats.json`.
"""
from __future__ import annotations

import argparse
import functools
import glob
import json
import os
import sys
import time

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def log(*a):
    from mxtrain.parallel import hvd
    if hvd.rank() == 0:
        print(time.strftime("[%m%d %H:%M:%S @train.py]"), *a, flush=True)


# ------------------------------------------------------------------------------ checkpoints
def save_ckpt(model, opt, logdir: str, step: int, epoch: int, keep: int = 5):
    from safetensors.torch import save_file
    sd = {k: v.detach().contiguous().cpu() for k, v in model.state_dict().items()}
    name = f"model-{step}"
    save_file(sd, os.path.join(logdir, f"{name}.data-00000-of-00001"))
    with open(os.path.join(logdir, f"{name}.index"), "w") as f:
        json.dump({"format": "mxtrain-safetensors-v1", "global_step": step, "epoch": epoch,
                   "tensors": {k: [list(v.shape), str(v.dtype)] for k, v in sd.items()}}, f)
    torch.save({"optimizer": opt.state_dict(), "step": step, "epoch": epoch},
               os.path.join(logdir, f"{name}.optim"))
    ckpts = sorted(glob.glob(os.path.join(logdir, "model-*.index")), key=lambda p: int(p.split("-")[-1][:-6]))
    for old in ckpts[:-keep]:
        base = old[:-6]
        for suf in (".index", ".data-00000-of-00001", ".optim"):
            if os.path.exists(base + suf):
                os.unlink(base + suf)
    with open(os.path.join(logdir, "checkpoint"), "w") as f:
        f.write(f'model_checkpoint_path: "{name}"\n')
        for p in sorted(glob.glob(os.path.join(logdir, "model-*.index")), key=lambda p: int(p.split("-")[-1][:-6])):
            f.write(f'all_model_checkpoint_paths: "{os.path.basename(p)[:-6]}"\n')


def latest_ckpt(logdir: str):
    c = glob.glob(os.path.join(logdir, "model-*.index"))
    if not c:
        return None
    return max(c, key=lambda p: int(p.split("-")[-1][:-6]))[:-6]


def load_ckpt(model, path: str, opt=None):
    from safetensors.torch import load_file
    if path.endswith(".index"):
        path = path[:-6]
    sd = load_file(path + ".data-00000-of-00001")
    model.load_state_dict(sd, strict=False)
    meta = json.load(open(path + ".index"))
    if opt is not None and os.path.exists(path + ".optim"):
        o = torch.load(path + ".optim", map_location="cpu", weights_only=True)
        opt.load_state_dict(o["optimizer"])
    return meta


# ------------------------------------------------------------------------------ eval
@torch.no_grad()
def run_inference(model, loader, device, with_masks=True):
    """Detections in original-image coordinates, for this rank's share of the data."""
    import numpy as np
    import torch.nn.functional as F
    from mxtrain.data.coco import CONTIG_TO_CAT
    m = model.module if hasattr(model, "module") else model
    m.eval()
    out = []
    for batch in loader:
        res = m(batch["images"].to(device, non_blocking=True), batch["hw"].to(device))
        for i in range(batch["images"].shape[0]):
            s = batch["scales"][i]
            valid = res["valid"][i].cpu()
            boxes = (res["boxes"][i].cpu() / s)[valid]
            scores = res["scores"][i].cpu()[valid]
            labels = res["labels"][i].cpu()[valid]
            rec = {"image_id": batch["image_ids"][i], "boxes": boxes.numpy(), "scores": scores.numpy(),
                   "labels": labels.numpy()}
            if with_masks and "masks" in res:
                rec["mask28"] = res["masks"][i].cpu()[valid].numpy()
            out.append(rec)
    m.train()
    return out


def paste_mask(m28, box, H, W, thresh=0.5):
    import numpy as np
    import torch.nn.functional as F
    x0, y0, x1, y1 = [float(v) for v in box]
    w, h = max(int(round(x1 - x0)), 1), max(int(round(y1 - y0)), 1)
    m = F.interpolate(torch.from_numpy(m28)[None, None], size=(h, w), mode="bilinear", align_corners=False)[0, 0]
    full = np.zeros((H, W), dtype=bool)
    xa, ya = int(round(x0)), int(round(y0))
    xs, ys = max(xa, 0), max(ya, 0)
    xe, ye = min(xa + w, W), min(ya + h, H)
    if xe > xs and ye > ys:
        full[ys:ye, xs:xe] = (m[ys - ya:ye - ya, xs - xa:xe - xa] >= thresh).numpy()
    return full


def coco_evaluate(dets, coco, with_masks=True):
    import numpy as np
    from PIL import Image, ImageDraw
    from mxtrain.workloads.maskrcnn.coco_eval import evaluate, tensorpack_stats
    from mxtrain.data.coco import CAT_TO_CONTIG
    gts_b, gts_m, d_b, d_m = [], [], [], []
    ids = {d["image_id"] for d in dets}
    for iid in ids:
        im = coco.images[iid]
        for a in coco.anns.get(iid, []):
            x, y, w, h = a["bbox"]
            gts_b.append({"image_id": iid, "category": CAT_TO_CONTIG[a["category_id"]],
                          "box": np.array([x, y, x + w, y + h]), "area": a.get("area")})
            if with_masks:
                mk = Image.new("L", (im["width"], im["height"]), 0)
                for poly in a.get("segmentation") or []:
                    ImageDraw.Draw(mk).polygon([tuple(p) for p in np.asarray(poly).reshape(-1, 2).tolist()], fill=1)
                gts_m.append({"image_id": iid, "category": CAT_TO_CONTIG[a["category_id"]],
                              "mask": np.asarray(mk, dtype=bool), "area": a.get("area")})
    for d in dets:
        im = coco.images[d["image_id"]]
        for k in range(len(d["scores"])):
            d_b.append({"image_id": d["image_id"], "category": int(d["labels"][k]), "score": float(d["scores"][k]),
                        "box": d["boxes"][k]})
            if with_masks and "mask28" in d:
                d_m.append({"image_id": d["image_id"], "category": int(d["labels"][k]),
                            "score": float(d["scores"][k]),
                            "mask": paste_mask(d["mask28"][k], d["boxes"][k], im["height"], im["width"])})
    stats = tensorpack_stats(evaluate(d_b, gts_b, "bbox"), "bbox")
    if with_masks and d_m:
        stats.update(tensorpack_stats(evaluate(d_m, gts_m, "segm"), "segm"))
    return stats


# ------------------------------------------------------------------------------ main
def use_shipped_find_db():
    """Point MIOpen's user find/perf db at a writable copy of the in-repo one
    (mxtrain/tuning/miopen: the conv solutions found for the training shapes of this model on
    gfx950 with this image's MIOpen), so a fresh node skips the ~4-minute search.  An
    explicitly set MIOPEN_USER_DB_PATH wins.  Returns the directory or None."""
    if os.environ.get("MIOPEN_USER_DB_PATH"):
        return os.environ["MIOPEN_USER_DB_PATH"]
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                       "tuning", "miopen")
    files = glob.glob(os.path.join(src, "*.txt"))
    if not files:
        return None
    import shutil
    import tempfile
    dst = os.path.join(tempfile.gettempdir(), f"mxtrain-miopen-{os.getuid()}")
    os.makedirs(dst, exist_ok=True)
    for f in files:
        t = os.path.join(dst, os.path.basename(f))
        if not os.path.exists(t) or os.path.getsize(t) < os.path.getsize(f):
            # N ranks of one node copy at once: write a private temporary and rename it
            # into place, so MIOpen never opens a half-written db
            tmp = f"{t}.tmp{os.getpid()}"
            shutil.copyfile(f, tmp)
            os.replace(tmp, t)
    os.environ["MIOPEN_USER_DB_PATH"] = dst
    return dst


def get_args(argv=None):
    p = argparse.ArgumentParser(allow_abbrev=False)
    p.add_argument("--logdir", default="train_log/maskrcnn")
    p.add_argument("--config", nargs="+", default=[])
    p.add_argument("--load", default=None)
    p.add_argument("--images_per_epoch", type=int, default=None)
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--evaluate", default=None, help="write val-set detections to this json and print AP")
    p.add_argument("--predict", nargs="+", default=None, help="images to run inference on")
    p.add_argument("--benchmark", action="store_true")
    p.add_argument("--throughput_log_freq", type=int, default=50)
    p.add_argument("--mx-max-steps", type=int, default=int(os.environ.get("MXTRAIN_MAX_STEPS", "0")) or None,
                   help="stop after N steps (bounded runs / benchmarks)")
    p.add_argument("--mx-warmup-steps", type=int, default=5, help="steps excluded from the images/s figure")
    p.add_argument("--mx-bench-json", default=None, help="append a JSON images/s record to this file")
    p.add_argument("--mx-graph", choices=("auto", "0", "1"), default=os.environ.get("MXTRAIN_GRAPH", "auto"),
                   help="replay the whole training step as a hipGraph (auto: on for 1 GPU, off in debug mode)")
    return p.parse_args(argv)


def main(argv=None):
    args = get_args(argv)
    # The whole-step hipGraph replays under the HIP runtime's graph packet capture (its
    # default: dispatch packets pre-built at instantiation, 0.5 ms of host time per replay
    # at 1 img/GPU instead of 9.0 ms with node-by-node dispatch).  That needs the graph's
    # memset nodes rewritten into fill kernels (graphed.py, csrc/graph.hip): MIOpen's
    # hipMemsetAsync nodes replay wrong in packet-capture mode, which made this step fault
    # after a few replays until round 3 (profiles/r3_s4/).
    from mxtrain.data.coco import AspectGroupedSampler, COCODetection, DetectionDataset, collate
    from mxtrain.models.maskrcnn import MaskRCNN
    from mxtrain.parallel import hvd
    from mxtrain.workloads.maskrcnn import config as C
    from mxtrain.workloads.maskrcnn.weights import load_tensorpack_npz

    cfg = C.make_config(args.config)
    hvd.init()
    world, rank = hvd.size(), hvd.rank()
    device = hvd.device()
    C.finalize(cfg, world, args.images_per_epoch)
    if device.type == "cuda" and hasattr(torch.backends.cuda, "preferred_blas_library"):
        torch.backends.cuda.preferred_blas_library("hipblaslt")
    os.makedirs(args.logdir, exist_ok=True)
    log(f"Config: world {world} x {cfg.TRAIN.BATCH_SIZE_PER_GPU} img/GPU, device {device}, "
        f"lr {cfg.TRAIN.LR:.5f}, steps/epoch {cfg.TRAIN.STEPS_PER_EPOCH}, epochs {cfg.TRAIN.MAX_EPOCH}")
    if rank == 0:
        with open(os.path.join(args.logdir, "config.json"), "w") as f:
            json.dump(cfg.to_dict(), f, indent=1, default=str)
    torch.manual_seed(1234 + rank)
    model = MaskRCNN(C.model_config(cfg))
    calibrate = False
    if cfg.BACKBONE.WEIGHTS and os.path.exists(cfg.BACKBONE.WEIGHTS) and not args.load:
        n = load_tensorpack_npz(model.backbone, cfg.BACKBONE.WEIGHTS)
        log(f"Loaded {n} backbone tensors from {cfg.BACKBONE.WEIGHTS}")
    elif not args.load:
        calibrate = True   # random-init backbone: calibrate FrozenBN on the first batch
    model.to(device)
    short, max_size = cfg.PREPROC.TRAIN_SHORT, int(cfg.PREPROC.MAX_SIZE)
    coll = functools.partial(collate, short=short, max_size=max_size)

    if args.predict or args.evaluate:
        path = args.load or latest_ckpt(args.logdir)
        if path:
            load_ckpt(model, path)
            log(f"Loaded model from {path}")
        if args.predict:
            from mxtrain.predict import predict_images
            predict_images(model, args.predict, device, args.logdir, short, max_size)
            return 0
        val = COCODetection(cfg.DATA.BASEDIR, cfg.DATA.VAL[0], training=False)
        vds = DetectionDataset(val, int(cfg.PREPROC.TEST_SHORT_EDGE_SIZE), max_size, training=False,
                               with_masks=False)
        idx = list(range(rank, len(vds), world))
        vl = torch.utils.data.DataLoader(torch.utils.data.Subset(vds, idx), batch_size=1, collate_fn=coll)
        dets = run_inference(model, vl, device, bool(cfg.MODE_MASK))
        alld = [None] * world
        if world > 1:
            dist.all_gather_object(alld, dets)
            dets = [d for part in alld for d in part]
        if rank == 0:
            stats = coco_evaluate(dets, val, bool(cfg.MODE_MASK))
            log(json.dumps(stats))
            with open(args.evaluate, "w") as f:
                json.dump([{"image_id": d["image_id"], "boxes": d["boxes"].tolist(), "scores": d["scores"].tolist(),
                            "labels": d["labels"].tolist()} for d in dets], f)
        return 0

    # ---------------------------------------------------------------- training
    # Convolution algorithm search: torch's benchmark mode runs MIOpen find once per conv
    # shape and caches the choice, so a steady-state conv call skips the per-call solution
    # query of immediate mode (~30 us host per call, ~240 calls per step) and gets the
    # found solver.  MIOPEN_FIND_MODE=FAST keeps the search to the fast candidates.
    # Measured on one MI355X: 1 img/GPU 51 -> 66 img/s, 4 img/GPU 108 -> 129 img/s; the
    # one-time search costs ~4 minutes on a fresh node (MIOpen's user find-db keeps it for
    # later runs).
    # Training only: the fixed training canvases make the search a one-time cost; predict /
    # evaluate see arbitrary image sizes and stay in immediate mode (evaluate_epoch too).
    torch.backends.cudnn.benchmark = True
    if torch.backends.cudnn.benchmark:
        os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
        db = use_shipped_find_db()
        log("Convolution algorithm search on (MIOpen find, FAST mode)" +
            (f"; find-db {db}" if db else ": the first steps of each input shape take minutes on a node "
             "without a MIOpen find-db"))
    tbw = None
    from mxtrain.obs.profile import StepProfiler, check_finite, check_finite_enabled
    prof = StepProfiler(rank, out_dir=os.path.join(args.logdir, "profile") if os.environ.get("MXTRAIN_PROFILE") else None)
    debug_finite = check_finite_enabled()
    train_sets = [COCODetection(cfg.DATA.BASEDIR, n, training=True) for n in cfg.DATA.TRAIN]
    flat_sgd = device.type == "cuda"
    # whole-step hipGraph: 1 GPU, or world > 1 with the fused flat SGD, whose bucketed
    # gradient all-reduces are captured into the graph -- RCCL by default, or the direct
    # xGMI kernel with MXTRAIN_XGMI=1/auto (checked against RCCL and timed on the live group)
    use_graph = (args.mx_graph == "1" or (args.mx_graph == "auto" and not debug_finite)) \
        and device.type == "cuda" and bool(cfg.MODE_MASK) and (world == 1 or flat_sgd)
    ds = DetectionDataset(train_sets[0], short, max_size, training=True, with_masks=bool(cfg.MODE_MASK), seed=rank,
                          mask_format="crops")
    train_coll = functools.partial(collate, short=short, max_size=max_size, fixed_gt=use_graph)
    bs = int(cfg.TRAIN.BATCH_SIZE_PER_GPU)
    # one endless loader stream for the whole run (tensorpack's RepeatedData): the workers
    # and their prefetch queue never drain at a dataset-epoch boundary, and every global
    # step has one orientation on all ranks
    sampler = AspectGroupedSampler(ds, bs, rank, world, seed=42, repeat=True)
    nw = int(cfg.DATA.NUM_WORKERS)
    loader = torch.utils.data.DataLoader(ds, batch_sampler=sampler, num_workers=nw, collate_fn=train_coll,
                                         pin_memory=device.type == "cuda", persistent_workers=nw > 0,
                                         prefetch_factor=4 if nw > 0 else None)
    decay, no_decay = [], []
    for n_, p in model.named_parameters():
        if p.requires_grad:
            (decay if p.ndim > 1 else no_decay).append(p)
    opt = torch.optim.SGD([{"params": decay, "weight_decay": float(cfg.TRAIN.WEIGHT_DECAY)},
                           {"params": no_decay, "weight_decay": 0.0}], lr=cfg.TRAIN.WARMUP_INIT_LR,
                          momentum=float(cfg.TRAIN.MOMENTUM))
    step = 0
    start_epoch = int(cfg.TRAIN.STARTING_EPOCH)
    ck = args.load or latest_ckpt(args.logdir)
    if ck:
        meta = load_ckpt(model, ck, opt)
        step = int(meta.get("global_step", 0))
        start_epoch = int(meta.get("epoch", 0)) + 1
        log(f"Resumed from {ck} at global_step {step}")
    if calibrate and not ck:
        from mxtrain.models.resnet import calibrate_frozen_bn
        b0 = collate([ds[i] for i in range(min(2, len(ds)))], short, max_size)
        x = (b0["images"].float().to(device) - model.pixel_mean) / model.pixel_std
        calibrate_frozen_bn(model.backbone, x)
        log("Calibrated FrozenBN statistics of the random-init backbone")
    hvd.broadcast_parameters(model.state_dict().values())
    params = decay + no_decay
    clip = float(cfg.TRAIN.GRADIENT_CLIP or 0.0)
    gstep = None
    fm = None
    if flat_sgd:
        # flat fp32 master / grads / momentum + persistent bf16 compute copies: one launch
        # each for the gradient cast, its norm and the clip + SGD + copy refresh; at world > 1
        # the flat gradient is all-reduced bucket by bucket as backward produces it
        from mxtrain.models.compute_weights import FlatMaster
        fm = FlatMaster(model, opt, clip)
        model.__dict__["_flat_master"] = fm
        log("Optimizer: fused flat SGD-momentum (+ clip, + bf16 compute copies)" +
            (f"; data-parallel: {len(fm.buckets)} gradient buckets all-reduced during backward" if world > 1 else ""))
        dmodel = model
    else:
        dmodel = hvd.DistributedDataParallel(model)
    if use_graph:
        from mxtrain.workloads.maskrcnn.graphed import GraphedTrainStep
        from mxtrain.data.coco import canvas
        ch, cw = canvas(short, max_size, 0)
        # every mask crop lies inside its image: bs x max_gt x canvas bytes bound the packed
        # payload, so the buffer (and the graphs that read its address) never regrows --
        # 0.45 GB at 4 img/GPU, sized for 288 GB of HBM
        gstep = GraphedTrainStep(model, opt, params, clip, device, flat_master=fm,
                                 flat_capacity=bs * 100 * ch * cw)
        log("Training step runs as a hipGraph (one graph per input shape)")
    max_steps = args.mx_max_steps
    timed_imgs, t_timed = 0, None
    t_wait = t_enq = 0.0
    done = False
    sampler.set_epoch(start_epoch)
    it = iter(loader)
    for epoch in range(start_epoch, int(cfg.TRAIN.MAX_EPOCH) + 1):
        log(f"Start Epoch {epoch} ...")
        t_ep = time.time()
        for k in range(int(cfg.TRAIN.STEPS_PER_EPOCH)):
            t_a = time.time()
            batch = next(it)
            t_b = time.time()
            lr = C.lr_at(cfg, step)
            for g in opt.param_groups:
                g["lr"] = lr
            if gstep is not None:
                losses = gstep(batch, lr)
            else:
                d = {kk: v.to(device, non_blocking=True) for kk, v in batch.items() if torch.is_tensor(v)}
                losses = dmodel(d["images"], d["hw"], d["gt_boxes"], d["gt_labels"], d["gt_count"],
                                d.get("gt_mask_flat", d.get("gt_masks")), d.get("gt_mask_table"))
                opt.zero_grad(set_to_none=True)
                losses["total_loss"].backward()
                if fm is not None:
                    fm.step(lr)
                else:
                    if clip > 0:
                        torch.nn.utils.clip_grad_norm_(params, clip)
                    opt.step()
            t_c = time.time()
            if t_timed is not None:   # host-side accounting: loader wait vs enqueue time
                t_wait += t_b - t_a
                t_enq += t_c - t_b
            step += 1
            prof.step(step)
            if debug_finite:
                check_finite(step, total_loss=losses["total_loss"])
            if step == args.mx_warmup_steps:
                if device.type == "cuda":
                    torch.cuda.synchronize()
                t_timed, timed_imgs = time.time(), 0
            elif t_timed is not None:
                timed_imgs += bs * world
            if args.verbose or step % args.throughput_log_freq == 0:
                lv = {kk: round(float(v.detach()), 4) for kk, v in losses.items()}
                ips = (timed_imgs / (time.time() - t_timed)) if t_timed and timed_imgs else 0.0
                nst = max(1, step - args.mx_warmup_steps)
                log(f"step {step} lr {lr:.5f} {lv} images/s {ips:.2f} "
                    f"(per step: loader wait {1e3 * t_wait / nst:.1f} ms, host enqueue {1e3 * t_enq / nst:.1f} ms)")
                if rank == 0:   # tensorpack writes its monitors as TensorBoard events in logdir
                    if tbw is None:
                        from mxtrain.obs.tensorboard import SummaryWriter
                        tbw = SummaryWriter(args.logdir)
                    tbw.add_scalars_flat(dict(lv, learning_rate=lr, **({"throughput": ips} if ips else {})),
                                         step)
                    tbw.flush()
            if max_steps and step >= max_steps:
                done = True
                break
        if device.type == "cuda":
            torch.cuda.synchronize()
        t_end = time.time()   # throughput excludes the checkpoint save / eval below
        log(f"Epoch {epoch} (global_step {step}) finished, time:{t_end - t_ep:.2f} sec.")
        last = done or epoch == int(cfg.TRAIN.MAX_EPOCH)
        if rank == 0 and (epoch % int(cfg.TRAIN.CHECKPOINT_PERIOD) == 0 or last):
            save_ckpt(model, opt, args.logdir, step, epoch)
            log(f"Model saved to {os.path.join(args.logdir, f'model-{step}')}")
        if (epoch % int(cfg.TRAIN.EVAL_PERIOD) == 0 or last) and cfg.DATA.VAL:
            evaluate_epoch(model, cfg, coll, device, rank, world, args.logdir, epoch, step)
        if done:
            break
    if t_timed is not None and timed_imgs:
        ips = timed_imgs / (t_end - t_timed)
        log(f"Throughput: {ips:.2f} images/s over {timed_imgs} images ({world} ranks)")
        if gstep is not None:
            log(f"Step path: hipGraph captures {gstep.captures}, replays {gstep.replays}, eager {gstep.eager_steps}"
                + (f"; fused flat SGD, gradient all-reduce via {sorted(fm.dp_routes)}" if fm is not None and world > 1
                   else "; fused flat SGD" if fm is not None else ""))
        if args.mx_bench_json and rank == 0:
            with open(args.mx_bench_json, "a") as f:
                f.write(json.dumps({"metric": "Mask R-CNN R50-FPN train images/sec", "value": round(ips, 2),
                                    "n_gpus": world, "batch_per_gpu": bs,
                                    "graph": None if gstep is None else
                                    {"captures": gstep.captures, "replays": gstep.replays,
                                     "eager": gstep.eager_steps,
                                     "packet_capture": os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "runtime default"),
                                     "nodes": [v for v in gstep.graph_info.values()]},
                                    "flat_sgd": fm is not None,
                                    "loader_wait_ms": round(1e3 * t_wait / max(1, step - args.mx_warmup_steps), 3),
                                    "host_enqueue_ms": round(1e3 * t_enq / max(1, step - args.mx_warmup_steps), 3),
                                    "dp_routes": sorted(fm.dp_routes) if fm is not None else None}) + "\n")
    hvd.shutdown()
    return 0


def evaluate_epoch(model, cfg, coll, device, rank, world, logdir, epoch, step):
    bench = torch.backends.cudnn.benchmark
    torch.backends.cudnn.benchmark = False   # arbitrary validation image sizes: no per-shape find
    try:
        _evaluate_epoch(model, cfg, coll, device, rank, world, logdir, epoch, step)
    finally:
        torch.backends.cudnn.benchmark = bench


def _evaluate_epoch(model, cfg, coll, device, rank, world, logdir, epoch, step):
    from mxtrain.data.coco import COCODetection, DetectionDataset
    try:
        val = COCODetection(cfg.DATA.BASEDIR, cfg.DATA.VAL[0], training=False)
    except FileNotFoundError:
        return
    vds = DetectionDataset(val, int(cfg.PREPROC.TEST_SHORT_EDGE_SIZE), int(cfg.PREPROC.MAX_SIZE), training=False,
                           with_masks=False)
    idx = list(range(rank, len(vds), world))
    vl = torch.utils.data.DataLoader(torch.utils.data.Subset(vds, idx), batch_size=1, collate_fn=coll, num_workers=2)
    dets = run_inference(model, vl, device, bool(cfg.MODE_MASK))
    if world > 1:
        alld = [None] * world
        dist.all_gather_object(alld, dets)
        dets = [d for part in alld for d in part]
    if rank == 0:
        stats = coco_evaluate(dets, val, bool(cfg.MODE_MASK))
        stats.update({"epoch_num": epoch, "global_step": step})
        p = os.path.join(logdir, "stats.json")
        hist = json.load(open(p)) if os.path.exists(p) else []
        hist.append(stats)
        with open(p, "w") as f:
            json.dump(hist, f, indent=1)
        log(" ".join(f"{k}: {v:.4f}" if isinstance(v, float) else f"{k}: {v}" for k, v in stats.items()))


if __name__ == "__main__":
    sys.exit(main())
