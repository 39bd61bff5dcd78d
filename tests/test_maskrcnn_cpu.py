"""Mask R-CNN workload plumbing on CPU: tensorpack --config parsing and schedule
derivation, COCO-format synthetic data + loader, COCO AP evaluator, model forward /
backward / inference shapes, checkpoint + predictor round trip."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tensorpack_config_overrides_and_schedule():
    from mxtrain.workloads.maskrcnn import config as C
    cfg = C.make_config(["MODE_MASK=True", "DATA.TRAIN=[\"coco_train2017\"]", "DATA.VAL=(\"coco_val2017\")",
                         "TRAIN.LR_SCHEDULE=[240000,320000,360000]", "TRAIN.BASE_LR=0.01", "TRAINER=horovod",
                         "TRAIN.STEPS_PER_EPOCH=7500", "BACKBONE.NORM=FreezeBN"])
    C.finalize(cfg, 16)
    assert cfg.DATA.VAL == ("coco_val2017",) and cfg.TRAINER == "horovod"
    assert abs(cfg.TRAIN.LR - 0.02) < 1e-9                 # linear scaling from total batch 8 to 16
    assert cfg.TRAIN.LR_STEPS[0][0] == 120000 and cfg.TRAIN.MAX_EPOCH == 24
    aws = C.make_config(["TRAIN.BATCH_SIZE_PER_GPU=4", "TRAIN.LR_EPOCH_SCHEDULE=[(16, 0.1), (20, 0.01), (24, None)]",
                         "TRAIN.BASE_LR=0.0015625", "DATA.TRAIN=[\"train2017\"]"])
    C.finalize(aws, 16, images_per_epoch=120000)
    assert abs(aws.TRAIN.LR - 0.1) < 1e-9 and aws.TRAIN.STEPS_PER_EPOCH == 1875 and aws.TRAIN.MAX_EPOCH == 24
    assert C.lr_at(aws, 17 * 1875) == pytest.approx(0.01)


def test_coco_eval_perfect_and_empty():
    from mxtrain.workloads.maskrcnn.coco_eval import evaluate
    gts = [{"image_id": 1, "category": 3, "box": np.array([0, 0, 10, 10.])},
           {"image_id": 1, "category": 5, "box": np.array([20, 20, 40, 50.])}]
    dets = [dict(g, score=0.9) for g in gts]
    assert evaluate(dets, gts)["AP"] == pytest.approx(1.0)
    shifted = [dict(g, score=0.9, box=g["box"] + 100) for g in gts]
    assert evaluate(shifted, gts)["AP"] == pytest.approx(0.0)


def test_coco_eval_area_ranges_and_recall():
    """COCOeval's area-range ignore rules and maxDets recall, hand-checked:
    one small and one large GT; the large one is found (0.9), a small FP fires (0.8)."""
    from mxtrain.workloads.maskrcnn.coco_eval import evaluate, tensorpack_stats
    gts = [{"image_id": 1, "category": 1, "box": np.array([0, 0, 10, 10.])},
           {"image_id": 1, "category": 1, "box": np.array([0, 0, 200, 200.])}]
    dets = [{"image_id": 1, "category": 1, "score": 0.9, "box": np.array([0, 0, 200, 200.])},
            {"image_id": 1, "category": 1, "score": 0.8, "box": np.array([500, 500, 505, 505.])}]
    r = evaluate(dets, gts)
    assert r["AP"] == pytest.approx(51 / 101)      # recall 0.5 at precision 1: 51 of 101 points
    assert r["APl"] == pytest.approx(1.0)          # the small FP is outside the range -> ignored
    assert r["APs"] == pytest.approx(0.0)          # large det matched an ignored GT; small FP counts
    assert r["APm"] == -1.0                        # no medium GT: missing, as COCOeval prints
    assert r["AR1"] == pytest.approx(0.5) and r["AR100"] == pytest.approx(0.5)
    assert r["ARl"] == pytest.approx(1.0) and r["ARs"] == pytest.approx(0.0)
    st = tensorpack_stats(r, "bbox")
    assert set(st) == {"mAP(bbox)/IoU=0.5:0.95", "mAP(bbox)/IoU=0.5", "mAP(bbox)/IoU=0.75", "mAP(bbox)/small",
                       "mAP(bbox)/medium", "mAP(bbox)/large"}
    # an explicit annotation area (COCO segment area) decides the range, not the box
    gts2 = [dict(gts[1], area=500.0)]
    r2 = evaluate(dets[:1], gts2)
    assert r2["APs"] == pytest.approx(1.0) and r2["APl"] == -1.0


@pytest.fixture(scope="module")
def coco_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("coco")
    from mxtrain.data.coco_synth import write_split
    write_split(str(d), "train2017", 6, 0, 1)
    write_split(str(d), "val2017", 3, 1, 1_000_000)
    write_split(str(d), "test2017", 1, 2, 2_000_000, with_anns=False)
    os.makedirs(d / "pretrained-models")
    return str(d)


def test_loader_shapes(coco_dir):
    from mxtrain.data.coco import AspectGroupedSampler, COCODetection, DetectionDataset, collate
    ds = DetectionDataset(COCODetection(coco_dir, "coco_train2017"), 320, 512)
    s = AspectGroupedSampler(ds, 2)
    for b in s:
        batch = collate([ds[i] for i in b], 320, 512)
        B, _, H, W = batch["images"].shape
        assert (H, W) in ((320, 512), (512, 320))
        assert batch["gt_masks"].shape[:2] == (B, (batch["gt_boxes"].shape[1] + 7) // 8 * 8)
        n = int(batch["gt_count"][0])
        x1, y1, x2, y2 = batch["gt_boxes"][0, 0].tolist()
        m = batch["gt_masks"][0, 0]
        assert m.sum() > 0 and m[int(y1):int(y2) + 1, int(x1):int(x2) + 1].sum() == m.sum()


def test_train_cli_checkpoint_and_predict(coco_dir, tmp_path):
    env = dict(os.environ, PYTHONPATH=REPO, MXTRAIN_CPU_ONLY="1")
    logdir = tmp_path / "train_log" / "maskrcnn"
    common = [f"DATA.BASEDIR={coco_dir}", "PREPROC.TRAIN_SHORT_EDGE_SIZE=[256,256]", "PREPROC.MAX_SIZE=384",
              "PREPROC.TEST_SHORT_EDGE_SIZE=256", "DATA.NUM_WORKERS=0", "RPN.TRAIN_PER_LEVEL_NMS_TOPK=300",
              "RPN.TRAIN_POST_NMS_TOPK=300", "RPN.TEST_PER_LEVEL_NMS_TOPK=200", "RPN.TEST_POST_NMS_TOPK=200",
              "FRCNN.BATCH_PER_IM=64"]
    r = subprocess.run([sys.executable, os.path.join(REPO, "mxtrain", "workloads", "maskrcnn", "train.py"),
                        "--logdir", str(logdir), "--mx-max-steps", "2", "--config", "MODE_MASK=True",
                        "MODE_FPN=True", "TRAINER=horovod", "TRAIN.STEPS_PER_EPOCH=2", "TRAIN.EVAL_PERIOD=1",
                        "TRAIN.CHECKPOINT_PERIOD=1"] + common, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "Epoch 1 (global_step 2) finished" in r.stdout
    assert (logdir / "model-2.index").exists() and (logdir / "checkpoint").exists()
    stats = json.load(open(logdir / "stats.json"))
    assert stats[-1]["global_step"] == 2 and "mAP(bbox)/IoU=0.5:0.95" in stats[-1]
    r = subprocess.run([sys.executable, "-m", "mxtrain.predict", "--logdir", str(tmp_path), "--data-dir", coco_dir,
                        "--score-thresh", "0.0", "--config"] + common, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert os.path.exists(rec["output"])


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_jupyter_chart_viewer_serves_predictions(coco_dir, tmp_path, monkeypatch):
    """maskrcnn-jupyter chart -> Deployment (prediction + metrics viewers) on the
    checkpoint of a 1-step training run; basic auth enforced."""
    import base64
    import hashlib
    import shutil
    import time
    import urllib.request
    monkeypatch.setenv("MXTRAIN_HOME", str(tmp_path / "home"))
    monkeypatch.setenv("MXTRAIN_NUM_GPUS", "0")
    monkeypatch.setenv("MXTRAIN_PV_LINK", "0")
    monkeypatch.setenv("MXTRAIN_CPU_ONLY", "1")
    pv = tmp_path / "home" / "pv" / "pv-fsx"
    logdir = pv / "logs" / "run1" / "train_log" / "maskrcnn"
    shutil.copytree(coco_dir, pv / "data" / "coco2017")
    env = dict(os.environ, PYTHONPATH=REPO)
    common = [f"DATA.BASEDIR={pv / 'data' / 'coco2017'}", "PREPROC.TRAIN_SHORT_EDGE_SIZE=[256,256]",
              "PREPROC.MAX_SIZE=384", "DATA.NUM_WORKERS=0", "RPN.TRAIN_PER_LEVEL_NMS_TOPK=300",
              "RPN.TRAIN_POST_NMS_TOPK=300", "FRCNN.BATCH_PER_IM=64"]
    r = subprocess.run([sys.executable, os.path.join(REPO, "mxtrain", "workloads", "maskrcnn", "train.py"),
                        "--logdir", str(logdir), "--mx-max-steps", "1", "--config", "TRAIN.STEPS_PER_EPOCH=1",
                        "TRAIN.EVAL_PERIOD=100", "DATA.VAL=()"] + common, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    with open(logdir / "stats.json", "w") as f:
        json.dump([{"epoch_num": 1, "global_step": 1, "mAP(bbox)/IoU=0.5:0.95": 0.0}], f)
    from mxtrain.launch import release as rel
    p1, p2 = _free_port(), _free_port()
    pw_hash = "{SHA}" + base64.b64encode(hashlib.sha1(b"secret").digest()).decode()
    rel.install(os.path.join(REPO, "charts", "machine-learning", "testing", "maskrcnn-jupyter"), "viewer",
                sets=["global.log_dir=logs/run1", f"jupyter.target_port={p1}", f"tensorboard.target_port={p2}",
                      "global.source_cidr=127.0.0.1/32", "nginx.tls=off"],
                set_strings=[f"nginx.htpasswd={pw_hash}"])
    try:
        auth = {"Authorization": "Basic " + base64.b64encode(b"tensorboard:secret").decode()}
        deadline = time.time() + 60
        while True:
            try:
                urllib.request.urlopen(urllib.request.Request(f"http://127.0.0.1:{p2}/healthz", headers=auth),
                                       timeout=2)
                break
            except Exception:  # noqa: BLE001
                assert time.time() < deadline, rel.logs("viewer")
                time.sleep(0.5)
        with pytest.raises(urllib.error.HTTPError):
            urllib.request.urlopen(f"http://127.0.0.1:{p2}/stats.json", timeout=5)
        stats = json.loads(urllib.request.urlopen(urllib.request.Request(
            f"http://127.0.0.1:{p2}/stats.json", headers=auth), timeout=10).read())
        assert stats[0]["global_step"] == 1
        rec = json.loads(urllib.request.urlopen(urllib.request.Request(
            f"http://127.0.0.1:{p1}/predict.json", headers=auth), timeout=120).read())
        assert rec["output"].endswith(".png") and isinstance(rec["boxes"], list)
        # ?image= is confined to --data-dir
        with pytest.raises(urllib.error.HTTPError) as ei:
            urllib.request.urlopen(urllib.request.Request(
                f"http://127.0.0.1:{p1}/predict.json?image=/etc/passwd", headers=auth), timeout=30)
        assert ei.value.code == 403
    finally:
        rel.uninstall("viewer")


def test_jupyter_chart_requires_auth_and_cidr():
    """the internet-facing testing charts must not render without an htpasswd
    and a source CIDR (the reference marks both `required`)."""
    from mxtrain.chart.render import load_chart, render_chart
    from mxtrain.chart.template import TemplateError
    for chart in ("maskrcnn-jupyter", "maskrcnn-optimized-jupyter"):
        c = load_chart(os.path.join(REPO, "charts", "machine-learning", "testing", chart))
        with pytest.raises(TemplateError, match="source_cidr"):
            render_chart(c, "v", set_strings=["nginx.htpasswd=x"])
        with pytest.raises(TemplateError, match="htpasswd"):
            render_chart(c, "v", sets=["global.source_cidr=10.0.0.0/8"])
        r = render_chart(c, "v", sets=["global.source_cidr=10.0.0.0/8"], set_strings=["nginx.htpasswd=x"])
        dep = [m for m in r.manifests if m["kind"] == "Deployment"][0]
        for ctr in dep["spec"]["template"]["spec"]["containers"]:
            assert "--htpasswd=/etc/nginx/.htpasswd" in ctr["args"] and "--tls=auto" in ctr["args"]


def test_viewer_fails_closed(tmp_path):
    from mxtrain.serve import viewer
    logdir = str(tmp_path)
    # no auth configured on a public bind address, a missing htpasswd, an empty one, a
    # missing certificate: the server refuses to start (exit 2) instead of degrading
    assert viewer.main(["--logdir", logdir]) == 2
    assert viewer.main(["--logdir", logdir, "--insecure-no-auth"]) == 2          # 0.0.0.0
    assert viewer.main(["--logdir", logdir, "--htpasswd", str(tmp_path / "none")]) == 2
    (tmp_path / "empty").write_text("\n")
    assert viewer.main(["--logdir", logdir, "--htpasswd", str(tmp_path / "empty")]) == 2
    (tmp_path / "pw").write_text("u:{SHA}abc\n")
    assert viewer.main(["--logdir", logdir, "--htpasswd", str(tmp_path / "pw"),
                        "--certfile", str(tmp_path / "c.crt"), "--keyfile", str(tmp_path / "c.key")]) == 2
    data = tmp_path / "data"
    (data / "test2017").mkdir(parents=True)
    (data / "test2017" / "a.jpg").write_bytes(b"x")
    assert viewer.safe_image_path(str(data), "test2017/a.jpg").endswith("a.jpg")
    for bad in ("/etc/passwd", "../pw", "test2017/../../pw"):
        with pytest.raises(PermissionError):
            viewer.safe_image_path(str(data), bad)


def test_prediction_flow_thresholds(tmp_path):
    """The notebooks' visualisation flow (mask-rcnn-tensorflow-viz.ipynb show_detection_results,
    get_mask; mask-rcnn-tensorpack-viz.ipynb newest model-*.index): newest checkpoint, boxes
    with score >= 0.7 only, mask pixels where the pasted mask >= 0.5."""
    import numpy as np
    from PIL import Image
    from mxtrain.predict import predict_images
    from mxtrain.workloads.maskrcnn.train import latest_ckpt
    for step in (5, 120, 40):
        (tmp_path / f"model-{step}.index").write_text("")
    assert latest_ckpt(str(tmp_path)).endswith("model-120")
    Image.fromarray(np.zeros((64, 96, 3), dtype=np.uint8)).save(tmp_path / "img.jpg")
    m = torch.zeros(3, 28, 28)
    m[0, :14] = 0.9      # top half above the mask threshold
    m[1] = 0.49          # everywhere just below it
    m[2] = 1.0

    class Fake(torch.nn.Module):
        def forward(self, images, sizes):
            return {"boxes": torch.tensor([[[0., 0., 40., 40.], [10., 10., 30., 30.], [5., 5., 9., 9.]]]),
                    "scores": torch.tensor([[0.95, 0.70, 0.69]]),
                    "labels": torch.tensor([[1, 2, 3]]), "masks": m[None]}
    rec = predict_images(Fake(), [str(tmp_path / "img.jpg")], "cpu", str(tmp_path / "out"), short=64, max_size=96)[0]
    assert rec["scores"] == pytest.approx([0.95, 0.7])   # 0.69 < 0.7 dropped
    assert rec["mask_pixels"][1] == 0                    # 0.49 < 0.5 everywhere
    assert 0 < rec["mask_pixels"][0] < 40 * 40
    assert os.path.exists(rec["output"])


def _small_model_cfg():
    from mxtrain.models.maskrcnn import MaskRCNNConfig
    return MaskRCNNConfig(train_per_level_topk=300, train_post_nms_topk=300, frcnn_batch_per_im=64,
                          fc_dim=256, mask_head_dim=64)


def test_mask_crops_equal_full_masks(coco_dir):
    """Packed per-instance crops carry the full-image masks (up to PIL tie rounding at
    single pixels), and the crop-table target op equals the full-mask op on them."""
    from mxtrain.data.coco import COCODetection, DetectionDataset, collate, unpack_mask_crops
    from mxtrain.ops import vision as V
    coco = COCODetection(coco_dir, "coco_train2017")
    full = DetectionDataset(coco, 320, 512)
    crop = DetectionDataset(coco, 320, 512, mask_format="crops")
    idx = [0, 1]
    bf = collate([full[i] for i in idx], 320, 512)
    bc = collate([crop[i] for i in idx], 320, 512, fixed_gt=True, max_gt=16)
    assert bc["gt_boxes"].shape[1] == 16 and bc["gt_mask_table"].shape == (2, 16, 5)
    B, G = bf["gt_boxes"].shape[:2]
    H, W = bf["images"].shape[2:]
    un = unpack_mask_crops(bc["gt_mask_flat"], bc["gt_mask_table"], H, W)
    ref = bf["gt_masks"][:, :G]
    mism = (un[:, :G] != ref).sum().item()
    assert mism <= max(2, ref.numel() // 100000), mism
    assert un[:, G:].sum() == 0 and bc["gt_mask_flat"].numel() < ref.numel() // 2
    g = torch.Generator().manual_seed(0)
    R = 40
    gid = torch.randint(0, G, (R,), generator=g)
    bi = torch.randint(0, B, (R,), generator=g)
    boxes = torch.gather(bf["gt_boxes"][bi], 1, gid[:, None, None].expand(-1, 1, 4))[:, 0]
    boxes = boxes + torch.randn(R, 4, generator=g) * 4
    a = V.crop_resize_mask_crops(bc["gt_mask_flat"], bc["gt_mask_table"].reshape(-1, 5), H, W, boxes,
                                 bi * 16 + gid)
    b = V.crop_resize_masks(un.reshape(-1, H, W), boxes, bi * 16 + gid)
    torch.testing.assert_close(a, b)


def test_sgd_momentum_matches_torch_sgd():
    from mxtrain.workloads.maskrcnn.graphed import sgd_momentum_
    torch.manual_seed(0)
    ps = [torch.randn(5, 3), torch.randn(7)]
    qs = [p.clone() for p in ps]
    o1 = torch.optim.SGD([{"params": [ps[0]], "weight_decay": 1e-4}, {"params": [ps[1]], "weight_decay": 0.0}],
                         lr=0.1, momentum=0.9)
    o2 = torch.optim.SGD([{"params": [qs[0]], "weight_decay": 1e-4}, {"params": [qs[1]], "weight_decay": 0.0}],
                         lr=0.1, momentum=0.9)
    for it in range(4):
        gs = [torch.randn_like(p) for p in ps]
        lr = 0.1 * (it + 1)
        for p, q, gg in zip(ps, qs, gs):
            p.grad, q.grad = gg.clone(), gg.clone()
        for grp in o1.param_groups:
            grp["lr"] = lr
        o1.step()
        sgd_momentum_(o2, torch.tensor(lr) if it % 2 else lr)
        for p, q in zip(ps, qs):
            torch.testing.assert_close(p, q, rtol=1e-6, atol=1e-6)
    # the state dict stays torch.optim.SGD's (checkpoints interchange)
    assert set(o2.state[qs[0]]) == {"momentum_buffer"}


def test_model_losses_crops_equal_full(coco_dir):
    """Training losses from packed crops == from the same masks unpacked to full images."""
    from mxtrain.data.coco import COCODetection, DetectionDataset, collate, unpack_mask_crops
    from mxtrain.models.maskrcnn import MaskRCNN
    crop = DetectionDataset(COCODetection(coco_dir, "coco_train2017"), 256, 384, mask_format="crops")
    b = collate([crop[0], crop[1]], 256, 384, fixed_gt=True, max_gt=12)
    H, W = b["images"].shape[2:]
    full = unpack_mask_crops(b["gt_mask_flat"], b["gt_mask_table"], H, W)
    torch.manual_seed(0)
    m = MaskRCNN(_small_model_cfg()).train()
    out = []
    for masks, table in ((b["gt_mask_flat"], b["gt_mask_table"]), (full, None)):
        torch.manual_seed(5)
        with torch.no_grad():
            out.append(m(b["images"], b["hw"], b["gt_boxes"], b["gt_labels"], b["gt_count"], masks, table))
    for k in out[0]:
        torch.testing.assert_close(out[0][k], out[1][k], rtol=1e-5, atol=1e-6)


def test_compute_weights_batched_cast_matches_per_tensor_casts():
    """models/compute_weights.py: one autograd node producing every bf16 compute copy
    (with a folded per-channel scale) gives the same outputs and fp32 gradients as the
    per-module casts it replaces."""
    import torch.nn.functional as F
    from mxtrain.models.compute_weights import ComputeWeights, cw
    torch.manual_seed(0)
    lin = torch.nn.Linear(8, 4)
    conv = torch.nn.Conv2d(3, 5, 3)
    s = (torch.rand(5, 1, 1, 1) + 0.5).expand_as(conv.weight).contiguous()
    x = torch.randn(2, 8).bfloat16()
    xi = torch.randn(2, 3, 6, 6).bfloat16()
    bf = torch.bfloat16

    def step(batched):
        for p in (lin.weight, lin.bias, conv.weight):
            p.grad = None
        specs = [(conv.weight, s), (lin.weight, None), (lin.bias, None)]
        with ComputeWeights(specs if batched else [], bf):
            wc = cw(conv.weight, bf) if batched else (conv.weight * s).to(bf)
            y = F.conv2d(xi, wc).float().square().sum() + F.linear(x, cw(lin.weight, bf), cw(lin.bias, bf)).float().square().sum()
        y.backward()
        return float(y), [p.grad.clone() for p in (lin.weight, lin.bias, conv.weight)]

    ya, ga = step(False)
    yb, gb = step(True)
    # (the batched conv copy is channels_last, so the bf16 conv may sum in another order)
    assert abs(ya - yb) <= 1e-5 * abs(ya)
    for a, b in zip(ga[:2], gb[:2]):
        assert a.dtype == torch.float32 and torch.equal(a, b)
    assert gb[2].dtype == torch.float32 and torch.allclose(ga[2], gb[2], rtol=2e-2, atol=1e-2)


@pytest.mark.parametrize("shapes", [[(16, 48), (8, 24), (4, 12), (2, 6), (1, 3)],    # landscape: one shelf
                                    [(48, 16), (24, 8), (12, 4), (6, 2), (3, 1)]])   # no fit: per level
def test_rpn_level_canvas_matches_per_level(shapes):
    """models/maskrcnn.py RPNHead.forward_levels (all FPN levels on one canvas, cls + box as
    one conv) against the per-level head, fp64: outputs and every gradient exact."""
    from mxtrain.models.maskrcnn import RPNHead, level_canvas
    torch.manual_seed(0)
    h = RPNHead(32, 3).double()
    for m in (h.conv, h.cls, h.box):
        torch.nn.init.normal_(m.weight, std=0.1)
        torch.nn.init.normal_(m.bias, std=0.1)
    P = [torch.randn(2, 32, a, b, dtype=torch.float64).contiguous(memory_format=torch.channels_last).requires_grad_()
         for a, b in shapes]
    res = {}
    try:
        for pack in (False, True):
            RPNHead.pack_levels = pack
            h.zero_grad()
            for p in P:
                p.grad = None
            lv = h.forward_levels(P)
            g = torch.Generator().manual_seed(1)
            loss = sum((l * torch.randn(l.shape, generator=g, dtype=l.dtype)).sum()
                       + (d * torch.randn(d.shape, generator=g, dtype=d.dtype)).sum() for l, d in lv)
            loss.backward()
            res[pack] = [t for l, d in lv for t in (l, d)] + [p.grad for p in P] + [q.grad for q in h.parameters()]
    finally:
        RPNHead.pack_levels = True
    assert (level_canvas(shapes) is None) == (shapes[0][0] > shapes[0][1])
    for a, b in zip(res[False], res[True]):
        assert a.shape == b.shape
        torch.testing.assert_close(a, b, rtol=0, atol=1e-10)


def test_sampler_global_step_orientation_lockstep(tmp_path):
    """Every global step has ONE orientation on all ranks (graphed.py captures a new canvas
    shape on every rank together), ranks draw disjoint images, and the endless stream
    (repeat=True) crosses epochs with the epoch folded into the indices."""
    from mxtrain.data.coco import AspectGroupedSampler, COCODetection, DetectionDataset
    from mxtrain.data.coco_synth import write_split
    write_split(str(tmp_path), "train2017", 40, 0, 1)
    ds = DetectionDataset(COCODetection(str(tmp_path), "coco_train2017"), 256, 384)
    n = len(ds)
    orients = {ds.orientation(i) for i in range(n)}
    assert orients == {0, 1}
    for world, bs in ((2, 1), (2, 2), (4, 1)):
        streams = [AspectGroupedSampler(ds, bs, r, world, seed=42, repeat=True) for r in range(world)]
        its = [iter(s) for s in streams]
        per_epoch = len(streams[0])
        seen = set()
        for step in range(3 * per_epoch):
            bl = [next(it) for it in its]
            o = {ds.orientation(i % n) for b in bl for i in b}
            assert len(o) == 1, (world, bs, step, bl)
            flat = [i for b in bl for i in b]
            assert len(flat) == len(set(flat)) == world * bs
            if step < per_epoch:
                assert all(i < n for i in flat)
                seen.update(flat)
            else:
                assert all(i >= n * (step // per_epoch) for i in flat)
        # an epoch covers all but the remainder batches of each orientation
        assert len(seen) >= n - 2 * world * bs
        # the finite (default) iterator yields exactly one epoch
        assert len(list(AspectGroupedSampler(ds, bs, 0, world, seed=42))) == per_epoch
    # the dataset maps a folded index back (epoch 2, image 3)
    assert ds[2 * n + 3]["image_id"] == ds[3]["image_id"]
