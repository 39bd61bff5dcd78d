"""bench.py contract rehearsed on the CPU: two gloo ranks through torch.distributed.run
(127.0.0.1 rendezvous), a tiny GPT, one JSON line from rank 0 with the driver's fields --
the N > 1 path (MAX over ranks, whole-job tokens/s) the scaling runs take on MI355X."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_json_line():
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--model", "gpt-tiny", "--no-maskrcnn",
           "--no-tuned-gemm", "--no-extra-configs"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["parallelism"].startswith("dp2") and d["value"] > 0
    # N > 1 default: xGMI autotune mode; on the CPU the collectives are gloo's
    assert d["config"]["xgmi_mode"] == "auto" and d["config"]["collectives"] == "gloo", d["config"]
    # whole-job tokens/s: global batch x seq / step time
    tok = d["config"]["global_batch"] * d["config"]["seq_len"]
    assert abs(d["value"] - tok / (d["ms_per_step"] / 1000.0)) / d["value"] < 0.01


def test_bench_two_ranks_gloo_maskrcnn_fields(tmp_path):
    """N > 1 Mask R-CNN half of the metric: every bench rank starts one child rank after the
    GPT window, the children rendezvous on a fresh port (torchrun's agent-store variables
    dropped) and rank 0 reports whole-job images/s for n_gpus = 2."""
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2")
    small = ("--images 4 --data {d} PREPROC.TRAIN_SHORT_EDGE_SIZE=[192,192] PREPROC.MAX_SIZE=256 "
             "RPN.TRAIN_PER_LEVEL_NMS_TOPK=200 RPN.TRAIN_POST_NMS_TOPK=200 FRCNN.BATCH_PER_IM=32").format(
                 d=tmp_path / "coco")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29537", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--model", "gpt-tiny", "--no-tuned-gemm",
           "--maskrcnn-batches", "1", "--maskrcnn-steps", "2:1", "--maskrcnn-workers", "0",
           "--maskrcnn-args", small, "--no-extra-configs"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["maskrcnn_img_s_1img"] and d["maskrcnn_img_s_1img"] > 0, d.get("maskrcnn_config")
    mc = d["maskrcnn_config"]
    assert mc["n_gpus"] == 2 and mc["1img"]["n_gpus"] == 2 and mc["parallelism"].startswith("dp2")


def test_bench_two_ranks_gloo_extra_config_fields():
    """BASELINE configs 4 and 5 in the bench line: the GPT-3 phase (a fresh N-rank child job:
    here a tiny GPT through the same --tp / --pp layout rule, TP2 at N = 2) and the
    Ray-Train ResNet-50 phase (rank 0's launcher with N workers; here small CPU images)."""
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29541", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--model", "gpt-tiny", "--no-tuned-gemm",
           "--no-maskrcnn", "--extra-steps", "2:1", "--resnet-steps", "5",
           "--gpt3-args", "--model gpt-tiny --no-tuned-gemm",
           "--resnet-args", "--cpu --batch-size 2 --image-size 64 --loader-workers 0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["gpt3_6.7b_tok_s"] and d["gpt3_6.7b_tok_s"] > 0, (d.get("gpt3_6.7b_config"), r.stderr[-2000:])
    g = d["gpt3_6.7b_config"]
    assert g["n_gpus"] == 2 and g["parallelism"].startswith("dp1_tp2"), g
    assert d["resnet50_img_s"] and d["resnet50_img_s"] > 0, (d.get("resnet50_config"), r.stderr[-2000:])
    assert d["resnet50_config"]["workers"] == 2
