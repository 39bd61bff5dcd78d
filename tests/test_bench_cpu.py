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


def _run2(args, env_extra=None, timeout=600, port=29545):
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2", **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--model", "gpt-tiny", "--no-tuned-gemm"] + args
    import time
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, lines, time.time() - t0


def test_bench_xgmi_preflight_failure_falls_back_to_rccl():
    """The xGMI preflight runs in throwaway children before the bench ranks touch a GPU; a
    child that exits non-zero on ONE rank (rank 1 here) must turn the direct kernels off on
    EVERY rank (MXTRAIN_XGMI=0), with the reason in the line (gloo stand-in children)."""
    r, lines, _ = _run2(["--no-maskrcnn", "--no-extra-configs"],
                        {"MXTRAIN_PREFLIGHT_CPU": "1", "MXTRAIN_PREFLIGHT_FAIL_RANK": "1"}, port=29547)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    pre = d["config"]["xgmi_preflight"]
    assert d["config"]["xgmi_mode"] == "0", d["config"]
    assert pre["ok"] is False and "rank 1" in pre["reason"] and "rc=3" in pre["reason"], pre


def test_bench_xgmi_preflight_success_keeps_auto():
    r, lines, _ = _run2(["--no-maskrcnn", "--no-extra-configs"], {"MXTRAIN_PREFLIGHT_CPU": "1"}, port=29549)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["config"]["xgmi_preflight"]["ok"] is True and d["config"]["xgmi_mode"] == "auto", d["config"]


def test_bench_hung_phase_cannot_erase_headline():
    """A GPT-3 child that never finishes is cut at the budget: the headline line still comes
    out (once), the GPT-3 field carries the timeout, and the ResNet phase that no longer
    fits is recorded as skipped."""
    r, lines, wall = _run2(["--no-maskrcnn", "--budget-s", "45", "--min-phase-s", "3", "--extra-steps", "1:1",
                            "--gpt3-args", "--model gpt-tiny --no-tuned-gemm --test-hang start",
                            "--resnet-args", "--cpu --batch-size 2 --image-size 32 --loader-workers 0"],
                           port=29551)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] and d["value"] > 0
    assert d["gpt3_6.7b_tok_s"] is None and "timeout" in d["gpt3_6.7b_config"]["error"], d["gpt3_6.7b_config"]
    assert "skipped: budget" in d["resnet50_config"]["error"], d["resnet50_config"]
    assert wall < 45 + 40, wall


def test_bench_deadline_prints_measured_fields():
    """A stuck phase inside the bench ranks themselves: the wall-budget thread prints the
    line with what was measured (the GPT-2 headline) and ends the job."""
    r, lines, wall = _run2(["--no-maskrcnn", "--no-extra-configs", "--budget-s", "30", "--test-hang", "after-gpt"],
                           port=29553)
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    d = json.loads(lines[0])
    assert d["value"] and d["value"] > 0 and "deadline" in d
    assert wall < 30 + 40, wall
