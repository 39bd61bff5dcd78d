"""The shipped example values files, end to end on CPU through the launcher (SURVEY §7.3
minimum slice): data-process(wikicorpus) -> pytorchjob-distributed(pretrain-ddp-zero1)
with the model shrunk and iterations cut, everything else as in the example file."""
import json
import os
import re

import pytest
import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(REPO, "examples")
CHARTS = os.path.join(REPO, "charts", "machine-learning")

TINY_GPT = ('  - export GPT_ARGS="--num-layers 2 --hidden-size 64 --num-attention-heads 2 --seq-length 32 '
            '--max-position-embeddings 32 --micro-batch-size 2 --lr 0.00015 --train-iters 6 --lr-decay-iters 6 '
            '--lr-decay-style cosine --min-lr 1.0e-5 --weight-decay 1e-2 --lr-warmup-fraction .01 --clip-grad 1.0 --fp16"')


def _shrink(path, tmp_path, nproc=2):
    doc = yaml.safe_load(open(path))
    pre = []
    for line in doc.get("pre_script", []):
        if line.startswith("export GPT_ARGS="):
            line = TINY_GPT[4:]
        if line.startswith("export OUTPUT_ARGS="):
            line = 'export OUTPUT_ARGS="--log-interval 2 --save-interval 3 --eval-interval 3 --eval-iters 1"'
        line = line.replace('train_micro_batch_size_per_gpu\\": 4', 'train_micro_batch_size_per_gpu\\": 2')
        line = re.sub(r'"train_micro_batch_size_per_gpu": \d+', '"train_micro_batch_size_per_gpu": 2', line)
        pre.append(line)
    doc["pre_script"] = pre
    for k in ("requests", "limits"):
        doc.setdefault("resources", {})[k] = {}
    if "nproc_per_node" in doc["resources"]:
        doc["resources"]["nproc_per_node"] = nproc
    out = tmp_path / os.path.basename(path)
    out.write_text(yaml.safe_dump(doc))
    return str(out)


@pytest.fixture()
def home(tmp_path, monkeypatch):
    monkeypatch.setenv("MXTRAIN_HOME", str(tmp_path / "home"))
    monkeypatch.setenv("MXTRAIN_NUM_GPUS", "0")
    monkeypatch.setenv("MXTRAIN_PV_LINK", "0")
    monkeypatch.setenv("NUM_DOCS", "300")
    return tmp_path


def test_wikicorpus_then_pretrain_ddp_zero1(home):
    from mxtrain.launch import release as rel
    vals = _shrink(os.path.join(EX, "megatron-deepspeed", "gpt2_345m", "wikicorpus.yaml"), home)
    st = rel.install(os.path.join(CHARTS, "data-prep", "data-process"), "mds-gpt2-345m", value_files=[vals],
                     wait=True, timeout=600)
    log = rel.logs("mds-gpt2-345m")
    assert st["phase"] == "Succeeded", log
    data = home / "home" / "pv" / "pv-fsx" / "home" / "mds-gpt2-345m" / "data" / "wikicorpus"
    assert (data / "gpt2_text_document.bin").exists() and (data / "gpt2-vocab.json").exists()
    rel.uninstall("mds-gpt2-345m")

    vals = _shrink(os.path.join(EX, "megatron-deepspeed", "gpt2_345m", "pretrain-ddp-zero1.yaml"), home)
    st = rel.install(os.path.join(CHARTS, "training", "pytorchjob-distributed"), "mds-gpt2-345m",
                     value_files=[vals], wait=True, timeout=900)
    log = rel.logs("mds-gpt2-345m")
    assert st["phase"] == "Succeeded", log
    assert "Training script done" in log
    assert "validation loss at iteration 3" in log
    ck = home / "home" / "pv" / "pv-fsx" / "home" / "mds-gpt2-345m" / "checkpoints" / "0"
    assert open(ck / "latest").read() == "global_step6"
    assert sorted(os.listdir(ck / "global_step6")) == [
        "mp_rank_00_model_states.pt", "zero_pp_rank_0_mp_rank_00_optim_states.pt",
        "zero_pp_rank_1_mp_rank_00_optim_states.pt"]
    out_log = home / "home" / "pv" / "pv-efs" / "home" / "mds-gpt2-345m" / "logs" / "0" / "pretrain-ddp-zero1.log"
    assert "iteration        6/       6" in out_log.read_text()


def test_config1_accelerate_bert_base_mrpc_cpu(home, monkeypatch):
    """BASELINE config 1: Accelerate BERT-base GLUE MRPC on CPU, world_size=1, through the
    elastic training chart."""
    from mxtrain.launch import release as rel
    monkeypatch.setenv("MAX_TRAIN_STEPS", "3")
    monkeypatch.setenv("MXTRAIN_CPU_ONLY", "1")
    vals = os.path.join(EX, "accelerate", "bert-glue-mrpc", "pretrain-cpu.yaml")
    st = rel.install(os.path.join(CHARTS, "training", "pytorchjob-elastic"), "accel-bert", value_files=[vals],
                     wait=True, timeout=900)
    log = rel.logs("accel-bert")
    assert st["phase"] == "Succeeded", log
    assert "epoch 0:" in log and "Training script done" in log
    hd = home / "home" / "pv" / "pv-efs" / "home" / "accel-bert"
    ck = hd / "checkpoints" / "pytorchjob-accel-bert-worker-0" / "epoch_0"
    assert (ck / "model.safetensors").exists() and (ck / "optimizer.bin").exists()
    metrics = hd / "project" / "pytorchjob-accel-bert-worker-0" / "complete_nlp_example" / "metrics.jsonl"
    rec = [json.loads(x) for x in metrics.read_text().splitlines()]
    assert rec[0]["epoch"] == 0 and 0.0 <= rec[0]["accuracy"] <= 1.0
    from safetensors.torch import load_file
    sd = load_file(str(ck / "model.safetensors"))
    assert sd["word_embeddings"].shape == (28996, 768) and len([k for k in sd if k.startswith("layers.")]) == 12 * 12


def test_raytrain_lightning_bert_example_cpu(home, monkeypatch):
    """raytrain chart -> RayJob controller -> raylike TorchTrainer worker group -> Lightning
    BERT loop (shrunk through env; CPU)."""
    import yaml as _y
    from mxtrain.launch import release as rel
    monkeypatch.setenv("MXTRAIN_CPU_ONLY", "1")
    doc = _y.safe_load(open(os.path.join(EX, "ray", "lightning-bert", "fine-tune.yaml")))
    doc["resources"] = {"requests": {}, "limits": {}, "nnodes": 2, "node_type": None}
    doc["train"]["args"] = ["$MXTRAIN_WORKLOADS/ray/fine_tune_text_classifier.py", "--model bert-tiny", "--cpu",
                            "--epochs 1", "--train-size 64", "--eval-size 32", "--storage-path $HOME/ray_results",
                            "2>&1 | tee $OUTPUT_LOG"]
    p = home / "ray.yaml"
    p.write_text(_y.safe_dump(doc))
    st = rel.install(os.path.join(CHARTS, "training", "raytrain"), "ray-bert", value_files=[str(p)], wait=True,
                     timeout=900)
    log = rel.logs("ray-bert")
    assert st["phase"] == "Succeeded", log
    assert "starting worker group: 2 workers" in log and "Training result:" in log
    res = home / "home" / "pv" / "pv-efs" / "home" / "ray-bert" / "ray_results" / "ptl-sent-classification"
    assert (res / "checkpoint_000000" / "checkpoint.ckpt").exists()


SMALL_MRCNN = ["PREPROC.TRAIN_SHORT_EDGE_SIZE=[256,256]", "PREPROC.MAX_SIZE=384", "PREPROC.TEST_SHORT_EDGE_SIZE=256",
               "DATA.NUM_WORKERS=0", "RPN.TRAIN_PER_LEVEL_NMS_TOPK=300", "RPN.TRAIN_POST_NMS_TOPK=300",
               "RPN.TEST_PER_LEVEL_NMS_TOPK=200", "RPN.TEST_POST_NMS_TOPK=200", "FRCNN.BATCH_PER_IM=64"]


def test_coco_data_then_mpijob_maskrcnn_cpu(home, monkeypatch):
    """coco-data chart (synthetic COCO on the PVC) -> mpijob chart with the tensorpack
    example: 2 ranks through the mpirun emulator, horovod-style RCCL/gloo DDP."""
    import yaml as _y
    from mxtrain.launch import release as rel
    monkeypatch.setenv("MXTRAIN_CPU_ONLY", "1")
    monkeypatch.setenv("MXTRAIN_MAX_STEPS", "2")
    st = rel.install(os.path.join(CHARTS, "data-prep", "coco-data"), "coco", value_files=[
        os.path.join(EX, "maskrcnn", "coco-data.yaml")], sets=["synthetic.num_train=6", "synthetic.num_val=2",
                                                                "synthetic.num_test=1"], wait=True, timeout=600)
    assert st["phase"] == "Succeeded", rel.logs("coco")
    data = home / "home" / "pv" / "pv-fsx" / "data" / "coco2017"
    assert (data / "annotations" / "instances_train2017.json").exists()
    assert (data / "pretrained-models" / "ImageNet-R50-AlignPadding.npz").exists()
    doc = _y.safe_load(open(os.path.join(EX, "maskrcnn", "train-maskrcnn-tensorpack.yaml")))
    doc["resources"] = {"gpu_nodes": 1, "gpus_per_node": 2, "gpu_instance_type": "mi355x.8x"}
    doc["train"]["args"] = [a.replace("TRAIN.STEPS_PER_EPOCH=15000", "TRAIN.STEPS_PER_EPOCH=2")
                            for a in doc["train"]["args"]] + SMALL_MRCNN
    p = home / "mr.yaml"
    p.write_text(_y.safe_dump(doc))
    st = rel.install(os.path.join(CHARTS, "training", "mpijob-horovod-tensorflow-gpu"), "maskrcnn-tensorpack",
                     value_files=[str(p)], wait=True, timeout=900)
    log = rel.logs("maskrcnn-tensorpack")
    assert st["phase"] == "Succeeded", log[-4000:]
    assert "[1,0]<stdout>:" in log and "Epoch 1 (global_step 2) finished" in log
    assert "Loaded 265 backbone tensors" in log
    logs = home / "home" / "pv" / "pv-efs" / "home" / "maskrcnn-tensorpack" / "logs"
    run = [d for d in os.listdir(logs) if d.startswith("maskrcnn-tensorpack-")]
    # every rank runs the script's `DATE=$(date ...)` (as in the reference), so ranks that start
    # on either side of a second boundary log to two directories; rank 0's holds the checkpoint
    assert run and any(f.endswith(".index") for r in run for f in os.listdir(logs / r))


def test_legacy_maskrcnn_chart_renders_inline_mpirun(home):
    from mxtrain.chart.render import load_chart, render_chart
    r = render_chart(load_chart(os.path.join(CHARTS, "training", "maskrcnn")), "mr")
    job = r.by_kind("MPIJob")[0]
    args = job["spec"]["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]["args"]
    assert args[args.index("-np") + 1] == "8" and "$(MXTRAIN_WORKLOADS)/maskrcnn/train.py" in args
    assert "TRAINER=horovod" in args and "TRAIN.CHECKPOINT_PERIOD=2" in args
    r2 = render_chart(load_chart(os.path.join(CHARTS, "training", "maskrcnn-optimized")), "mr")
    a2 = r2.by_kind("MPIJob")[0]["spec"]["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]["args"]
    assert "--images_per_epoch" in a2 and "TRAIN.BATCH_SIZE_PER_GPU=4" in a2 and "PREPROC.PREDEFINED_PADDING=True" in a2


def test_redpajama_data_chart_offline(home):
    """redpajama-data chart: idempotent download step writes DATA_DIR/data.jsonl (synthetic
    RedPajama-style documents on the offline node) on the claim."""
    import json as _j
    from mxtrain.launch import release as rel
    st = rel.install(os.path.join(CHARTS, "data-prep", "redpajama-data"), "rp", sets=["synthetic.num_docs=50"],
                     wait=True, timeout=300)
    assert st["phase"] == "Succeeded", rel.logs("rp")
    f = home / "home" / "pv" / "pv-fsx" / "data" / "redpajama" / "data.jsonl"
    lines = f.read_text().splitlines()
    assert len(lines) == 50 and "text" in _j.loads(lines[0])
    st = rel.install(os.path.join(CHARTS, "data-prep", "redpajama-data"), "rp2", sets=["synthetic.num_docs=50"],
                     wait=True, timeout=300)
    assert "already exists" in rel.logs("rp2")
