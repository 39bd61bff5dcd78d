"""Megatron-compatible workload plumbing on CPU: mmap indexed dataset format, native
sample-index builder, preprocess_data, pretrain_gpt CLI (DeepSpeed JSON subset),
DeepSpeed-layout checkpoints and exact resume."""
import json
import os
import struct
import subprocess
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MEG = os.path.join(REPO, "mxtrain", "workloads", "megatron")


def test_indexed_dataset_roundtrip(tmp_path):
    from mxtrain.data.indexed import IndexedDatasetBuilder, MMapIndexedDataset
    prefix = str(tmp_path / "d")
    b = IndexedDatasetBuilder(prefix + ".bin", np.uint16)
    docs = [[1, 2, 3], [4], [5, 6, 7, 8, 9]]
    for d in docs:
        b.add_item(d)
        b.end_document()
    b.finalize(prefix + ".idx")
    raw = open(prefix + ".idx", "rb").read()
    assert raw[:9] == b"MMIDIDX\x00\x00"
    assert struct.unpack("<Q", raw[9:17])[0] == 1 and raw[17] == 8       # version 1, uint16
    assert struct.unpack("<QQ", raw[18:34]) == (3, 4)
    ds = MMapIndexedDataset(prefix)
    assert [list(ds[i]) for i in range(3)] == docs
    assert list(ds.doc_idx) == [0, 1, 2, 3]
    assert list(ds.get(2, 1, 3)) == [6, 7, 8]
    assert os.path.getsize(prefix + ".bin") == 9 * 2


def _sample_idx_py(sizes, doc_idx, seq, n):
    out = np.zeros((n + 1, 2), np.int64)
    di, off = 0, 0
    for s in range(1, n + 1):
        rem = seq + 1
        while rem:
            dl = sizes[doc_idx[di]] - off
            rem -= dl
            if rem <= 0:
                off += rem + dl - 1
                rem = 0
            else:
                di += 1
                off = 0
        out[s] = (di, off)
    return out


def test_native_sample_idx_matches_python():
    from mxtrain.runtime import native
    rng = np.random.RandomState(0)
    sizes = rng.randint(1, 50, size=200).astype(np.int32)
    doc_idx = np.concatenate([rng.permutation(200) for _ in range(3)]).astype(np.int32)
    seq = 16
    n = native.sample_count(3, int(sizes.sum()), seq)
    got = native.build_sample_idx(sizes, doc_idx, seq, n)
    np.testing.assert_array_equal(got, _sample_idx_py(sizes, doc_idx, seq, n))
    di, dsi = native.build_blending_indices([0.25, 0.75], 100)
    assert abs(int((di == 1).sum()) - 75) <= 1


def test_gpt_dataset_samples_are_contiguous_stream(tmp_path):
    from mxtrain.data.gpt_dataset import GPTDataset
    from mxtrain.data.indexed import IndexedDatasetBuilder, MMapIndexedDataset
    prefix = str(tmp_path / "d")
    b = IndexedDatasetBuilder(prefix + ".bin", np.int32)
    tok = 0
    for n in [7, 3, 11, 5, 9, 2, 13]:
        b.add_item(list(range(tok, tok + n)))
        b.end_document()
        tok += n
    b.finalize(prefix + ".idx")
    ds = GPTDataset("train", MMapIndexedDataset(prefix), np.arange(7), 10, 8, seed=3,
                    cache_dir=str(tmp_path / "cache"))
    for i in range(len(ds)):
        x = ds.tokens(i)
        assert x.shape == (9,)
    # cached index files are reused
    ds2 = GPTDataset("train", MMapIndexedDataset(prefix), np.arange(7), 10, 8, seed=3,
                     cache_dir=str(tmp_path / "cache"))
    np.testing.assert_array_equal(ds.tokens(3), ds2.tokens(3))


def test_preprocess_data_cli(tmp_path):
    from mxtrain.data.indexed import MMapIndexedDataset
    from mxtrain.data.text_synth import write_corpus
    from mxtrain.data.tokenizer import GPT2BPETokenizer
    env = dict(os.environ, PYTHONPATH=REPO, DATA_ROOT=str(tmp_path))
    write_corpus(str(tmp_path / "train.json"), 200, seed=1)
    subprocess.run(["bash", os.path.join(MEG, "dataset", "download_vocab.sh")], cwd=tmp_path, env=env, check=True,
                   capture_output=True)
    vocab = json.load(open(tmp_path / "gpt2-vocab.json"))
    assert len(vocab) == 50257 and vocab["<|endoftext|>"] == 50256
    r = subprocess.run([sys.executable, os.path.join(MEG, "tools", "preprocess_data.py"), "--input",
                        str(tmp_path / "train.json"), "--output-prefix", str(tmp_path / "gpt2"), "--vocab-file",
                        "gpt2-vocab.json", "--dataset-impl", "mmap", "--tokenizer-type", "GPT2BPETokenizer",
                        "--merge-file", "gpt2-merges.txt", "--append-eod", "--workers", "3"],
                       cwd=tmp_path, env=env, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    ds = MMapIndexedDataset(str(tmp_path / "gpt2_text_document"))
    assert len(ds) == 200 and ds.dtype == np.uint16
    tok = GPT2BPETokenizer(str(tmp_path / "gpt2-vocab.json"), str(tmp_path / "gpt2-merges.txt"))
    first = json.loads(open(tmp_path / "train.json").readline())["text"]
    ids = list(ds[0])
    assert ids[-1] == 50256 and ids[:-1] == tok.tokenize(first)
    assert tok.detokenize(ids[:-1]) == first


def _run_pretrain(argv):
    from mxtrain.workloads.megatron import pretrain_gpt
    return pretrain_gpt.main(argv)


TINY = ["--num-layers", "2", "--hidden-size", "64", "--num-attention-heads", "2", "--seq-length", "32",
        "--max-position-embeddings", "32", "--micro-batch-size", "2", "--lr", "1e-3", "--lr-decay-style", "cosine",
        "--min-lr", "1e-5", "--weight-decay", "1e-2", "--lr-warmup-fraction", ".1", "--clip-grad", "1.0", "--fp16",
        "--mock-data", "--vocab-size", "500", "--log-interval", "2", "--eval-iters", "0",
        "--distributed-backend", "nccl"]


def test_pretrain_resume_is_exact(tmp_path, monkeypatch):
    monkeypatch.setenv("MXTRAIN_CPU_ONLY", "1")
    ds = tmp_path / "ds.json"
    ds.write_text(json.dumps({"fp16": {"enabled": True}, "zero_optimization": {"stage": 1},
                              "train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2}))
    base = TINY + ["--deepspeed", "--deepspeed_config", str(ds), "--lr-decay-iters", "8",
                   "--mx-metrics-dir", str(tmp_path / "logs")]
    assert _run_pretrain(base + ["--train-iters", "8", "--save", str(tmp_path / "a")]) == 0
    assert _run_pretrain(base + ["--train-iters", "4", "--save", str(tmp_path / "b")]) == 0
    assert _run_pretrain(base + ["--train-iters", "8", "--save", str(tmp_path / "b"), "--load",
                                 str(tmp_path / "b")]) == 0
    assert open(tmp_path / "a" / "latest").read() == "global_step8"
    assert open(tmp_path / "b" / "latest_checkpointed_iteration.txt").read() == "8"
    a = torch.load(tmp_path / "a" / "global_step8" / "mp_rank_00_model_states.pt", weights_only=True)
    b = torch.load(tmp_path / "b" / "global_step8" / "mp_rank_00_model_states.pt", weights_only=True)
    assert a["iteration"] == 8 and a["global_samples"] == 8 * 4
    assert "language_model.encoder.layers.1.self_attention.query_key_value.weight" in a["module"]
    for k in a["module"]:
        torch.testing.assert_close(a["module"][k], b["module"][k], rtol=0, atol=0, msg=k)
    oa = torch.load(tmp_path / "a" / "global_step8" / "zero_pp_rank_0_mp_rank_00_optim_states.pt",
                    weights_only=True)["optimizer_state_dict"]
    assert oa["zero_stage"] == 1 and oa["base_optimizer_state"]["state"][0]["step"] == 8
    lines = [json.loads(x) for x in open(tmp_path / "logs" / "metrics-rank0.jsonl")]
    assert [r["step"] for r in lines if "loss" in r][:4] == [2, 4, 6, 8]
    # the --fp16 -> bf16 rewrite and the effective dropout settings are recorded, not silent
    cfg_ev = [r for r in lines if r.get("event") == "config"]
    assert cfg_ev and cfg_ev[0]["effective"]["attention_dropout"] == 0.1
    assert any("--fp16 -> bf16" in d for d in cfg_ev[0]["deviations"])
    assert a["args"]["mx_effective"]["compute_dtype"] == "bf16"
    assert any("--fp16 -> bf16" in d for d in a["args"]["mx_deviations"])


def test_async_save_resume_is_exact(tmp_path, monkeypatch):
    """--async-save: snapshots + background writes every --save-interval; `latest` only
    ever names a finished checkpoint; resuming from the async checkpoint reproduces the
    synchronous run bit for bit."""
    monkeypatch.setenv("MXTRAIN_CPU_ONLY", "1")
    ds = tmp_path / "ds.json"
    ds.write_text(json.dumps({"zero_optimization": {"stage": 1}, "train_micro_batch_size_per_gpu": 2,
                              "gradient_accumulation_steps": 2}))
    base = TINY + ["--deepspeed", "--deepspeed_config", str(ds), "--lr-decay-iters", "8",
                   "--mx-metrics-dir", str(tmp_path / "logs")]
    assert _run_pretrain(base + ["--train-iters", "8", "--save", str(tmp_path / "s")]) == 0
    assert _run_pretrain(base + ["--train-iters", "4", "--save-interval", "2", "--async-save",
                                 "--save", str(tmp_path / "a")]) == 0
    assert open(tmp_path / "a" / "latest").read() == "global_step4"
    assert sorted(os.listdir(tmp_path / "a" / "global_step2")) == sorted(os.listdir(tmp_path / "a" / "global_step4"))
    assert not [f for f in os.listdir(tmp_path / "a" / "global_step4") if ".tmp" in f]
    assert _run_pretrain(base + ["--train-iters", "8", "--async-save", "--save", str(tmp_path / "a"),
                                 "--load", str(tmp_path / "a")]) == 0
    assert open(tmp_path / "a" / "latest_checkpointed_iteration.txt").read() == "8"
    for name in ("mp_rank_00_model_states.pt", "zero_pp_rank_0_mp_rank_00_optim_states.pt"):
        s = torch.load(tmp_path / "s" / "global_step8" / name, weights_only=True)
        a = torch.load(tmp_path / "a" / "global_step8" / name, weights_only=True)
        if "module" in s:
            for k in s["module"]:
                torch.testing.assert_close(s["module"][k], a["module"][k], rtol=0, atol=0, msg=k)
        else:
            so, ao = s["optimizer_state_dict"], a["optimizer_state_dict"]
            torch.testing.assert_close(so["single_partition_of_fp32_groups"][0],
                                       ao["single_partition_of_fp32_groups"][0], rtol=0, atol=0)
            torch.testing.assert_close(so["base_optimizer_state"]["state"][0]["exp_avg_sq"],
                                       ao["base_optimizer_state"]["state"][0]["exp_avg_sq"], rtol=0, atol=0)


def test_async_checkpointer_snapshot_is_isolated(tmp_path):
    """The snapshot holds the values at save() time even when training mutates the
    parameters before the background write runs; a write error surfaces in wait()."""
    from mxtrain.checkpoint import AsyncCheckpointer
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.parallel.state import ParallelState
    from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch
    cfg = GPTConfig(num_layers=2, hidden_size=32, num_attention_heads=4, seq_length=16,
                    max_position_embeddings=16, vocab_size=64)
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=2), ParallelState())
    tok, lab = synthetic_batch(cfg, 1, 2, "cpu", torch.Generator().manual_seed(0))
    tr.train_step(tok, lab)
    ck = AsyncCheckpointer(tr)
    tr.ckpt_fence = ck.fence
    before = {k: v.clone() for k, v in tr.flat.params.items()}
    master = tr.opt.master.clone()
    ck.save(str(tmp_path), 1)
    tr.train_step(tok, lab)   # mutates params / master while the writer may still be running
    ck.wait()
    assert open(tmp_path / "latest").read() == "global_step1"
    m = torch.load(tmp_path / "global_step1" / "mp_rank_00_model_states.pt", weights_only=True)["module"]
    torch.testing.assert_close(m["language_model.embedding.word_embeddings.weight"], before["wte"], rtol=0, atol=0)
    o = torch.load(tmp_path / "global_step1" / "zero_pp_rank_0_mp_rank_00_optim_states.pt", weights_only=True)
    torch.testing.assert_close(o["optimizer_state_dict"]["single_partition_of_fp32_groups"][0], master,
                               rtol=0, atol=0)
    assert not torch.equal(tr.flat.params["wte"], before["wte"])
    # a failing write (target is a file, not a directory) is raised on the training thread
    bad = tmp_path / "notadir"
    bad.write_text("x")
    with pytest.raises(Exception):
        ck.save(str(bad), 2)
        ck.wait()


def test_qkv_megatron_interleave_roundtrip():
    from mxtrain.checkpoint import qkv_from_megatron, qkv_to_megatron
    for hl, kvl in ((4, 4), (4, 2), (8, 1)):
        D = 3
        t = torch.randn((hl + 2 * kvl) * D, 5)
        m = qkv_to_megatron(t, hl, kvl, D)
        torch.testing.assert_close(qkv_from_megatron(m, hl, kvl, D), t)
    # MHA: Megatron rows are [q0 k0 v0 q1 k1 v1 ...]
    D, H = 2, 2
    t = torch.arange(3 * H * D).float()
    m = qkv_to_megatron(t, H, H, D)
    assert m.tolist() == [0, 1, 4, 5, 8, 9, 2, 3, 6, 7, 10, 11]


def test_ds_config_and_megatron_flags(tmp_path):
    from mxtrain.workloads.megatron.arguments import parse_args
    ds = tmp_path / "ds.json"
    ds.write_text(json.dumps({"fp16": {"enabled": True}, "zero_optimization": {"stage": 1},
                              "train_micro_batch_size_per_gpu": 8, "gradient_accumulation_steps": 1}))
    a = parse_args(["--deepspeed", "--deepspeed_config", str(ds), "--num-layers", "24", "--train-iters", "500000",
                    "--lr-decay-iters", "320000", "--lr-warmup-fraction", ".01", "--no-masked-softmax-fusion",
                    "--tensor-model-parallel-size", "1"])
    assert a.micro_batch_size == 8 and a.zero_stage == 1 and a.fp16
    assert a.lr_warmup_iters == 3200 and a.global_batch_size == 8
    assert any("--no-masked-softmax-fusion" in d for d in a.mx_deviations)
    assert a.mx_effective["attention_dropout"] == 0.1 and not a.mx_recompute
    b = parse_args(["--checkpoint-activations", "--zero-stage", "2"])
    assert b.mx_recompute and b.mx_effective["activation_recompute"] == "full"
    assert any("ZeRO stage 2 -> stage 1" in d for d in b.mx_deviations)


def test_gpu_sampler_fake_sysfs(tmp_path):
    """§5.5: power / clock / temperature sampling from the amdgpu hwmon nodes."""
    import time
    from mxtrain.obs.metrics import GPUSampler, gpu_sample
    hw = tmp_path / "class/drm/card3/device/hwmon/hwmon0"
    hw.mkdir(parents=True)
    (hw / "power1_average").write_text("750000000\n")      # uW
    (hw / "freq1_input").write_text("2400000000\n")        # Hz
    (hw / "temp2_input").write_text("65000\n")             # mC
    s = gpu_sample(3, str(tmp_path))
    assert s == {"power_w": 750.0, "sclk_mhz": 2400.0, "temp_junction_c": 65.0}
    smp = GPUSampler(3, interval_s=0.02, root=str(tmp_path))
    time.sleep(0.2)
    (hw / "power1_average").write_text("950000000\n")
    time.sleep(0.2)
    out = smp.take()
    smp.close()
    assert out["gpu_samples"] >= 3 and out["gpu_power_w_max"] == 950.0
    assert 750.0 <= out["gpu_power_w_mean"] <= 950.0 and out["gpu_sclk_mhz_mean"] == 2400.0
    assert GPUSampler(None).take() == {}


def _async_fail_worker(rank, world, port, root, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mxtrain.checkpoint import AsyncCheckpointer

        class _T:   # the writer path only needs .device / .trainer
            device = torch.device("cpu")

        ck = AsyncCheckpointer(_T())
        good = os.path.join(root, f"r{rank}.pt")
        bad = os.path.join(root, "notadir", f"r{rank}.pt")   # parent is a file: open() fails
        path = bad if rank == 1 else good
        ck._commit_args = (root, 3, rank == 0)
        ck._err = None
        import threading
        ck._thread = threading.Thread(target=ck._write, args=([(path, {"x": torch.ones(2)})], None))
        ck._thread.start()
        try:
            ck.wait()
            q.put((rank, "no-error"))
        except RuntimeError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_async_write_failure_raises_on_every_rank(tmp_path):
    """one rank's failed background write must fail the save on EVERY rank
    (an all-reduced error flag before the commit barrier), not leave the others blocked in
    _commit; `latest` is not advanced."""
    import socket
    import torch.multiprocessing as mp
    (tmp_path / "notadir").write_text("x")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_async_fail_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict(q.get(timeout=5) for _ in range(2))
    assert "failed" in res[0] and "another rank" in res[0]
    assert "failed" in res[1] and "another rank" not in res[1]
    assert not (tmp_path / "latest").exists()
