"""Asynchronous checkpointing on the GPU path (mxtrain/checkpoint.py AsyncCheckpointer:
pinned host buffers filled on a side stream, event-fenced before the optimizer mutates the
state, background file writes).  The CPU tests (tests/test_megatron_cpu.py) run the
synchronous-clone fallback; this one runs the device snapshot."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _files(d):
    out = {}
    for name in sorted(os.listdir(d)):
        out[name] = torch.load(os.path.join(d, name), weights_only=True)
    return out


def _same(a, b, path=""):
    if isinstance(a, torch.Tensor):
        assert isinstance(b, torch.Tensor) and a.dtype == b.dtype and torch.equal(a.cpu(), b.cpu()), path
    elif isinstance(a, dict):
        assert set(a) == set(b), path
        for k in a:
            _same(a[k], b[k], f"{path}/{k}")
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            _same(x, y, f"{path}[{i}]")
    else:
        assert a == b, path


def test_async_save_then_step_matches_sync_save(tmp_path):
    """Async save at iteration 1, one more (dropout) step while the snapshot/writes may be in
    flight, then wait: the files equal a synchronous save of iteration 1 taken before the
    step -- parameters, fp32 master, Adam moments and the dropout seed included."""
    from mxtrain.checkpoint import AsyncCheckpointer, save_checkpoint
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.parallel.state import ParallelState
    from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch
    dev = torch.device("cuda", 0)
    cfg = GPTConfig(num_layers=2, hidden_size=128, num_attention_heads=2, seq_length=128,
                    max_position_embeddings=128, vocab_size=512, hidden_dropout=0.1, attention_dropout=0.1)
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=2), ParallelState(device=dev))
    tok, lab = synthetic_batch(cfg, 1, 2, dev, torch.Generator().manual_seed(0))
    tr.train_step(tok, lab)
    torch.cuda.synchronize()
    save_checkpoint(str(tmp_path / "sync"), tr, 1)
    ck = AsyncCheckpointer(tr)
    tr.ckpt_fence = ck.fence
    ck.save(str(tmp_path / "async"), 1)
    tr.train_step(tok, lab)
    ck.wait()
    torch.cuda.synchronize()
    s = _files(tmp_path / "sync" / "global_step1")
    a = _files(tmp_path / "async" / "global_step1")
    assert set(s) == set(a) and s
    for name in s:
        _same(s[name], a[name], name)
