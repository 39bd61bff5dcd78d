"""Per-rank HBM sizing (runtime/memory_plan.py): the activation model is checked against
the tensors a real GPT layer keeps for backward, and GPT-3 6.7B at TP=2 x PP=2 x DP=2
(BASELINE.json config 4) must fit one 288 GB MI355X."""
import torch

from mxtrain.models.gpt import GPT_CONFIGS, GPTConfig, GPTLayerFn
from mxtrain.runtime import memory_plan as mp


def _saved_bytes(obj, seen):
    if isinstance(obj, torch.Tensor):
        key = (obj.untyped_storage().data_ptr(), obj.storage_offset(), tuple(obj.shape))
        if key in seen or obj.numel() == 0:
            return 0
        seen.add(key)
        return obj.numel() * obj.element_size()
    if isinstance(obj, (tuple, list)):
        return sum(_saved_bytes(o, seen) for o in obj)
    return 0


def _measure(cfg_kw, B, monkeypatch, dtype=torch.bfloat16):
    from mxtrain.parallel.state import ParallelState
    from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch
    cfg = GPTConfig(**cfg_kw)
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=B), ParallelState(), dtype=dtype)
    per_layer = []
    orig = GPTLayerFn._forward_body

    def spy(rt, i, next_norm, h, a, recomputing=False, micro=0):
        out = orig(rt, i, next_norm, h, a, recomputing=recomputing, micro=micro)
        per_layer.append(_saved_bytes(out[2], set()))
        return out

    monkeypatch.setattr(GPTLayerFn, "_forward_body", staticmethod(spy))
    tok, lab = synthetic_batch(cfg, 1, B, "cpu", torch.Generator().manual_seed(0))
    tr.train_step(tok, lab)
    return cfg, per_layer


def test_layer_activation_model_matches_saved_tensors(monkeypatch):
    kw = dict(num_layers=2, hidden_size=64, num_attention_heads=4, seq_length=32, max_position_embeddings=32,
              vocab_size=256, hidden_dropout=0.0, attention_dropout=0.0)
    cfg, per_layer = _measure(kw, 2, monkeypatch)
    assert len(per_layer) == 2
    model = mp.layer_saved_bytes(cfg, 2 * 32, tp=1)
    # the model may over-count the LN statistics of the last layer's throwaway norm
    for got in per_layer:
        assert abs(got - model) <= 0.02 * model, (got, model)


def test_llama_style_layer_activation_model(monkeypatch):
    kw = dict(num_layers=2, hidden_size=64, num_attention_heads=4, num_kv_heads=2, seq_length=32,
              max_position_embeddings=32, vocab_size=256, normalization="rmsnorm", position_embedding="rope",
              swiglu=True, ffn_hidden_size=96, hidden_dropout=0.0, attention_dropout=0.0)
    cfg, per_layer = _measure(kw, 2, monkeypatch)
    model = mp.layer_saved_bytes(cfg, 2 * 32, tp=1)
    for got in per_layer:
        assert abs(got - model) <= 0.05 * model, (got, model)


def test_param_count_matches_config_formula():
    cfg = GPTConfig(**GPT_CONFIGS["gpt3-6.7b"])
    total = sum(mp.stage_numel(cfg, 1, 1, 0) for _ in range(1))
    assert total == cfg.num_params()
    # TP=2 x PP=2 shards partition the matrices (replicated LN / bias vectors excepted); the
    # last stage holds the tied output embedding's copy (Megatron word_embeddings_for_head)
    parts = sum(mp.stage_numel(cfg, 2, 2, r) for r in range(2)) * 2
    tied = cfg.padded_vocab(2) * cfg.hidden_size
    assert cfg.num_params() + tied <= parts <= (cfg.num_params() + tied) * 1.002


def test_gpt3_6p7b_tp2_pp2_dp2_fits_288gb():
    cfg = GPTConfig(**GPT_CONFIGS["gpt3-6.7b"], hidden_dropout=0.1, attention_dropout=0.1)
    # the reference's 6.7B layout: TP 2 x PP 2 x DP 2, micro-batch 2, seq 2048, sequence parallel
    plan = mp.rank_memory(cfg, tp=2, pp=2, dp=2, micro_batch=2, num_micro=8, sequence_parallel=True)
    s = plan.summary()
    assert plan.fits(), s
    # ~1.68 B parameters per rank: 3.4 GB bf16 params, 3.4 GB grads, ~10 GB ZeRO-1 fp32 state
    assert 3.0 < s["params_GB"] < 3.8 and 9.0 < s["optimizer_GB"] < 11.5, s
    assert s["total_GB"] < 60, s
    # the whole model on ONE GPU (DP only, what bench.py --model gpt3-6.7b runs) also fits
    one = mp.rank_memory(cfg, tp=1, pp=1, dp=1, micro_batch=2)
    assert one.fits(), one.summary()
    assert 90 < one.summary()["total_GB"] < 288, one.summary()
    # and 288 GB is what makes DP-only 6.7B possible: an 80 GB part would not hold it
    assert not one.fits(hbm=80 * 10 ** 9)
