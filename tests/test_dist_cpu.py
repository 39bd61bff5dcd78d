"""Distributed parity on CPU (gloo, 2 processes): DP+ZeRO-1, TP (+SP) and PP runs of the
same GPT must reproduce the single-process loss and parameter updates (fp32, dropout 0).

This is the CPU stand-in for the 8-GPU RCCL runs: every collective the GPU path issues
(reduce-scatter, all-gather, all-reduce, batched p2p) goes through the same code with the
gloo backend."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.dist

CFG = dict(num_layers=2, hidden_size=64, num_attention_heads=4, seq_length=16,
           max_position_embeddings=16, vocab_size=256, hidden_dropout=0.0, attention_dropout=0.0)


# LLaMA-style variant: RoPE + GQA + RMSNorm + SwiGLU (column-parallel [a|b] fc1 split)
CFG_LLAMA = dict(CFG, num_kv_heads=2, normalization="rmsnorm", position_embedding="rope",
                 swiglu=True, ffn_hidden_size=96)


# attention dropout on: the keep-mask is keyed on the GLOBAL head index, so TP / CP head
# shards must still reproduce the single-process run exactly
CFG_ADROP = dict(CFG, attention_dropout=0.1)


# hidden + attention dropout 0.1 (the reference config's Megatron defaults): the masks are
# keyed on the global micro-batch index and global element / head indices, so every
# parallel layout draws the single-process masks
CFG_DROP = dict(CFG, hidden_dropout=0.1, attention_dropout=0.1)


def _cfg(mode):
    if mode.endswith(":drop"):
        return CFG_DROP
    if mode.endswith(":llama"):
        return CFG_LLAMA
    if mode.endswith(":adrop"):
        return CFG_ADROP
    return CFG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    g = torch.Generator().manual_seed(7)
    x = torch.randint(0, CFG["vocab_size"], (2, 2, CFG["seq_length"] + 1), generator=g)
    return x[..., :-1].contiguous(), x[..., 1:].contiguous()


def _reference(steps=2):
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.parallel.state import ParallelState
    from mxtrain.training import GPTTrainer, TrainConfig
    cfg = GPTConfig(**CFG)
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=2, global_batch_size=4, lr=1e-3,
                                     overlap_grad_reduce=False), ParallelState(),
                    dtype=torch.float32)
    tok, lab = _data()
    losses = [float(tr.train_step(tok, lab)) for _ in range(steps)]
    return losses, {n: p.clone() for n, p in tr.flat.params.items()}, tr.flat.state_dict()


def _worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.manual_seed(0)
    ccfg = _cfg(mode)
    full_mode = mode
    if mode.endswith(":sync"):
        os.environ["MXTRAIN_TP_OVERLAP"] = "0"   # collectives complete before the next GEMM
    mode = mode.split(":")[0]
    from mxtrain.models.gpt import GPTConfig, shard_gpt_state
    from mxtrain.parallel import state as pstate
    from mxtrain.training import GPTTrainer, TrainConfig
    tp = 2 if mode in ("tp", "sp", "3d", "3dsp", "tpcp") else 1
    pp = 2 if mode in ("pp", "3d", "3dsp") else 1
    cp = 2 if mode in ("cp", "tpcp") else 1
    ps = pstate.initialize_model_parallel(tp=tp, pp=pp, sequence_parallel=mode in ("sp", "3dsp"),
                                          backend="gloo", device_type="cpu", cp=cp)
    cfg = GPTConfig(**ccfg)
    # reference init (identical on every rank), then take this rank's shard
    _, _, init_sd = _ref_init(ccfg)
    mb1 = ":mb1" in full_mode   # 4 micro-batches of 1 sequence: deeper 1F1B steady state
    tcfg = TrainConfig(micro_batch_size=1 if mb1 else 2, global_batch_size=4, lr=1e-3, overlap_grad_reduce=False)
    tr = GPTTrainer(cfg, tcfg, ps, dtype=torch.float32)
    if ps.dp > 1:
        # exercise the deferred (next-step, per-bucket) ZeRO-1 parameter all-gather path
        tr.opt.overlap_param_gather = True
    local = shard_gpt_state(init_sd, cfg, ps.tp, ps.tp_rank, ps.pp, ps.pp_rank)
    tr.flat.load_state_dict(local)
    tr.opt._refresh_master()
    tok, lab = _data()
    if ps.dp > 1:
        tok, lab = tok[ps.dp_rank:ps.dp_rank + 1], lab[ps.dp_rank:ps.dp_rank + 1]
    if mb1:
        tok, lab = tok.reshape(-1, 1, tok.shape[-1]), lab.reshape(-1, 1, lab.shape[-1])
    losses = [float(tr.train_step(tok, lab)) for _ in range(2)]
    tr.sync_params()
    # numpy copies: tensors sent through a spawn queue are fd-shared and vanish with the
    # worker process
    q.put((rank, mode, losses, {n: p.detach().clone().numpy() for n, p in tr.flat.params.items()},
           (ps.tp_rank, ps.pp_rank, ps.dp_rank)))
    pstate.destroy()


_REF = {}


def _ref_init(ccfg=CFG):
    key = "init_llama" if ccfg is CFG_LLAMA else "init"
    if key not in _REF:
        from mxtrain.models.gpt import GPTConfig
        from mxtrain.parallel.state import ParallelState
        from mxtrain.training import GPTTrainer, TrainConfig
        cfg = GPTConfig(**ccfg)
        tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=2, global_batch_size=4),
                        ParallelState(), dtype=torch.float32)
        _REF[key] = (None, None, tr.flat.state_dict())
    return _REF[key]


def _run(mode, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = [(r, m, l, {n: torch.from_numpy(a) for n, a in p.items()}, ids) for r, m, l, p, ids in res]
    return sorted(res, key=lambda t: t[0])


def _make_reference(ccfg):
    # the reference trainer must start from the same init the workers shard
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.parallel.state import ParallelState
    from mxtrain.training import GPTTrainer, TrainConfig
    cfg = GPTConfig(**ccfg)
    _, _, init_sd = _ref_init(ccfg)
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=2, global_batch_size=4, lr=1e-3,
                                     overlap_grad_reduce=False), ParallelState(),
                    dtype=torch.float32)
    tr.flat.load_state_dict(init_sd)
    tr.opt._refresh_master()
    tok, lab = _data()
    losses = [float(tr.train_step(tok, lab)) for _ in range(2)]
    return cfg, losses, tr.flat.state_dict()


@pytest.fixture(scope="module")
def reference():
    return _make_reference(CFG)


def _check(mode, reference, loss_ranks):
    from mxtrain.models.gpt import shard_gpt_state
    cfg, ref_losses, ref_sd = reference
    res = _run(mode)
    for rank, _, losses, params, (tpr, ppr, dpr) in res:
        if rank in loss_ranks:
            for a, b in zip(losses, ref_losses):
                assert abs(a - b) < 2e-5 * max(1.0, abs(b)), (mode, rank, losses, ref_losses)
        m = mode.split(":")[0]
        exp = shard_gpt_state(ref_sd, cfg, 2 if m in ("tp", "sp", "tpcp") else 1, tpr,
                              2 if m == "pp" else 1, ppr)
        for n, t in exp.items():
            assert torch.allclose(params[n], t, atol=3e-5, rtol=1e-4), (mode, rank, n,
                                                                        (params[n] - t).abs().max())


def test_dp_zero1_matches_single(reference):
    # DP ranks report their own micro-batch loss; the parameters must match exactly
    from mxtrain.models.gpt import shard_gpt_state
    cfg, ref_losses, ref_sd = reference
    res = _run("dp")
    mean_first = sum(r[2][0] for r in res) / 2
    assert abs(mean_first - ref_losses[0]) < 2e-5 * max(1.0, abs(ref_losses[0]))
    for rank, _, losses, params, _ in res:
        for n, t in ref_sd.items():
            assert torch.allclose(params[n], t, atol=3e-5, rtol=1e-4), (rank, n)


def test_tp2_matches_single(reference):
    _check("tp", reference, loss_ranks=(0, 1))


def test_tp2_sequence_parallel_matches_single(reference):
    _check("sp", reference, loss_ranks=(0, 1))


def test_tp2_sp_llama_style_matches_single():
    """RoPE + GQA + RMSNorm + SwiGLU under TP2 + sequence parallel."""
    _check("sp:llama", _make_reference(CFG_LLAMA), loss_ranks=(0, 1))


def test_ulysses_cp2_matches_single(reference):
    """Ulysses context parallelism (P8): each rank holds half of every sequence; the
    attention runs on half the heads over whole sequences after an all-to-all."""
    _check("cp", reference, loss_ranks=(0, 1))


def test_ulysses_cp2_rope_gqa_matches_single():
    _check("cp:llama", _make_reference(CFG_LLAMA), loss_ranks=(0, 1))


def test_tp2_x_ulysses_cp2_matches_single(reference):
    """4 ranks: TP2 (heads split) x CP2 (sequence split, head groups within each TP shard)."""
    cfg, ref_losses, ref_sd = reference
    from mxtrain.models.gpt import shard_gpt_state
    res = _run("tpcp", world=4)
    for rank, _, losses, params, (tpr, ppr, dpr) in res:
        for a, b in zip(losses, ref_losses):
            assert abs(a - b) < 2e-5 * max(1.0, abs(b)), (rank, losses, ref_losses)
        exp = shard_gpt_state(ref_sd, cfg, 2, tpr, 1, 0)
        for n, t in exp.items():
            assert torch.allclose(params[n], t, atol=3e-5, rtol=1e-4), (rank, n, (params[n] - t).abs().max())


@pytest.mark.parametrize("mode", ["tp:adrop", "cp:adrop"])
def test_attention_dropout_sharded_matches_single(mode):
    """Attention dropout 0.1 under TP2 (heads split) and Ulysses CP2 (head groups after the
    all-to-all): the shards draw the single-process keep-mask, so losses and updates match."""
    _check(mode, _make_reference(CFG_ADROP), loss_ranks=(0, 1))


@pytest.mark.parametrize("mode", ["tp", "sp"])
def test_tp_comm_overlap_bit_identical(mode):
    """TP communication overlap (async dgrad all-reduce / reduce-scatter across the
    weight-gradient GEMMs; under SP the all-gather overlapping the own-chunk GEMM) gives
    bit-identical losses and parameters to the synchronous path."""
    a, b = _run(mode), _run(mode + ":sync")
    for (ra, _, la, pa, _), (rb, _, lb, pb, _) in zip(a, b):
        assert ra == rb and la == lb, (mode, la, lb)
        for n in pa:
            assert torch.equal(pa[n], pb[n]), (mode, ra, n, (pa[n] - pb[n]).abs().max())


def test_pp2_1f1b_matches_single(reference):
    _check("pp", reference, loss_ranks=(1,))


def test_pp2_1f1b_four_microbatches_matches_single(reference):
    """Non-blocking p2p with prefetched receives over a longer 1F1B steady state."""
    _check("pp:mb1", reference, loss_ranks=(1,))


@pytest.mark.parametrize("mode", ["3d", "3dsp"])
def test_tp2_pp2_dp2_matches_single(reference, mode):
    """BASELINE config 4 topology (TP=2 x PP=2 x DP=2 = 8 ranks, + SP variant) on a tiny
    GPT: every rank's parameter shard after two ZeRO-1 steps equals the single-process
    result, and the DP-mean of the last stage's losses equals the reference loss."""
    from mxtrain.models.gpt import shard_gpt_state
    cfg, ref_losses, ref_sd = reference
    res = _run(mode, world=8)
    last = [r for r in res if r[4][1] == 1 and r[4][0] == 0]           # last stage, tp rank 0
    assert len(last) == 2
    mean_first = sum(r[2][0] for r in last) / 2
    assert abs(mean_first - ref_losses[0]) < 2e-5 * max(1.0, abs(ref_losses[0]))
    for rank, _, losses, params, (tpr, ppr, dpr) in res:
        exp = shard_gpt_state(ref_sd, cfg, 2, tpr, 2, ppr)
        for n, t in exp.items():
            assert torch.allclose(params[n], t, atol=3e-5, rtol=1e-4), (mode, rank, n, (params[n] - t).abs().max())


@pytest.mark.parametrize("mode", ["dp:drop", "sp:drop", "3dsp:drop"])
def test_dropout_masks_layout_invariant(mode):
    """Hidden and attention dropout 0.1 under DP2 (global micro-batch index), TP2 + SP
    (sequence shards keyed by global element index) and TP2 x PP2 x DP2 + SP: every rank's
    parameters after two steps equal the single-process run with the same micro-batches,
    and the losses match (DP: their mean)."""
    from mxtrain.models.gpt import shard_gpt_state
    cfg, ref_losses, ref_sd = _make_reference(CFG_DROP)
    m = mode.split(":")[0]
    res = _run(mode, world=8 if m.startswith("3d") else 2)
    tp = 2 if m in ("sp", "3dsp") else 1
    pp = 2 if m.startswith("3d") else 1
    dp = 2 if m in ("dp", "3dsp") else 1
    last = [r for r in res if r[4][1] == pp - 1 and r[4][0] == 0]
    assert len(last) == dp
    for step in range(2):
        mean = sum(r[2][step] for r in last) / dp
        assert abs(mean - ref_losses[step]) < 2e-5 * max(1.0, abs(ref_losses[step])), (mode, step, mean, ref_losses)
    for rank, _, losses, params, (tpr, ppr, dpr) in res:
        exp = shard_gpt_state(ref_sd, cfg, tp, tpr, pp, ppr)
        for n, t in exp.items():
            assert torch.allclose(params[n], t, atol=3e-5, rtol=1e-4), (mode, rank, n, (params[n] - t).abs().max())
