"""Mixture of Experts (P9): routing semantics against an independent loop reference,
the hand-written GPT layer with MoE MLPs against plain autograd (loss + every gradient,
including the load-balancing aux-loss term), and expert parallelism (EP=2 over DP=2,
gloo all-to-all) against the single-process run with all experts local."""
import math
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

from mxtrain.models.gpt import GPTConfig, GPTStage, gpt_param_specs
from mxtrain.models.moe import capacity, moe_param_specs, route
from mxtrain.parallel.buffers import FlatParams
from gpt_reference import gelu_tanh, ref_loss

MOE = dict(num_layers=2, hidden_size=32, num_attention_heads=2, seq_length=8,
           max_position_embeddings=8, vocab_size=64, hidden_dropout=0.0, attention_dropout=0.0, num_experts=4,
           expert_interval=1, moe_topk=2, moe_train_capacity_factor=1.0, moe_min_capacity=2,
           moe_loss_coeff=0.05)


def _loop_route(probs, k, C):
    """Token-by-token reference of capacity routing (first choices before second)."""
    T, E = probs.shape
    topv, topi = probs.topk(k, -1)
    fill = [0] * E
    slot = torch.full((T, k), -1, dtype=torch.long)
    for j in range(k):
        for t in range(T):
            e = int(topi[t, j])
            if fill[e] < C:
                slot[t, j] = e * C + fill[e]
            fill[e] += 1
    gate = topv * (slot >= 0)
    if k > 1:
        gate = gate / gate.sum(-1, keepdim=True).clamp_min(torch.finfo(torch.float32).eps)
    return slot, gate


@pytest.mark.parametrize("k", [1, 2])
def test_route_matches_loop_reference(k):
    g = torch.Generator().manual_seed(k)
    logits = torch.randn(37, 5, generator=g)
    C = 6
    slot, gate, l_aux, frac = route(logits, k, C)
    rs, rg = _loop_route(torch.softmax(logits, -1), k, C)
    assert torch.equal(slot, rs)
    assert torch.allclose(gate, rg, atol=1e-6)
    assert (slot < 0).any()                           # capacity actually drops tokens
    p = torch.softmax(logits, -1)
    top1 = F.one_hot(p.argmax(-1), 5).float()
    assert math.isclose(float(l_aux), float(5 * (p.mean(0) * top1.mean(0)).sum()), rel_tol=1e-5)


def _moe_ref_mlp(x, P, i, cfg):
    """Independent dense-math MoE: per-expert masks, no dispatch buffers."""
    E, k = cfg.num_experts, cfg.moe_topk
    logits = x @ P[f"layers.{i}.router_w"].t()
    probs = torch.softmax(logits, -1)
    T = x.shape[0]
    C = capacity(cfg, T, True)
    slot, gate = _loop_route(probs.detach(), k, C)
    topv, topi = probs.topk(k, -1)
    kept = slot >= 0
    g = topv * kept
    if k > 1:
        g = g / g.sum(-1, keepdim=True).clamp_min(torch.finfo(torch.float32).eps)
    y = torch.zeros_like(x)
    e = f"layers.{i}.experts."
    for j in range(k):
        for ex in range(E):
            sel = (topi[:, j] == ex) & kept[:, j]
            if sel.any():
                hdn = gelu_tanh(x[sel] @ P[e + "fc1_w"][ex].t() + P[e + "fc1_b"][ex])
                out = hdn @ P[e + "fc2_w"][ex].t() + P[e + "fc2_b"][ex]
                y = y.index_add(0, sel.nonzero()[:, 0], out * g[sel, j:j + 1])
    top1 = F.one_hot(topi[:, 0], E).float()
    aux = E * (probs.mean(0) * top1.mean(0)).sum()
    return y, aux


def test_moe_gpt_layer_matches_autograd():
    cfg = GPTConfig(**MOE)
    B, S = 2, 8
    gen = torch.Generator().manual_seed(0)
    dense = FlatParams(gpt_param_specs(cfg), "cpu", torch.float32)
    dense.initialize(gen, cfg.num_layers)
    ex = FlatParams(moe_param_specs(cfg, 0, cfg.num_layers, 1), "cpu", torch.float32)
    ex.initialize(gen, cfg.num_layers)
    for s in ex.specs:   # non-trivial expert biases
        if s.init == "zeros":
            ex.params[s.name].normal_(0, 0.1, generator=gen)
    st = GPTStage(cfg, dense.params, dense.grads, eparams=ex.params, egrads=ex.grads)
    st.rt.grad_scale = 1.0 / (B * S)
    st.rt.aux_scale = cfg.moe_loss_coeff      # one micro-batch
    st.rt.aux_log = []
    ids = torch.randint(0, cfg.vocab_size, (B * S,), generator=gen)
    labels = torch.randint(0, cfg.vocab_size, (B * S,), generator=gen)
    loss = st.forward(ids=ids, labels=labels, B=B, S=S)
    loss.backward()
    assert len(st.rt.aux_log) == 2

    P = {n: p.detach().clone().requires_grad_(True) for n, p in {**dense.params, **ex.params}.items()}
    auxes = []

    def mlp_hook(x, i):
        y, a = _moe_ref_mlp(x, P, i, cfg)
        auxes.append(a)
        return y
    ref = ref_loss(P, ids, labels, cfg, B, S, mlp_hook=mlp_hook)
    total = ref + cfg.moe_loss_coeff * sum(auxes)
    total.backward()
    assert torch.allclose(loss, ref, atol=1e-5), (float(loss), float(ref))
    for a, b in zip(st.rt.aux_log, auxes):
        assert math.isclose(float(a), float(b), rel_tol=1e-5)
    grads = {**dense.grads, **ex.grads}
    for n, p in P.items():
        assert torch.allclose(grads[n], p.grad, atol=3e-5, rtol=1e-4), (n, (grads[n] - p.grad).abs().max())


# --------------------------------------------------------------------------- EP=2
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    g = torch.Generator().manual_seed(11)
    x = torch.randint(0, MOE["vocab_size"], (2, 2, MOE["seq_length"] + 1), generator=g)
    return x[..., :-1].contiguous(), x[..., 1:].contiguous()


def _trainer(ps, ep):
    from mxtrain.training import GPTTrainer, TrainConfig
    return GPTTrainer(GPTConfig(**MOE), TrainConfig(micro_batch_size=2, global_batch_size=4, lr=1e-3,
                                                    overlap_grad_reduce=False, moe_expert_parallel_size=ep),
                      ps, dtype=torch.float32)


def _ep_worker(rank, world, port, init, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from mxtrain.parallel import state as pstate
    try:
        ps = pstate.initialize_model_parallel(backend="gloo", device_type="cpu")
        tr = _trainer(ps, ep=2)
        dense_sd, ex_sd = init
        tr.flat.load_state_dict(dense_sd)
        El = MOE["num_experts"] // 2
        tr.eflat.load_state_dict({n: t[tr.ep_rank * El:(tr.ep_rank + 1) * El] for n, t in ex_sd.items()})
        tr.opt._refresh_master()
        tr.eopt._refresh_master()
        tok, lab = _data()
        tok, lab = tok[ps.dp_rank:ps.dp_rank + 1], lab[ps.dp_rank:ps.dp_rank + 1]
        losses = [float(tr.train_step(tok, lab)) for _ in range(2)]
        tr.sync_params()
        q.put((rank, tr.ep_rank, losses, {n: p.detach().clone().numpy() for n, p in tr.flat.params.items()},
               {n: p.detach().clone().numpy() for n, p in tr.eflat.params.items()}, None))
        pstate.destroy()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, None, None, None, None, traceback.format_exc()))


def test_expert_parallel_ep2_matches_single():
    from mxtrain.parallel.state import ParallelState
    ref = _trainer(ParallelState(), ep=1)
    init = (ref.flat.state_dict(), ref.eflat.state_dict())
    tok, lab = _data()
    ref_losses = [float(ref.train_step(tok, lab)) for _ in range(2)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_ep_worker, args=(r, 2, port, init, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ep_rank, losses, dense, experts, err in res:
        assert err is None, err
        El = MOE["num_experts"] // 2
        assert abs(sum(r[2][0] for r in res) / 2 - ref_losses[0]) < 2e-5
        for n, t in ref.flat.params.items():
            assert torch.allclose(torch.from_numpy(dense[n]), t, atol=3e-5, rtol=1e-4), (rank, n)
        for n, t in ref.eflat.params.items():
            mine = t[ep_rank * El:(ep_rank + 1) * El]
            assert torch.allclose(torch.from_numpy(experts[n]), mine, atol=3e-5, rtol=1e-4), (rank, n)


def test_moe_checkpoint_resume_is_exact(tmp_path):
    """DeepSpeed MoE layout: per-expert model files + expert optimizer shard; resuming
    continues the exact trajectory."""
    from mxtrain.checkpoint import load_checkpoint, save_checkpoint
    from mxtrain.parallel.state import ParallelState
    tok, lab = _data()
    a = _trainer(ParallelState(), ep=1)
    for _ in range(2):
        a.train_step(tok, lab)
    save_checkpoint(str(tmp_path), a, iteration=2)
    files = sorted(os.listdir(tmp_path / "global_step2"))
    assert "layer_0_expert_3_mp_rank_00_model_states.pt" in files
    assert "expp_rank_0_zero_pp_rank_0_mp_rank_00_optim_states.pt" in files
    la = float(a.train_step(tok, lab))
    b = _trainer(ParallelState(), ep=1)
    info = load_checkpoint(str(tmp_path), b)
    assert info["iteration"] == 2
    lb = float(b.train_step(tok, lab))
    assert la == lb
    for n, t in a.eflat.params.items():
        assert torch.equal(t, b.eflat.params[n]), n
