"""Tensor / sequence / data parallelism on real HIP streams (the side-stream code that
the gloo CPU tests only exercise synchronously): 2 ranks as 2 processes on the test box's
one MI355X, the direct xGMI kernels (parallel/xgmi.py) as the TP / DP transport, gloo as
the control plane (RCCL cannot put two ranks on one GPU).

* TP2 and TP2 + SP with ``tp_overlap`` / ``sp_gemm_overlap`` on (async dgrad all-reduce /
  reduce-scatter across the wgrad GEMMs on a side stream; the SP all-gather overlapping the
  own-chunk GEMM) must be BIT-identical to the same run with the overlap off, and track the
  single-rank GPU trajectory to bf16 tolerance;
* DP2 with the deferred, per-bucket LN / bias column reductions (ops/norm.py
  ColReduceQueue.flush_group before each bucket's reduce-scatter) must be bit-identical to
  immediate reductions;
* DP2 with the whole step captured in a hipGraph -- its ZeRO-1 reduce-scatter / all-gather
  and the gradient-norm all-reduce on the xGMI kernels inside the graph -- must be
  bit-identical to the eager DP2 step (the N > 1 bench step, bench.py).
Hidden and attention dropout are 0.1 (the reference config): the masks are keyed on global
micro-batch / element / head indices, so the TP / SP / DP runs draw the single-rank masks
and track the single-rank trajectory.
Reference: examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-tp-pp-zero1.yaml:39-40."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(num_layers=2, hidden_size=256, num_attention_heads=4, seq_length=256, max_position_embeddings=256,
           vocab_size=1024, hidden_dropout=0.1, attention_dropout=0.1)
STEPS = 3
DRIFT = 0.15   # parameter drift bound vs the single-rank run, as a fraction of the update norm


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    g = torch.Generator().manual_seed(11)
    x = torch.randint(0, CFG["vocab_size"], (1, 4, CFG["seq_length"] + 1), generator=g)
    return x[..., :-1].contiguous(), x[..., 1:].contiguous()


def _run_trainer(ps, init_sd, tok, lab, env, graph=False):
    from mxtrain.models.gpt import GPTConfig, shard_gpt_state
    from mxtrain.training import GPTTrainer, TrainConfig
    os.environ.update(env)
    cfg = GPTConfig(**CFG)
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=tok.shape[1], global_batch_size=tok.shape[0] * tok.shape[1] * ps.dp,
                                     lr=1e-3), ps)
    tr.flat.load_state_dict(shard_gpt_state(init_sd, cfg, ps.tp, ps.tp_rank, ps.pp, ps.pp_rank))
    tr.opt._refresh_master()
    dev = ps.device
    tok, lab = tok.to(dev), lab.to(dev)
    if graph:
        # step 1 runs eagerly inside capture() (warm-up), steps 2.. replay the graph
        losses = [float(tr.capture(tok, lab, warmup=1))]
        assert tr._graph is not None
        losses += [float(tr.train_step(tok, lab)) for _ in range(STEPS - 1)]
    else:
        losses = [float(tr.train_step(tok, lab)) for _ in range(STEPS)]
    tr.sync_params()
    torch.cuda.synchronize()
    return losses, {n: p.detach().float().cpu().numpy() for n, p in tr.flat.params.items()}, tr


def _worker(rank, world, port, mode, init_path, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK="0", MXTRAIN_XGMI="1", MXTRAIN_XGMI_TIMEOUT_S="20", MXTRAIN_XGMI_MAX_MB="32")
        from mxtrain.parallel import state as pstate
        from mxtrain.parallel import xgmi
        tp = 2 if mode in ("tp", "sp", "tppp", "tpppdp") else 1
        pp = 2 if mode in ("tppp", "tpppdp") else 1
        ps = pstate.initialize_model_parallel(tp=tp, pp=pp, sequence_parallel=mode == "sp", backend="gloo",
                                              device_type="cuda")
        init_sd = torch.load(init_path, weights_only=True)
        tok, lab = _data()
        if mode in ("tppp", "tpppdp"):
            # two micro-batches of two sequences per step (DP2: one per data-parallel rank);
            # pipeline p2p on the xGMI channels, TP collectives on the xGMI kernels
            tok, lab = tok.reshape(2, 2, -1), lab.reshape(2, 2, -1)
            if ps.dp > 1:
                tok, lab = tok[ps.dp_rank:ps.dp_rank + 1], lab[ps.dp_rank:ps.dp_rank + 1]
            a = _run_trainer(ps, init_sd, tok, lab, {"MXTRAIN_TP_OVERLAP": "1"})
            assert a[2].pipeline is not None and a[2].pipeline._xp is not None
            b = _run_trainer(ps, init_sd, tok, lab, {"MXTRAIN_TP_OVERLAP": "0"})
            c = _run_trainer(ps, init_sd, tok, lab, {"MXTRAIN_TP_OVERLAP": "1"}, graph=True)
            for x in xgmi._P2PS.values():
                if x is not None:
                    x.check()
            extra = {"graph_losses": c[0], "graph_params": c[1], "pp_rank": ps.pp_rank, "last": ps.is_last_stage}
        elif mode == "dpgraph":
            tok, lab = tok[:, 2 * rank:2 * rank + 2], lab[:, 2 * rank:2 * rank + 2]
            a = _run_trainer(ps, init_sd, tok, lab, {}, graph=True)
            b = _run_trainer(ps, init_sd, tok, lab, {})
            extra = {"graph_nodes": a[2].graph_census}
        elif mode == "dp":
            tok, lab = tok[:, 2 * rank:2 * rank + 2], lab[:, 2 * rank:2 * rank + 2]
            a = _run_trainer(ps, init_sd, tok, lab, {"MXTRAIN_DEFER_COLREDUCE": "1"})
            assert a[2].stage.rt.colq is not None and a[2].opt.pre_reduce is not None
            deferred = a[2].stage.rt.colq.layout is not None and len(a[2].stage.rt.colq.tables) >= 1
            b = _run_trainer(ps, init_sd, tok, lab, {"MXTRAIN_DEFER_COLREDUCE": "0"})
            extra = {"deferred": deferred, "groups": len(a[2].stage.rt.colq.tables)}
        else:
            a = _run_trainer(ps, init_sd, tok, lab, {"MXTRAIN_TP_OVERLAP": "1"})
            assert a[2].stage.rt.tp_overlap
            b = _run_trainer(ps, init_sd, tok, lab, {"MXTRAIN_TP_OVERLAP": "0"})
            extra = {}
        for c in xgmi._COMMS.values():
            if c is not None:
                c.check()
        q.put((rank, a[0], a[1], b[0], b[1], (ps.tp_rank, ps.dp_rank), extra))
        import torch.distributed as dist
        dist.barrier()
        xgmi.destroy_all()
        pstate.destroy()
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()[-3000:], None, None, None, None))
        raise


def _reference(tmp_path, micro=4):
    """Single-rank GPU run from the same init (the init is also what the workers shard);
    micro=2: two micro-batches of two sequences, the micro-batches of a DP2 step."""
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.parallel.state import ParallelState
    from mxtrain.training import GPTTrainer, TrainConfig
    cfg = GPTConfig(**CFG)
    ps = ParallelState(device=torch.device("cuda"))
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=micro, global_batch_size=4, lr=1e-3), ps)
    init = {k: v.detach().cpu().clone() for k, v in tr.flat.state_dict().items()}
    path = tmp_path / "init.pt"
    torch.save(init, path)
    tok, lab = _data()
    if micro == 2:
        tok, lab = tok.reshape(2, 2, -1), lab.reshape(2, 2, -1)
    losses = [float(tr.train_step(tok.cuda(), lab.cuda())) for _ in range(STEPS)]
    final = {k: v.detach().float().cpu() for k, v in tr.flat.state_dict().items()}
    return cfg, str(path), init, losses, final


def _spawn(mode, init_path, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, init_path, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=200 + 20 * world) for _ in procs], key=lambda t: t[0])
        for p in procs:
            p.join(timeout=30)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    for r in res:
        assert r[1] != "error", r[2]
    return res


@pytest.mark.timeout(280)
@pytest.mark.parametrize("mode", ["tp", "sp"])
def test_tp2_side_streams_on_gpu(tmp_path, mode):
    import numpy as np
    from mxtrain.models.gpt import shard_gpt_state
    cfg, init_path, init, ref_losses, ref_final = _reference(tmp_path)
    res = _spawn(mode, init_path)
    for rank, la, pa, lb, pb, (tpr, _), _ in res:
        # overlap on == overlap off, bit for bit
        assert la == lb, (mode, rank, la, lb)
        for n in pa:
            assert np.array_equal(pa[n], pb[n]), (mode, rank, n)
        # and the single-rank trajectory to bf16 tolerance
        for x, y in zip(la, ref_losses):
            assert abs(x - y) <= 2e-2 * abs(y), (mode, rank, la, ref_losses)
        exp = shard_gpt_state(ref_final, cfg, 2, tpr, 1, 0)
        ini = shard_gpt_state(init, cfg, 2, tpr, 1, 0)
        num = sum(float(((torch.from_numpy(pa[n]) - t) ** 2).sum()) for n, t in exp.items()) ** 0.5
        den = sum(float(((t - ini[n].float()) ** 2).sum()) for n, t in exp.items()) ** 0.5
        # (Adam's first steps move every weight by ~lr whatever the gradient's size, so
        # bf16 rounding differences in near-zero gradients show up as sign flips)
        print(f"[{mode} rank {rank}] parameter drift vs single rank: {num / den:.4f} of the update norm")
        assert num < DRIFT * den, (mode, rank, num / den)


@pytest.mark.timeout(280)
def test_dp2_deferred_colreduce_bit_identical_on_gpu(tmp_path):
    import numpy as np
    cfg, init_path, init, ref_losses, ref_final = _reference(tmp_path)
    res = _spawn("dp", init_path)
    for rank, la, pa, lb, pb, _, extra in res:
        assert extra["deferred"] and extra["groups"] >= 1, extra
        assert la == lb, (rank, la, lb)
        for n in pa:
            assert np.array_equal(pa[n], pb[n]), (rank, n)
    # both DP ranks hold the same parameters
    for n in res[0][2]:
        assert np.array_equal(res[0][2][n], res[1][2][n]), n


@pytest.mark.timeout(280)
def test_dp2_graph_captured_step_bit_identical_on_gpu(tmp_path):
    """The N > 1 bench step: DP2 + ZeRO-1 with the whole step in a hipGraph (reduce-scatter,
    all-gather and the gradient-norm all-reduce captured on the xGMI transport) equals the
    eager DP2 step bit for bit, and both ranks track the single-rank run with the same
    two micro-batches (dropout masks are layout-invariant)."""
    import numpy as np
    from mxtrain.models.gpt import shard_gpt_state
    cfg, init_path, init, ref_losses, ref_final = _reference(tmp_path, micro=2)
    res = _spawn("dpgraph", init_path)
    for rank, la, pa, lb, pb, _, extra in res:
        assert extra["graph_nodes"]["kernel"] > 0, extra
        assert la == lb, (rank, la, lb)
        for n in pa:
            assert np.array_equal(pa[n], pb[n]), (rank, n)
    for n in res[0][2]:
        assert np.array_equal(res[0][2][n], res[1][2][n]), n
    # mean of the two ranks' losses = the single-rank loss of the same two micro-batches
    for step in range(STEPS):
        mean = (res[0][1][step] + res[1][1][step]) / 2
        assert abs(mean - ref_losses[step]) <= 2e-2 * abs(ref_losses[step]), (step, mean, ref_losses)
    pa = res[0][2]
    exp = shard_gpt_state(ref_final, cfg, 1, 0, 1, 0)
    ini = shard_gpt_state(init, cfg, 1, 0, 1, 0)
    num = sum(float(((torch.from_numpy(pa[n]) - t) ** 2).sum()) for n, t in exp.items()) ** 0.5
    den = sum(float(((t - ini[n].float()) ** 2).sum()) for n, t in exp.items()) ** 0.5
    print(f"[dpgraph] parameter drift vs single rank: {num / den:.4f} of the update norm")
    assert num < DRIFT * den, num / den


@pytest.mark.timeout(420)
@pytest.mark.parametrize("mode,world", [("tppp", 4), ("tpppdp", 8)])
def test_tp2_pp2_on_gpu(tmp_path, mode, world):
    """BASELINE config 4's topology on real HIP streams: TP2 x PP2 (4 processes) and
    TP2 x PP2 x DP2 (8 processes) on the box's one GPU -- 1F1B over the xGMI p2p channels,
    TP all-reduces and ZeRO-1 collectives on the xGMI kernels, hidden + attention dropout
    0.1.  Against the single-rank run with the same two micro-batches: losses within 2 %,
    parameter drift < 10 % of the update norm; TP overlap on / off bit-identical; the
    hipGraph-captured step (p2p, TP and DP collectives inside) bit-identical to eager."""
    import numpy as np
    from mxtrain.models.gpt import shard_gpt_state
    cfg, init_path, init, ref_losses, ref_final = _reference(tmp_path, micro=2)
    res = _spawn(mode, init_path, world=world)
    last_losses = []
    for rank, la, pa, lb, pb, (tpr, dpr), extra in res:
        assert la == lb, (mode, rank, la, lb)
        assert la == extra["graph_losses"], (mode, rank, la, extra["graph_losses"])
        for n in pa:
            assert np.array_equal(pa[n], pb[n]), (mode, rank, n)
            assert np.array_equal(pa[n], extra["graph_params"][n]), (mode, rank, n, "graph")
        ppr = extra["pp_rank"]
        exp = shard_gpt_state(ref_final, cfg, 2, tpr, 2, ppr)
        ini = shard_gpt_state(init, cfg, 2, tpr, 2, ppr)
        num = sum(float(((torch.from_numpy(pa[n]) - t) ** 2).sum()) for n, t in exp.items()) ** 0.5
        den = sum(float(((t - ini[n].float()) ** 2).sum()) for n, t in exp.items()) ** 0.5
        print(f"[{mode} rank {rank}] parameter drift vs single rank: {num / den:.4f} of the update norm")
        assert num < 0.10 * den, (mode, rank, num / den)
        if extra["last"] and tpr == 0:
            last_losses.append(la)
    dp = 2 if mode == "tpppdp" else 1
    assert len(last_losses) == dp
    for step in range(STEPS):
        mean = sum(l[step] for l in last_losses) / dp
        assert abs(mean - ref_losses[step]) <= 2e-2 * abs(ref_losses[step]), (mode, step, mean, ref_losses)
