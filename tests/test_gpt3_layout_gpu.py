"""BASELINE config 4's layout at its REAL shapes on the box's one MI355X: GPT-3 6.7B geometry
(hidden 4096, 32 heads of D = 128, seq 2048, vocab 50304, micro-batch 2, hidden + attention
dropout 0.1) through TP2 x PP2 x DP2 = 8 processes, depth cut to 4 layers so that eight
ranks' parameters, ZeRO-1 states and activations fit in one GPU's 288 GB.

Transport as on an 8-GPU node with --xgmi 1: TP all-reduces and ZeRO-1 reduce-scatter /
all-gather on the direct xGMI kernels, the 1F1B activations / gradients on the xGMI p2p
channels, gloo as the control plane (RCCL cannot put two ranks on one GPU).  Checked:

* the mean loss of the last pipeline stage's data-parallel ranks is within 2 % of a
  single-rank (DP1, TP1, PP1) run of the same model on the same 4 micro-batches;
* parameters drift from that run by < 10 % of its update norm;
* the hipGraph-captured step (p2p, TP and DP collectives inside the graph) is bit-identical
  to the eager step;
* every rank prints its peak memory (the committed log: profiles/r6/gpt3_layout_memory.txt).

Reference: examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-tp-pp-zero1.yaml:39-40
(--tensor-model-parallel-size 2 --pipeline-model-parallel-size 2 on 8 GPUs)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(num_layers=4, hidden_size=4096, num_attention_heads=32, seq_length=2048, max_position_embeddings=2048,
           hidden_dropout=0.1, attention_dropout=0.1)
STEPS = 3
MICRO = 2          # sequences per micro-batch (the config-4 micro-batch)
N_MICRO = 4        # micro-batches per step over the whole job (2 per data-parallel rank)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    from mxtrain.models.gpt import GPTConfig
    V = GPTConfig(**CFG).vocab_size
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, V, (N_MICRO, MICRO, CFG["seq_length"] + 1), generator=g)
    return x[..., :-1].contiguous(), x[..., 1:].contiguous()


def _trainer(ps, init_sd, n_local):
    from mxtrain.models.gpt import GPTConfig, shard_gpt_state
    from mxtrain.training import GPTTrainer, TrainConfig
    cfg = GPTConfig(**CFG)
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=MICRO, global_batch_size=n_local * MICRO * ps.dp, lr=1e-4), ps)
    tr.flat.load_state_dict(shard_gpt_state(init_sd, cfg, ps.tp, ps.tp_rank, ps.pp, ps.pp_rank))
    tr.opt._refresh_master()
    return cfg, tr


def _worker(rank, world, port, paths, q):
    import time
    t0 = time.time()
    os.makedirs(paths["logdir"], exist_ok=True)
    logf = open(os.path.join(paths["logdir"], f"gpt3_layout_r{rank}.log"), "a", buffering=1)

    def log(msg):   # per-rank progress (a long silent run looks hung to the box's watchdog)
        logf.write(f"[{time.time() - t0:7.1f}s] {msg}\n")

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK="0", MXTRAIN_XGMI="1", MXTRAIN_XGMI_TIMEOUT_S="30", MXTRAIN_XGMI_MAX_MB="640",
                          MXTRAIN_TP_OVERLAP="1")
        from mxtrain.models.gpt import shard_gpt_state
        from mxtrain.parallel import state as pstate
        from mxtrain.parallel import xgmi
        ps = pstate.initialize_model_parallel(tp=2, pp=2, backend="gloo", device_type="cuda")
        log(f"initialised: tp {ps.tp_rank} pp {ps.pp_rank} dp {ps.dp_rank}")
        init_sd = torch.load(paths["init"], weights_only=True)
        log("init loaded")
        tok, lab = _data()
        per = N_MICRO // ps.dp
        tok = tok[ps.dp_rank * per:(ps.dp_rank + 1) * per].to(ps.device)
        lab = lab[ps.dp_rank * per:(ps.dp_rank + 1) * per].to(ps.device)
        torch.cuda.reset_peak_memory_stats()
        # eager
        cfg, tr = _trainer(ps, init_sd, per)
        la = []
        for i in range(STEPS):
            la.append(float(tr.train_step(tok, lab)))
            log(f"eager step {i}: loss {la[-1]}")
        assert tr.pipeline is not None and tr.pipeline._xp is not None, "1F1B must run on the xGMI p2p channels"
        tr.sync_params()
        torch.cuda.synchronize()
        pa = {n: p.detach().float().cpu() for n, p in tr.flat.params.items()}
        peak_eager = torch.cuda.max_memory_allocated()
        del tr
        torch.cuda.empty_cache()
        # captured: step 1 eager inside capture(), steps 2.. replay the graph
        _, tg = _trainer(ps, init_sd, per)
        lg = [float(tg.capture(tok, lab, warmup=1))]
        assert tg._graph is not None
        log(f"captured: loss {lg[-1]}")
        for i in range(STEPS - 1):
            lg.append(float(tg.train_step(tok, lab)))
            log(f"replay {i}: loss {lg[-1]}")
        tg.sync_params()
        torch.cuda.synchronize()
        same = all(torch.equal(pa[n], p.detach().float().cpu()) for n, p in tg.flat.params.items())
        census = getattr(tg, "graph_census", None)
        for c in list(xgmi._COMMS.values()) + list(xgmi._P2PS.values()):
            if c is not None:
                c.check()
        # drift against the single-rank run, on this rank's shard
        ref_final = torch.load(paths["final"], weights_only=True)
        exp = shard_gpt_state(ref_final, cfg, 2, ps.tp_rank, 2, ps.pp_rank)
        ini = shard_gpt_state(init_sd, cfg, 2, ps.tp_rank, 2, ps.pp_rank)
        num = sum(float(((pa[n] - t.float()) ** 2).sum()) for n, t in exp.items()) ** 0.5
        den = sum(float(((t.float() - ini[n].float()) ** 2).sum()) for n, t in exp.items()) ** 0.5
        nparams = sum(p.numel() for p in pa.values())
        log(f"drift {num / max(den, 1e-30):.4f}, bit-identical graph {same}")
        q.put((rank, dict(eager=la, graph=lg, same=same, drift=num / max(den, 1e-30), tp=ps.tp_rank, pp=ps.pp_rank,
                          dp=ps.dp_rank, last=ps.is_last_stage, peak_gib=round(max(peak_eager, torch.cuda.max_memory_allocated()) / 2**30, 2),
                          params_m=round(nparams / 1e6, 1), census=census)))
        import torch.distributed as dist
        dist.barrier()
        xgmi.destroy_all()
        pstate.destroy()
    except Exception:
        import traceback
        log(traceback.format_exc())
        q.put((rank, {"error": traceback.format_exc()[-3000:]}))
        raise


@pytest.mark.timeout(900)
def test_gpt3_tp2_pp2_dp2_real_shapes(tmp_path):
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.parallel.state import ParallelState
    from mxtrain.training import GPTTrainer, TrainConfig
    # single-rank reference from the same init, same 4 micro-batches of 2 sequences
    cfg = GPTConfig(**CFG)
    ps = ParallelState(device=torch.device("cuda"))
    tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=MICRO, global_batch_size=N_MICRO * MICRO, lr=1e-4), ps)
    init = {k: v.detach().cpu().clone() for k, v in tr.flat.state_dict().items()}
    paths = {"init": str(tmp_path / "init.pt"), "final": str(tmp_path / "final.pt"),
             "logdir": os.path.join(os.environ.get("GRAFT_REPO_ROOT", str(tmp_path)), "gpurun_out")}
    torch.save(init, paths["init"])
    tok, lab = _data()
    ref = [float(tr.train_step(tok.cuda(), lab.cuda())) for _ in range(STEPS)]
    torch.save({k: v.detach().float().cpu() for k, v in tr.flat.state_dict().items()}, paths["final"])
    ref_peak = torch.cuda.max_memory_allocated() / 2**30
    del tr, init
    torch.cuda.empty_cache()
    print(f"[gpt3-layout] reference DP1 ({cfg.num_layers} layers, h {cfg.hidden_size}, seq {cfg.seq_length}): "
          f"losses {ref}, peak {ref_peak:.2f} GiB", flush=True)

    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, paths, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=800) for _ in procs)
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert "error" not in res[r], res[r]["error"]
    for r in range(world):
        d = res[r]
        print(f"[gpt3-layout rank {r}] tp {d['tp']} pp {d['pp']} dp {d['dp']}: {d['params_m']} M params, "
              f"peak {d['peak_gib']} GiB, drift {d['drift']:.4f}, eager {d['eager']}, graph {d['graph']}", flush=True)
    tot = sum(res[r]["peak_gib"] for r in range(world))
    print(f"[gpt3-layout] sum of the 8 ranks' peaks: {tot:.1f} GiB (one 288 GB MI355X)", flush=True)
    for r in range(world):
        d = res[r]
        assert d["same"] and d["eager"] == d["graph"], (r, d["eager"], d["graph"])
        assert d["drift"] < 0.10, (r, d["drift"])
    last = [res[r]["eager"] for r in range(world) if res[r]["last"] and res[r]["tp"] == 0]
    assert len(last) == 2
    for s in range(STEPS):
        mean = sum(l[s] for l in last) / len(last)
        assert abs(mean - ref[s]) <= 2e-2 * abs(ref[s]), (s, mean, ref)
