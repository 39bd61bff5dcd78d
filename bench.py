#!/usr/bin/env python3
"""Headline benchmark: Megatron-DeepSpeed-style GPT-2 345M pre-training throughput.

Config (BASELINE.json config 2 / SURVEY §6): GPT-2 345M (24 x 1024, 16 heads, seq 1024,
learned positions, tied embeddings, hidden dropout 0.1), micro-batch 4 per GPU, bf16
compute with fp32 master weights, AdamW + grad clip 1.0, ZeRO-1 over DP = N GPUs
(weak scaling: global batch = 4 * N sequences).  Synthetic token data and random-init
weights (no dataset / checkpoint on the box).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        bench.py --gpus 8 --steps 20 --warmup 5

Rank 0 prints exactly one JSON line (value = whole-job tokens/s, max step time over ranks).

On one GPU the line also carries the second half of BASELINE.json's metric, Mask R-CNN
R50-FPN training images/s at the reference's two configs (tensorpack: 1 img/GPU,
examples/maskrcnn/train-maskrcnn-tensorpack.yaml:16-35; aws-samples: 4 img/GPU,
examples/maskrcnn/train-maskrcnn-aws.yaml:29), measured after the GPT window by
scripts/bench_maskrcnn.py in a child process (synthetic COCO-shaped 800 x <=1333 images,
random-init weights, full training step incl. SGD; the in-repo MIOpen find-db skips the
conv search).  --no-maskrcnn skips it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def _coll_summary(tr):
    comms = getattr(tr, "xgmi_comms", {}) or {}
    if not comms:
        return "rccl"
    out = {}
    for name, c in comms.items():
        if c is None:
            out[name] = "rccl (xgmi setup failed)"
        elif c.prefer is None:
            out[name] = "xgmi"
        else:
            out[name] = {op: [[nb, "xgmi" if win else "rccl"] for nb, win in v] for op, v in c.prefer.items()} \
                or "rccl (xgmi check failed)"
    return out


def run_maskrcnn(batch: int, steps: int, warmup: int, timeout: float = 420.0) -> dict:
    """One Mask R-CNN training throughput run (child process) -> {"img_s": .., ...}."""
    import subprocess
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    out = tempfile.mktemp(prefix="mx_mrcnn_", suffix=".jsonl")
    cmd = [sys.executable, os.path.join(here, "scripts", "bench_maskrcnn.py"), "--batch", str(batch),
           "--steps", str(steps), "--warmup", str(warmup), "--out", out]
    t0 = time.time()
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
        rec = json.loads(open(out).read().splitlines()[-1]) if r.returncode == 0 and os.path.exists(out) else None
        if rec is None:
            return {"error": f"rc={r.returncode}: " + r.stdout[-300:]}
        return {"img_s": rec["value"], "steps": steps, "warmup": warmup, "wall_s": round(time.time() - t0, 1)}
    except Exception as e:  # noqa: BLE001 -- the GPT number must still be reported
        return {"error": repr(e)[:300]}
    finally:
        if os.path.exists(out):
            os.remove(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="gpt2-345m")
    ap.add_argument("--micro-batch-size", type=int, default=4)
    ap.add_argument("--global-batch-size", type=int, default=None,
                    help="default micro-batch x DP (one micro-batch per step); larger values accumulate "
                         "micro-batches (needed to fill a pipeline)")
    ap.add_argument("--sequence-parallel", action="store_true")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--pp", type=int, default=1)
    ap.add_argument("--cp", type=int, default=1, help="Ulysses context-parallel size (sequence split)")
    ap.add_argument("--seq-length", type=int, default=None, help="override the model's sequence length")
    ap.add_argument("--num-experts", type=int, default=0, help="MoE: experts per MoE layer (every 2nd layer)")
    ap.add_argument("--ep", type=int, default=1, help="MoE expert-parallel size")
    ap.add_argument("--topk", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true", help="disable hipGraph step capture")
    ap.add_argument("--graph", action="store_true",
                    help="capture the step in a hipGraph also when N > 1 (default: single GPU only; "
                         "eager and graph steps measure the same on MI355X, the step is GPU-bound)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--overlap-optimizer", action="store_true",
                    help="defer each step's AdamW per bucket into the next step's forward on a side "
                         "stream (default: AdamW at the end of the step)")
    ap.add_argument("--no-tuned-gemm", action="store_true",
                    help="do not load the checked-in TunableOp GEMM solution tables")
    ap.add_argument("--tune-gemm", action="store_true",
                    help="TunableOp: benchmark every GEMM solution during warmup and write the table "
                         "to $PYTORCH_TUNABLEOP_FILENAME (see scripts/tune_gemms.sh)")
    ap.add_argument("--wgrad-stream", action="store_true",
                    help="run weight-gradient GEMMs on a concurrent side stream")
    ap.add_argument("--no-fused-linear", action="store_true",
                    help="hipBLASLt for the Linear forward / dgrad GEMMs + separate bias-GeLU kernels "
                         "(default: csrc/gemm_nt.hip with fused epilogues)")
    ap.add_argument("--no-maskrcnn", action="store_true",
                    help="skip the Mask R-CNN images/s measurements (run on one GPU only)")
    ap.add_argument("--xgmi", choices=["0", "1", "auto"], default="0",
                    help="direct xGMI peer-to-peer collectives (csrc/comm/xgmi.hip) for the DP "
                         "reduce-scatter / all-gather and TP all-reduce: 0 = RCCL only (default: the "
                         "xGMI kernels have only been exercised by processes sharing one GPU, so the "
                         "scaling runs use RCCL over xGMI), 1 = always, auto = verify against RCCL and "
                         "keep the faster per message size (N > 1)")
    args = ap.parse_args()
    os.environ.setdefault("MXTRAIN_XGMI", args.xgmi)

    import torch
    import torch.distributed as dist

    def _sync():
        if torch.cuda.is_available():   # (CPU / gloo rehearsal runs: tests/test_bench_cpu.py)
            torch.cuda.synchronize()

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from mxtrain.models.gpt import GPT_CONFIGS, GPTConfig
    from mxtrain.parallel import state as pstate
    from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch

    ps = pstate.initialize_model_parallel(tp=args.tp, pp=args.pp, sequence_parallel=args.sequence_parallel,
                                          cp=args.cp)
    world = ps.world_size
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.backends.cuda.matmul.allow_tf32 = False
    try:
        torch.backends.cuda.preferred_blas_library("hipblaslt")
    except Exception:
        pass
    from mxtrain.runtime.gemm_tuning import use_tuned_gemms
    n_tables = 0 if args.no_tuned_gemm else use_tuned_gemms(tune=args.tune_gemm,
                                                               tables=[] if args.tune_gemm else None)
    mcfg = dict(GPT_CONFIGS[args.model])
    if args.seq_length:
        mcfg.update(seq_length=args.seq_length,
                    max_position_embeddings=max(args.seq_length, mcfg.get("max_position_embeddings", 0)))
    if args.num_experts > 1:
        mcfg.update(num_experts=args.num_experts, moe_topk=args.topk)
    cfg = GPTConfig(**mcfg)
    tcfg = TrainConfig(micro_batch_size=args.micro_batch_size, global_batch_size=args.global_batch_size,
                       overlap_grad_reduce=not args.no_overlap, lr_warmup_iters=0,
                       wgrad_stream=args.wgrad_stream, moe_expert_parallel_size=args.ep,
                       overlap_optimizer=args.overlap_optimizer, fused_linear=not args.no_fused_linear)
    tr = GPTTrainer(cfg, tcfg, ps)
    gen = torch.Generator().manual_seed(1 + ps.dp_rank)
    tokens, labels = synthetic_batch(cfg, tr.num_micro, args.micro_batch_size, ps.device, gen)

    def barrier():
        if world > 1:
            dist.barrier()

    use_graph = not args.no_graph and (world == 1 or args.graph)
    graph_err = None
    for _ in range(args.warmup):
        tr.train_step(tokens, labels)
    if use_graph:
        try:
            tr.capture(tokens, labels, warmup=1)
        except Exception as e:  # keep the bench alive; report eager numbers instead
            graph_err = repr(e)[:300]
            use_graph = False
            tr._graph = None
            print(f"graph capture failed, running eager: {graph_err}", file=sys.stderr)
        if world > 1:
            # every rank must take the same path (captured collectives never ran, so a
            # rank whose capture failed left the communicators untouched)
            ok = torch.tensor([1 if use_graph else 0], dtype=torch.int32, device=ps.device)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0 and use_graph:
                use_graph = False
                tr._graph = None
                graph_err = graph_err or "capture failed on another rank"
    for _ in range(2 if use_graph else 0):
        tr.train_step(tokens, labels)
    _sync()
    barrier()
    _sync()
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = tr.train_step(tokens, labels)
    # a deferred AdamW (overlap_optimizer) of the last step is applied inside the timed
    # window too: K + 1 optimizer updates are timed for K steps
    tr.sync_params()
    _sync()
    barrier()
    _sync()
    t1 = time.perf_counter()
    ms = (t1 - t0) * 1000.0 / args.steps
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64, device=ps.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    tokens_per_step = tr.global_batch * cfg.seq_length
    value = tokens_per_step / (ms / 1000.0)
    flops = cfg.flops_per_token() * value
    if ps.rank == 0:
        out = {
            "metric": ("tokens/sec Megatron-DeepSpeed GPT-2 345M pretrain (DP+ZeRO-1)" if args.model == "gpt2-345m"
                       else f"tokens/sec Megatron-DeepSpeed {args.model} pretrain"),
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random tokens, random-init weights)",
            "config": {
                "model": args.model,
                "global_batch": tr.global_batch,
                "micro_batch": args.micro_batch_size,
                "seq_len": cfg.seq_length,
                "parallelism": f"dp{ps.dp}" + (f"_tp{args.tp}" if args.tp > 1 else "")
                               + (f"_pp{args.pp}" if args.pp > 1 else "")
                               + ("_sp" if ps.sequence_parallel else "") + (f"_cp{ps.cp}" if ps.cp > 1 else "")
                               + (f"_moe{args.num_experts}x_ep{args.ep}_top{args.topk}" if args.num_experts > 1 else "")
                               + "_zero1",
                "hidden_dropout": cfg.hidden_dropout,
                "attention_dropout": cfg.attention_dropout,
                "hipgraph": use_graph,
                "wgrad_stream": args.wgrad_stream,
                "optimizer": "adamw_deferred_overlapped" if tr.opt.overlap_update else "adamw",
                "tuned_gemm_tables": n_tables,
                "collectives": _coll_summary(tr),
                "fused_linear": not args.no_fused_linear,
            },
            "tflops_per_gpu": round(flops / world / 1e12, 1),
            "mfu_bf16_dense_2.5pf": round(flops / world / 2.5e15, 4),
            "loss": round(float(loss.item()), 4) if loss is not None else None,
        }
        if graph_err:
            out["graph_error"] = graph_err
        if use_graph and getattr(tr, "graph_census", None):
            out["graph_nodes"] = tr.graph_census
        if world == 1 and not args.no_maskrcnn:
            # BASELINE.json metric, part 2: Mask R-CNN images/s (outside the GPT timed window)
            del tr
            if torch.cuda.is_available():
                torch.cuda.empty_cache()
            m1 = run_maskrcnn(1, 60, 15)
            m4 = run_maskrcnn(4, 40, 10)
            out["maskrcnn_img_s_1img"] = m1.get("img_s")
            out["maskrcnn_img_s_4img"] = m4.get("img_s")
            out["maskrcnn_config"] = {
                "model": "Mask R-CNN R50-FPN (tensorpack layout)", "n_gpus": 1, "dtype": "bf16",
                "data": "synthetic COCO-shaped 800x<=1333, random-init weights",
                "1img": {k: v for k, v in m1.items() if k != "img_s"},
                "4img": {k: v for k, v in m4.items() if k != "img_s"},
                "unit": "images/s", "conv_search": "MIOpen find (in-repo find-db)",
                "step": "whole-step hipGraph replay (1 GPU), runtime packet capture on, memset nodes as fill kernels"}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
