"""GPT pre-training entry point, command-line compatible with Megatron-DeepSpeed's
`pretrain_gpt.py` as the reference launches it:

    torchrun $DISTRIBUTED_ARGS pretrain_gpt.py --deepspeed --deepspeed_config ds.json \\
        $GPT_ARGS $DATA_ARGS $OUTPUT_ARGS --distributed-backend nccl --save $SAVE 2>&1 | tee log

One process per MI355X; RCCL ("nccl") process groups for DP/TP/PP(+SP); the GPT model
runs on mxtrain's HIP kernels; ZeRO-1 AdamW; Megatron-style log lines plus a JSONL
metrics stream; DeepSpeed-layout checkpoints (mxtrain/checkpoint.py).
"""
from __future__ import annotations

import os
import sys
import time

if __package__ in (None, ""):
    # run as a script (`torchrun pretrain_gpt.py`): make the mxtrain package importable
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

import torch
import torch.distributed as dist

from mxtrain.workloads.megatron.arguments import parse_args  # noqa: E402


def print_rank_last(ps, *a):
    if ps.is_last_stage and ps.tp_rank == 0 and ps.dp_rank == 0:
        print(*a, flush=True)


def print_rank_0(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, flush=True)


def main(argv=None):
    args = parse_args(argv)
    from mxtrain.checkpoint import AsyncCheckpointer, latest_iteration, load_checkpoint, save_checkpoint
    from mxtrain.data.gpt_dataset import DistributedSampleLoader, build_train_valid_test
    from mxtrain.models.gpt import GPTConfig
    from mxtrain.obs.fault import FaultInjector, Watchdog
    from mxtrain.obs.metrics import GPUSampler, MetricsWriter, drm_card_for_device, hbm_stats, megatron_line
    from mxtrain.parallel import state as pstate
    from mxtrain.training import GPTTrainer, TrainConfig

    use_cuda = torch.cuda.is_available() and os.environ.get("MXTRAIN_CPU_ONLY") != "1"
    backend = "nccl" if (use_cuda and args.distributed_backend in ("nccl", "rccl")) else "gloo"
    if use_cuda and hasattr(torch.backends.cuda, "preferred_blas_library"):
        torch.backends.cuda.preferred_blas_library("hipblaslt")
        from mxtrain.runtime.gemm_tuning import use_tuned_gemms
        use_tuned_gemms()
    ps = pstate.initialize_model_parallel(args.tensor_model_parallel_size, args.pipeline_model_parallel_size,
                                          args.sequence_parallel, backend=backend,
                                          device_type="cuda" if use_cuda else "cpu",
                                          cp=args.ds_sequence_parallel_size)
    print_rank_0(f"> initialized mxtrain: world {ps.world_size} = TP {ps.tp} x PP {ps.pp} x CP {ps.cp} x DP {ps.dp}, "
                 f"backend {backend}{' (RCCL)' if backend == 'nccl' else ''}, device {ps.device}")

    # ---------------------------------------------------------------- tokenizer / vocab
    vocab_size = args.vocab_size
    tokenizer = None
    if not args.mock_data and args.data_path and args.vocab_file:
        from mxtrain.data.tokenizer import build_tokenizer
        tokenizer = build_tokenizer(args.tokenizer_type, args.vocab_file, args.merge_file, args.vocab_size)
        vocab_size = tokenizer.vocab_size
    vocab_size = vocab_size or 50257
    cfg = GPTConfig(num_layers=args.num_layers, hidden_size=args.hidden_size,
                    num_attention_heads=args.num_attention_heads,
                    num_kv_heads=args.num_key_value_heads if args.group_query_attention or args.num_key_value_heads else None,
                    ffn_hidden_size=args.ffn_hidden_size, vocab_size=vocab_size,
                    make_vocab_size_divisible_by=args.make_vocab_size_divisible_by, seq_length=args.seq_length,
                    max_position_embeddings=args.max_position_embeddings, hidden_dropout=args.hidden_dropout,
                    attention_dropout=args.attention_dropout, layernorm_epsilon=args.layernorm_epsilon,
                    init_method_std=args.init_method_std, normalization=args.normalization,
                    position_embedding="rope" if args.position_embedding_type == "rope" else "learned",
                    rotary_percent=args.rotary_percent, rotary_base=args.rotary_base,
                    swiglu=args.swiglu,
                    num_experts=max(args.num_experts), expert_interval=args.expert_interval,
                    moe_topk=args.topk, moe_train_capacity_factor=args.moe_train_capacity_factor,
                    moe_eval_capacity_factor=args.moe_eval_capacity_factor,
                    moe_min_capacity=args.moe_min_capacity, moe_loss_coeff=args.moe_loss_coeff,
                    tie_embeddings=not args.untie_embeddings_and_output_weights,
                    recompute=args.mx_recompute)
    tcfg = TrainConfig(micro_batch_size=args.micro_batch_size, global_batch_size=args.global_batch_size,
                       lr=args.lr, min_lr=args.min_lr, lr_warmup_iters=args.lr_warmup_iters,
                       lr_decay_iters=args.lr_decay_iters, lr_decay_style=args.lr_decay_style,
                       weight_decay=args.weight_decay, adam_beta1=args.adam_beta1, adam_beta2=args.adam_beta2,
                       adam_eps=args.adam_eps, clip_grad=args.clip_grad, seed=args.seed,
                       moe_expert_parallel_size=args.moe_expert_parallel_size)
    t0 = time.time()
    trainer = GPTTrainer(cfg, tcfg, ps)
    print_rank_0(f"> GPT: {cfg.num_layers} layers, hidden {cfg.hidden_size}, heads {cfg.num_attention_heads}, "
                 f"vocab {vocab_size} (padded {cfg.padded_vocab(ps.tp)}), params {cfg.num_params() / 1e6:.2f}M, "
                 f"built in {time.time() - t0:.1f}s")

    # ---------------------------------------------------------------- checkpoint resume
    consumed = 0
    load_dir = args.load
    if args.mx_auto_resume and not load_dir and args.save and latest_iteration(args.save) is not None:
        load_dir = args.save
    if load_dir and latest_iteration(load_dir) is not None:
        info = load_checkpoint(load_dir, trainer, load_optim=not args.no_load_optim and not args.finetune)
        if args.finetune:
            trainer.iteration = 0
            trainer.opt.step_count = 0
        else:
            consumed = info["consumed_samples"]
        print_rank_0(f"> loaded checkpoint from {load_dir} at iteration {info['iteration']}")

    # ---------------------------------------------------------------- data
    gb = trainer.global_batch
    n_train = args.train_iters * gb
    n_eval = (args.train_iters // max(args.eval_interval, 1) + 1) * args.eval_iters * gb if args.eval_iters else 0
    n_test = args.eval_iters * gb
    data_prefix = args.data_path[-1] if args.data_path else None
    train_ds, valid_ds, test_ds = build_train_valid_test(
        data_prefix, args.split, [n_train, n_eval, n_test], args.seq_length, args.seed, args.data_cache_path,
        vocab_size=vocab_size, mock=args.mock_data or not data_prefix)
    loader = DistributedSampleLoader(train_ds, args.micro_batch_size, gb, ps.dp_rank, ps.dp, consumed)
    valid_loader = (DistributedSampleLoader(valid_ds, args.micro_batch_size, gb, ps.dp_rank, ps.dp)
                    if valid_ds is not None else None)

    def to_device(x):
        x = x.pin_memory() if use_cuda else x
        x = x.to(ps.device, non_blocking=True)
        return x[..., :-1].contiguous(), x[..., 1:].contiguous()

    # ---------------------------------------------------------------- observability
    logs_dir = args.mx_metrics_dir or os.environ.get("LOGS_DIR") or os.path.join(os.environ.get("HOME", "."), "logs")
    metrics = MetricsWriter(logs_dir, ps.rank)
    # power / clocks of this rank's GPU (sysfs, background thread) and the DP collectives'
    # GPU time per step, reported per logging interval
    sampler = GPUSampler(drm_card_for_device(ps.device) if use_cuda else None)
    trainer.opt.comm_timing = trainer.opt.comm_timing or (use_cuda and ps.dp > 1 and not args.mx_graph)
    # effective settings + every deviation from the requested flags, once, in the JSONL
    metrics.write(step=trainer.iteration, event="config", effective=args.mx_effective,
                  deviations=args.mx_deviations)
    tb = None
    if args.tensorboard_dir and ps.is_last_stage and ps.tp_rank == 0 and ps.dp_rank == 0:
        from mxtrain.obs.tensorboard import SummaryWriter
        tb = SummaryWriter(args.tensorboard_dir)
    fault = FaultInjector(ps.rank)
    watchdog = Watchdog(os.path.join(logs_dir, "heartbeat"), ps.rank, args.mx_watchdog)
    from mxtrain.obs.profile import StepProfiler, check_finite, check_finite_enabled
    profiler = StepProfiler(ps.rank, out_dir=os.path.join(logs_dir, "profile") if args.mx_profile else None,
                            mode="torch" if args.mx_profile else None)
    debug_finite = check_finite_enabled()

    # ---------------------------------------------------------------- checkpoint writer
    ackpt = None
    if args.save and args.async_save:
        ackpt = AsyncCheckpointer(trainer)
        trainer.ckpt_fence = ackpt.fence

    def save(it):
        if ackpt is not None:
            ackpt.save(args.save, it, loader.consumed, args=_plain(vars(args)), ds_config=args.ds_config)
            print_rank_0(f"  checkpoint at iteration {it:7d} snapshotted in {ackpt.last_snapshot_s:.2f}s, "
                         f"writing to {args.save} in the background")
        else:
            save_checkpoint(args.save, trainer, it, loader.consumed, args=_plain(vars(args)), ds_config=args.ds_config)
            print_rank_0(f"  successfully saved checkpoint at iteration {it:7d} to {args.save}")

    # ---------------------------------------------------------------- train loop
    it = trainer.iteration
    flops_tok = cfg.flops_per_token()
    start_wall = time.time()
    print_rank_0(f"> training {args.train_iters} iterations, global batch {gb} "
                 f"({trainer.num_micro} micro-batches x {args.micro_batch_size} x DP {ps.dp})")
    t_log = time.time()
    it_log = it
    loss_acc = torch.zeros((), dtype=torch.float32, device=ps.device)
    graph_ready = False
    while it < args.train_iters:
        fault.maybe_fire(it + 1)
        tokens, labels = to_device(loader.next_batch())
        if args.mx_graph and use_cuda and not graph_ready and it >= 2:
            # the capture's warm-up step is this iteration's real step
            loss = trainer.capture(tokens, labels, warmup=1)
            graph_ready = True
        else:
            loss = None
        if loss is None:
            loss = trainer.train_step(tokens, labels)
        profiler.step(it + 1)
        if debug_finite:
            check_finite(it + 1, loss=loss, grad_norm_sq=trainer.opt.normsq)
        it += 1
        loss_acc += loss
        watchdog.beat(it)
        if it % args.log_interval == 0 or it == args.train_iters:
            if use_cuda:
                torch.cuda.synchronize()
            dt = (time.time() - t_log) / max(it - it_log, 1)
            n = it - it_log
            lr = trainer.opt.schedule(trainer.opt.step_count)
            gn = float(trainer.opt.normsq.sqrt().item())
            lv = float(loss_acc.item()) / n
            toks = gb * cfg.seq_length / dt
            tflops = toks * flops_tok / ps.world_size / 1e12
            print_rank_last(ps, megatron_line(it, args.train_iters, loader.consumed, dt * 1000, lr, gb, lv, gn,
                                              samples_per_sec=gb / dt, tflops=tflops, tokens_per_sec=toks))
            comm_ms = trainer.opt.take_comm_ms()
            extra = dict(hbm_stats(ps.device), **sampler.take())
            if comm_ms is not None:
                extra["dp_comm_ms_per_step"] = comm_ms / n
            if ps.is_last_stage and ps.tp_rank == 0:
                metrics.write(step=it, loss=lv, lr=lr, grad_norm=gn, ms_per_step=dt * 1000, tokens_per_s=toks,
                              samples_per_s=gb / dt, tflops_per_gpu=tflops, consumed_samples=loader.consumed,
                              **extra)
            if tb is not None:   # Megatron's tensorboard tags
                tb.add_scalars_flat({"lm loss": lv, "learning-rate": lr, "grad-norm": gn,
                                     "iteration-time": dt, "tokens-per-sec": toks,
                                     "lm loss vs samples": lv}, it)
                tb.flush()
            loss_acc.zero_()
            t_log, it_log = time.time(), it
        if valid_loader is not None and args.eval_interval and it % args.eval_interval == 0 and args.eval_iters:
            evaluate(trainer, valid_loader, args.eval_iters, to_device, ps, it, metrics, "validation")
            t_log = time.time()
        if args.save and args.save_interval and it % args.save_interval == 0:
            save(it)
            t_log = time.time()
        if args.exit_interval and it % args.exit_interval == 0:
            break
        if args.exit_duration_in_mins and (time.time() - start_wall) / 60 > args.exit_duration_in_mins:
            break
    if args.save and (not args.save_interval or it % args.save_interval != 0):
        save(it)
    if ackpt is not None:
        ackpt.wait()
        print_rank_0(f"  successfully saved checkpoint at iteration {it:7d} to {args.save} "
                     f"(last background write {ackpt.last_write_s:.2f}s)")
    if test_ds is not None and args.eval_iters:
        test_loader = DistributedSampleLoader(test_ds, args.micro_batch_size, gb, ps.dp_rank, ps.dp)
        evaluate(trainer, test_loader, args.eval_iters, to_device, ps, it, metrics, "test")
    watchdog.stop()
    if dist.is_initialized():
        dist.barrier()
    print_rank_0(f"> training finished after {it} iterations ({time.time() - start_wall:.1f}s)")
    pstate.destroy()
    sampler.close()
    return 0


def evaluate(trainer, loader, iters, to_device, ps, it, metrics, name):
    total = torch.zeros((), dtype=torch.float32, device=ps.device)
    for _ in range(iters):
        tokens, labels = to_device(loader.next_batch())
        total += trainer.eval_step(tokens, labels)
    if ps.dp > 1:
        dist.all_reduce(total, group=ps.dp_group)
    lv = float(total.item()) / iters / ps.dp
    import math
    ppl = math.exp(min(20.0, lv))
    line = f" {name} loss at iteration {it} | lm loss value: {lv:.6E} | lm loss PPL: {ppl:.6E} | "
    print_rank_last(ps, "-" * (len(line) + 1))
    print_rank_last(ps, line)
    print_rank_last(ps, "-" * (len(line) + 1))
    if ps.is_last_stage and ps.tp_rank == 0:
        metrics.write(step=it, **{f"{name}_loss": lv, f"{name}_ppl": ppl})


def _plain(d):
    out = {}
    for k, v in d.items():
        if isinstance(v, (int, float, str, bool)) or v is None:
            out[k] = v
        elif isinstance(v, (list, tuple)) and all(isinstance(x, (int, float, str, bool)) for x in v):
            out[k] = list(v)
        elif isinstance(v, dict) and k == "mx_effective":   # effective settings (deviations recorded)
            out[k] = {kk: vv for kk, vv in v.items() if isinstance(vv, (int, float, str, bool)) or vv is None}
    return out


if __name__ == "__main__":
    sys.exit(main())
