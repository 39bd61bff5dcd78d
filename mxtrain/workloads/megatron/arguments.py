"""Megatron-DeepSpeed command-line subset + DeepSpeed JSON subset.

Every flag the reference's GPT examples pass (pretrain-ddp-zero1.yaml:39-55,78-83 and the
TP/PP variant) is accepted with Megatron's spelling and meaning; common extra Megatron
flags are accepted too.  Flags that only select CUDA-specific implementations
(``--no-masked-softmax-fusion``, ``--use-flash-attn``, ...) are accepted and ignored:
on MI355X the fused HIP kernels are always used.

Precision: ``--fp16`` (the reference's setting) runs the MI355X-native bf16 path --
same 16-bit storage/throughput class, no loss scaling needed; ``--bf16`` is explicit.

Nothing is rewritten silently: every place where the effective run differs from what the
flags ask for (``--fp16`` -> bf16 and its loss-scaler settings, ZeRO stage > 1 -> 1,
ignored implementation-selection flags) is collected in ``args.mx_deviations``, printed
once at start-up and recorded in the checkpoint ``args`` and the metrics JSONL
(``args.mx_effective`` holds the effective precision / dropout / recompute settings).
"""
from __future__ import annotations

import argparse
import json
import os
from typing import List, Optional

# flags that only pick a CUDA implementation (or a Megatron code path with no numerical
# effect here); they are accepted, listed in args.mx_deviations when given, and ignored
IGNORED_FLAGS = [
    "--no-masked-softmax-fusion", "--no-bias-gelu-fusion", "--no-bias-dropout-fusion",
    "--no-gradient-accumulation-fusion", "--use-flash-attn", "--use-flash-attn-v2",
    "--no-async-tensor-model-parallel-allreduce", "--no-pipeline-parallel",
    "--use-cpu-initialization", "--log-timers-to-tensorboard", "--log-batch-size-to-tensorboard",
    "--log-validation-ppl-to-tensorboard", "--log-memory-to-tensorboard", "--log-num-zeros-in-grad",
    "--log-params-norm", "--use-distributed-optimizer", "--overlap-grad-reduce", "--overlap-param-gather",
    "--no-query-key-layer-scaling", "--apply-query-key-layer-scaling",
    "--attention-softmax-in-fp32", "--accumulate-allreduce-grads-in-fp32", "--no-load-rng",
    "--use-contiguous-buffers-in-local-ddp", "--sync-tp-duplicated-parameters", "--empty-unused-memory-level",
]


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="mxtrain Megatron-compatible GPT pre-training", allow_abbrev=False)
    a = p.add_argument
    # model
    a("--num-layers", type=int, default=24)
    a("--hidden-size", type=int, default=1024)
    a("--ffn-hidden-size", type=int, default=None)
    a("--num-attention-heads", type=int, default=16)
    a("--num-key-value-heads", "--num-query-groups", dest="num_key_value_heads", type=int, default=None)
    a("--group-query-attention", action="store_true")
    a("--seq-length", type=int, default=1024)
    a("--max-position-embeddings", type=int, default=None)
    a("--make-vocab-size-divisible-by", type=int, default=128)
    a("--vocab-size", type=int, default=None)
    a("--hidden-dropout", type=float, default=0.1)
    a("--attention-dropout", type=float, default=0.1)
    a("--init-method-std", type=float, default=0.02)
    a("--layernorm-epsilon", "--norm-epsilon", dest="layernorm_epsilon", type=float, default=1e-5)
    a("--normalization", default="LayerNorm", choices=["LayerNorm", "RMSNorm", "layernorm", "rmsnorm"])
    a("--position-embedding-type", default="learned_absolute", choices=["learned_absolute", "rope"])
    a("--use-rotary-position-embeddings", action="store_true")
    a("--rotary-percent", type=float, default=1.0)
    a("--rotary-base", "--rope-theta", dest="rotary_base", type=float, default=10000.0)
    a("--untie-embeddings-and-output-weights", action="store_true")
    a("--swiglu", action="store_true")
    # Megatron-DeepSpeed MoE
    a("--num-experts", type=int, nargs="+", default=[1])
    a("--expert-interval", type=int, default=2)
    a("--topk", type=int, default=1)
    a("--moe-expert-parallel-size", "--ep-world-size", dest="moe_expert_parallel_size", type=int, default=1)
    a("--moe-train-capacity-factor", type=float, default=1.0)
    a("--moe-eval-capacity-factor", type=float, default=1.0)
    a("--moe-min-capacity", type=int, default=4)
    a("--moe-loss-coeff", type=float, default=0.1)
    # training
    a("--micro-batch-size", type=int, default=4)
    a("--global-batch-size", type=int, default=None)
    a("--rampup-batch-size", nargs="*", default=None)
    a("--train-iters", type=int, default=None)
    a("--train-samples", type=int, default=None)
    a("--lr", type=float, default=1.5e-4)
    a("--min-lr", type=float, default=0.0)
    a("--lr-decay-style", default="linear", choices=["constant", "linear", "cosine"])
    a("--lr-decay-iters", type=int, default=None)
    a("--lr-decay-samples", type=int, default=None)
    a("--lr-warmup-fraction", type=float, default=None)
    a("--lr-warmup-iters", type=int, default=0)
    a("--lr-warmup-samples", type=int, default=0)
    a("--weight-decay", type=float, default=0.01)
    a("--clip-grad", type=float, default=1.0)
    a("--adam-beta1", type=float, default=0.9)
    a("--adam-beta2", type=float, default=0.999)
    a("--adam-eps", type=float, default=1e-8)
    a("--optimizer", default="adam", choices=["adam", "adamw"])
    a("--fp16", action="store_true")
    a("--bf16", action="store_true")
    a("--loss-scale", type=float, default=None)
    a("--initial-loss-scale", type=float, default=None)
    a("--seed", type=int, default=1234)
    a("--exit-interval", type=int, default=None)
    a("--exit-duration-in-mins", type=float, default=None)
    # activation recompute (Megatron / DeepSpeed spellings): "full" re-runs each
    # transformer layer's forward inside its backward instead of keeping its activations
    a("--recompute-activations", action="store_true")
    a("--checkpoint-activations", action="store_true")
    a("--deepspeed-activation-checkpointing", action="store_true")
    a("--recompute-granularity", default=None, choices=[None, "full", "selective"])
    # parallelism
    a("--tensor-model-parallel-size", type=int, default=1)
    a("--pipeline-model-parallel-size", type=int, default=1)
    a("--sequence-parallel", action="store_true")
    a("--distributed-backend", default="nccl", choices=["nccl", "gloo", "rccl"])
    a("--local_rank", "--local-rank", dest="local_rank", type=int, default=None)
    a("--DDP-impl", default="local")
    # Ulysses context parallelism (DeepSpeed --ds-sequence-parallel-size; Megatron-core
    # spelling --context-parallel-size is accepted too)
    a("--ds-sequence-parallel-size", "--context-parallel-size", dest="ds_sequence_parallel_size",
      type=int, default=1)
    # data
    a("--data-path", nargs="*", default=None)
    a("--data-cache-path", default=None)
    a("--split", default="969, 30, 1")
    a("--data-impl", default="mmap", choices=["mmap", "infer", "lazy", "cached"])
    a("--vocab-file", default=None)
    a("--merge-file", default=None)
    a("--tokenizer-type", default="GPT2BPETokenizer")
    a("--mock-data", action="store_true")
    a("--num-workers", type=int, default=2)
    # logging / checkpoint / eval
    a("--log-interval", type=int, default=100)
    a("--save-interval", type=int, default=None)
    a("--eval-interval", type=int, default=1000)
    a("--eval-iters", type=int, default=100)
    a("--save", default=None)
    a("--load", default=None)
    a("--no-load-optim", action="store_true")
    a("--no-save-optim", action="store_true")
    a("--finetune", action="store_true")
    a("--tensorboard-dir", default=None)
    a("--log-throughput", action="store_true")
    a("--timing-log-level", type=int, default=0)
    # deepspeed
    a("--deepspeed", action="store_true")
    a("--deepspeed_config", "--deepspeed-config", dest="deepspeed_config", default=None)
    a("--zero-stage", type=int, default=None)
    # mxtrain extensions
    a("--mx-graph", action="store_true", help="capture the whole step in a hipGraph after warm-up")
    a("--mx-metrics-dir", default=None, help="per-rank JSONL metrics (default $LOGS_DIR or $HOME/logs)")
    a("--mx-watchdog", type=float, default=0.0, help="abort a rank after N s without progress")
    a("--mx-auto-resume", action="store_true", help="--load from --save if a checkpoint exists")
    a("--async-save", "--mx-async-save", dest="async_save", action="store_true",
      help="checkpoint writes overlap training (pinned snapshot + writer thread; checkpoint.AsyncCheckpointer)")
    a("--mx-profile", action="store_true", help="torch.profiler trace of steps 5-7 into <metrics>/profile")
    for f in IGNORED_FLAGS:
        p.add_argument(f, action="store_true", help=argparse.SUPPRESS)
    return p


def load_ds_config(path: Optional[str]) -> dict:
    if not path:
        return {}
    with open(path) as f:
        return json.load(f)


def parse_args(argv: Optional[List[str]] = None):
    p = build_parser()
    args, unknown = p.parse_known_args(argv)
    if unknown:
        # Megatron would reject these; keep going but make it visible
        print(f"[mxtrain] ignoring unrecognised arguments: {' '.join(unknown)}", flush=True)
    args.normalization = args.normalization.lower()
    if args.use_rotary_position_embeddings:
        args.position_embedding_type = "rope"
    if args.max_position_embeddings is None:
        args.max_position_embeddings = args.seq_length
    if args.swiglu and args.ffn_hidden_size is None:
        # Megatron-DeepSpeed: 2/3 of 4h (keeps the MLP FLOPs of the GeLU variant), 64-aligned
        args.ffn_hidden_size = int((4 * args.hidden_size * 2 / 3) / 64) * 64
    ds = load_ds_config(args.deepspeed_config) if args.deepspeed else {}
    args.ds_config = ds
    # DeepSpeed JSON subset: batch geometry, ZeRO stage, precision, clipping, optimizer
    if ds.get("train_micro_batch_size_per_gpu"):
        args.micro_batch_size = int(ds["train_micro_batch_size_per_gpu"])
    args.gradient_accumulation_steps = int(ds.get("gradient_accumulation_steps", 1) or 1)
    if "gradient_clipping" in ds:
        args.clip_grad = float(ds["gradient_clipping"])
    zero = (ds.get("zero_optimization") or {}).get("stage")
    args.zero_stage = int(args.zero_stage if args.zero_stage is not None else (zero if zero is not None else 1))
    if (ds.get("fp16") or {}).get("enabled"):
        args.fp16 = True
    if (ds.get("bf16") or {}).get("enabled"):
        args.bf16 = True
    opt = ds.get("optimizer") or {}
    if opt.get("params"):
        pr = opt["params"]
        args.lr = float(pr.get("lr", args.lr))
        if "betas" in pr:
            args.adam_beta1, args.adam_beta2 = (float(x) for x in pr["betas"])
        args.adam_eps = float(pr.get("eps", args.adam_eps))
        args.weight_decay = float(pr.get("weight_decay", args.weight_decay))
    args.ds_train_batch_size = ds.get("train_batch_size")
    args.world_size = int(os.environ.get("WORLD_SIZE", "1"))
    args.rank = int(os.environ.get("RANK", "0"))
    mp = args.tensor_model_parallel_size * args.pipeline_model_parallel_size * args.ds_sequence_parallel_size
    if args.world_size % mp:
        raise SystemExit(f"world size {args.world_size} not divisible by TP*PP*CP={mp}")
    args.data_parallel_size = args.world_size // mp
    if args.global_batch_size is None:
        args.global_batch_size = (args.ds_train_batch_size or
                                  args.micro_batch_size * args.data_parallel_size * args.gradient_accumulation_steps)
    if args.train_iters is None:
        args.train_iters = (args.train_samples // args.global_batch_size) if args.train_samples else 10
    if args.lr_decay_iters is None and args.lr_decay_samples:
        args.lr_decay_iters = args.lr_decay_samples // args.global_batch_size
    if args.lr_decay_iters is None:
        args.lr_decay_iters = args.train_iters
    if args.lr_warmup_fraction is not None:
        args.lr_warmup_iters = int(args.lr_warmup_fraction * args.lr_decay_iters)
    elif args.lr_warmup_samples:
        args.lr_warmup_iters = args.lr_warmup_samples // args.global_batch_size
    _effective(args, argv)
    return args


def _effective(args, argv):
    """Fill args.mx_effective / args.mx_deviations and print every deviation once."""
    dev = []
    if args.fp16:
        msg = "--fp16 -> bf16 compute (fp32 master weights); no dynamic loss scaler is needed or used"
        if args.loss_scale or args.initial_loss_scale:
            msg += f" (loss_scale={args.loss_scale}, initial_loss_scale={args.initial_loss_scale} ignored)"
        dev.append(msg)
    if args.zero_stage > 1:
        dev.append(f"ZeRO stage {args.zero_stage} -> stage 1 (optimizer state sharded; "
                   "288 GB HBM holds the full bf16 gradients)")
    if args.recompute_granularity == "selective":
        dev.append("--recompute-granularity selective -> full layer recompute")
    given = set(a.split("=")[0] for a in (argv if argv is not None else __import__("sys").argv[1:]))
    ign = [f for f in IGNORED_FLAGS if f in given]
    if ign:
        dev.append("accepted without effect (implementation selection only): " + " ".join(ign))
    recompute = bool(args.recompute_activations or args.checkpoint_activations
                     or args.deepspeed_activation_checkpointing or args.recompute_granularity)
    args.mx_recompute = recompute
    args.mx_effective = {
        "compute_dtype": "bf16", "master_dtype": "fp32", "loss_scaling": False,
        "requested_precision": "fp16" if args.fp16 else ("bf16" if args.bf16 else "fp32-flag (bf16 kernels)"),
        "hidden_dropout": args.hidden_dropout, "attention_dropout": args.attention_dropout,
        "activation_recompute": "full" if recompute else None,
        "zero_stage": 1,
    }
    args.mx_deviations = dev
    if int(os.environ.get("RANK", "0")) == 0:
        for d in dev:
            print(f"[mxtrain] WARNING: {d}", flush=True)
