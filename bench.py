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

The line also carries the second half of BASELINE.json's metric, Mask R-CNN R50-FPN
training images/s (whole job, the same N GPUs) at the reference's two configs (tensorpack:
1 img/GPU, examples/maskrcnn/train-maskrcnn-tensorpack.yaml:16-35; aws-samples: 4 img/GPU,
examples/maskrcnn/train-maskrcnn-aws.yaml:29), measured after the GPT window by
scripts/bench_maskrcnn.py: every bench rank starts one child rank, so at N > 1 the children
are an N-rank data-parallel job (synthetic COCO-shaped 800 x <=1333 images, random-init
weights, full training step incl. SGD; the in-repo MIOpen find-db skips the conv search).
--no-maskrcnn skips it.

Both steps are whole-step hipGraph replays at every N: at N > 1 the captured GPT step holds
its ZeRO-1 reduce-scatter / all-gather, and the Mask R-CNN step its bucketed gradient
all-reduces.  At N > 1 each collective runs on RCCL or on the direct 7-link xGMI kernels,
whichever the autotune (--xgmi auto, the N > 1 default) measured faster for its size.
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import sys
import time


def _coll_summary(tr):
    comms = getattr(tr, "xgmi_comms", {}) or {}
    if not comms:
        return "rccl" if tr.device.type == "cuda" else "gloo"
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


def _child_env(world: int, rank: int, port: int) -> dict:
    """Environment of a Mask R-CNN child rank: the parent's rank / local rank, a NEW
    rendezvous (own port, own TCPStore hosted by child rank 0).  torchrun's agent-store
    variables are dropped: with TORCHELASTIC_USE_AGENT_STORE the child would wait for an
    agent store on the new port that nobody hosts."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    for k in ("GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE", "ROLE_NAME"):
        env.pop(k, None)
    if world > 1:
        env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                   LOCAL_RANK=os.environ.get("LOCAL_RANK", str(rank)),
                   LOCAL_WORLD_SIZE=os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    else:
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
            env.pop(k, None)
    return env


def run_maskrcnn(batch: int, steps: int, warmup: int, world: int = 1, rank: int = 0, port: int = 0,
                 extra=(), workers: int = 6, timeout: float = 300.0) -> dict:
    """One Mask R-CNN training throughput run -> {"img_s": .., ...} (rank 0) / {"rc": 0} (others).

    Every bench rank starts ONE child process (``scripts/bench_maskrcnn.py``) with its own
    rank, so at N > 1 the children form an N-rank data-parallel job (fresh rendezvous on
    ``port``) -- the reference's Horovod MPIJob shape, one rank per GPU
    (examples/maskrcnn/train-maskrcnn-tensorpack.yaml:7,34).  A child, never an exec: this
    process has initialised the GPU.  The whole-job images/s comes from child rank 0."""
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    out = tempfile.mktemp(prefix=f"mx_mrcnn_r{rank}_", suffix=".jsonl")
    cmd = [sys.executable, os.path.join(here, "scripts", "bench_maskrcnn.py"), "--batch", str(batch),
           "--steps", str(steps), "--warmup", str(warmup), "--out", out, "--workers", str(workers)] + list(extra)
    t0 = time.time()
    try:
        rc, text = _run_child(cmd, world, rank, port, timeout)
        if rc != 0:
            return {"error": f"rank {rank} rc={rc}: " + text[-400:]}
        if rank != 0:
            return {"rc": 0}
        rec = json.loads(open(out).read().splitlines()[-1]) if os.path.exists(out) else None
        if rec is None:
            return {"error": "no result record: " + text[-300:]}
        res = {"img_s": rec["value"], "n_gpus": rec.get("n_gpus", world), "steps": steps, "warmup": warmup,
               "wall_s": round(time.time() - t0, 1)}
        if rec.get("graph"):
            res["hipgraph"] = {k: rec["graph"][k] for k in ("captures", "replays", "eager")}
        if rec.get("dp_routes"):
            res["dp_routes"] = rec["dp_routes"]
        for k in ("loader_wait_ms", "host_enqueue_ms"):   # host time per step (child rank 0)
            if k in rec:
                res[k] = rec[k]
        return res
    except Exception as e:  # noqa: BLE001 -- the GPT number must still be reported
        return {"error": f"rank {rank}: " + repr(e)[:300]}
    finally:
        if os.path.exists(out):
            os.remove(out)


def gpt3_layout(world: int):
    """BASELINE config 4 (GPT-3 6.7B, TP2 x PP2 x DP2 at 8 GPUs;
    examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-tp-pp-zero1.yaml:39-40) scaled to the
    job: (tp, pp, global batch) with micro-batch 2 -- the whole model on one 288 GB GPU at
    N = 1, TP2 at 2, TP2 x PP2 (4 micro-batches: the 1F1B pipeline filled) at 4, and DP over
    that at 8."""
    if world >= 4 and world % 4 == 0:
        return 2, 2, 8 * (world // 4)
    if world % 2 == 0:
        return 2, 1, 2 * (world // 2)
    return 1, 1, 2 * world


_CHILDREN: set = set()   # live child processes (the deadline kills their process groups)


def _run_child(cmd, world: int, rank: int, port: int, timeout: float, env=None):
    """One child rank (never an exec: this process has initialised the GPU) -> (rc, stdout).
    The child leads its own session, so a timeout or the bench deadline ends the child and
    everything it started (loader workers, Ray-style workers)."""
    import signal
    import subprocess
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         env=env if env is not None else _child_env(world, rank, port), start_new_session=True)
    _CHILDREN.add(p)
    try:
        out, _ = p.communicate(timeout=max(1.0, timeout))
        return p.returncode, out
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        out, _ = p.communicate()
        return 124, (out or "") + f"\n[timeout after {timeout:.0f} s]"
    finally:
        _CHILDREN.discard(p)


def _last_json(text: str):
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{") and line.endswith("}"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


def run_gpt3(world: int, rank: int, port: int, steps: int, warmup: int, extra=(), timeout: float = 300.0) -> dict:
    """BASELINE config 4 phase: every bench rank starts one child rank of a fresh N-rank
    GPT-3 6.7B job (this file, --model gpt3-6.7b, no further phases); child rank 0's JSON
    line is the result."""
    tp, pp, gb = gpt3_layout(world)
    here = os.path.dirname(os.path.abspath(__file__))
    cmd = [sys.executable, os.path.join(here, "bench.py"), "--gpus", str(world), "--model", "gpt3-6.7b",
           "--micro-batch-size", "2", "--global-batch-size", str(gb), "--tp", str(tp), "--pp", str(pp),
           "--steps", str(steps), "--warmup", str(warmup), "--no-maskrcnn", "--no-extra-configs"] + list(extra)
    t0 = time.time()
    rc, out = _run_child(cmd, world, rank, port, timeout)
    if rc != 0:
        return {"error": f"rank {rank} rc={rc}: " + out[-400:]}
    if rank != 0:
        return {"rc": 0}
    rec = _last_json(out)
    if rec is None:
        return {"error": "no result line: " + out[-300:]}
    return {"tok_s": rec["value"], "ms_per_step": rec["ms_per_step"], "steps": steps, "warmup": warmup,
            "tflops_per_gpu": rec.get("tflops_per_gpu"), "mfu_bf16_dense_2.5pf": rec.get("mfu_bf16_dense_2.5pf"),
            "global_batch": gb, "micro_batch": 2, "seq_len": rec["config"]["seq_len"],
            "parallelism": rec["config"]["parallelism"], "hipgraph": rec["config"].get("hipgraph"),
            "loss": rec.get("loss"), "wall_s": round(time.time() - t0, 1)}


def run_resnet(world: int, steps: int, extra=(), timeout: float = 300.0) -> dict:
    """BASELINE config 5 phase (rank 0 only): the Ray-Train-style ResNet-50 launcher
    (mxtrain/workloads/ray/train_resnet50.py, the raytrain chart's workload) with one worker
    per GPU, batch 256 per worker, synthetic ImageNet 224^2; images/s over the steps after
    the first three, as the launcher reports it (data loading included)."""
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    out = tempfile.mktemp(prefix="mx_resnet_", suffix=".jsonl")
    store = tempfile.mkdtemp(prefix="mx_resnet_ckpt_")
    cmd = [sys.executable, os.path.join(here, "mxtrain", "workloads", "ray", "train_resnet50.py"),
           "--num-workers", str(world), "--batch-size", "256", "--epochs", "1", "--steps-per-epoch", str(steps),
           "--storage-path", store, "--result-json", out] + list(extra)
    t0 = time.time()
    try:
        rc, text = _run_child(cmd, 1, 0, 0, timeout)
        graphed = True
        if rc != 0 and time.time() - t0 < timeout / 2:
            # the launcher's hipGraph step failed hard (a crash is not catchable inside the
            # worker): once more with eager steps, in what is left of the phase's time
            print(f"resnet50: graphed run failed (rc={rc}), retrying eagerly: {text[-300:]}", file=sys.stderr,
                  flush=True)
            env = _child_env(1, 0, 0)
            env["MXTRAIN_LIGHTNING_GRAPH"] = "0"
            graphed = False
            rc, text = _run_child(cmd, 1, 0, 0, timeout - (time.time() - t0), env=env)
        if rc != 0:
            return {"error": f"rc={rc}: " + text[-400:]}
        rec = json.loads(open(out).read().splitlines()[-1]) if os.path.exists(out) else None
        if rec is None or rec.get("value") is None:
            return {"error": "no result record: " + text[-300:]}
        return {"img_s": round(rec["value"], 1), "workers": world, "batch_per_worker": 256, "steps": steps,
                "warmup": "3 eager steps + the hipGraph capture step" if graphed and world == 1 else 3,
                "timed_steps": steps - (4 if graphed and world == 1 else 3),
                "hipgraph": graphed and world == 1, "wall_s": round(time.time() - t0, 1)}
    finally:
        import shutil
        if os.path.exists(out):
            os.remove(out)
        shutil.rmtree(store, ignore_errors=True)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_T_START = time.monotonic()
_LINE = {"out": None, "printed": False, "rank": 0}   # the one JSON line (rank 0) and whether it went out
_LINE_LOCK = None


def _emit(final: bool = True):
    """Print the JSON line once (rank 0).  The deadline thread / SIGTERM handler call this
    with whatever has been measured so far, so a phase that overruns never erases the
    numbers of the phases before it."""
    with _LINE_LOCK:
        if _LINE["printed"] or _LINE["rank"] != 0 or _LINE["out"] is None:
            return
        _LINE["printed"] = True
        if not final:
            _LINE["out"]["deadline"] = "bench wall budget reached: later phases cut short"
        print(json.dumps(_LINE["out"]), flush=True)


def _deadline(reason: str):
    """Budget exhausted (or SIGTERM): emit the line, end every child process group, exit."""
    import signal
    print(f"[bench] {reason}: printing the measured fields and exiting", file=sys.stderr, flush=True)
    _emit(final=False)
    for p in list(_CHILDREN):
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
    os._exit(0)


def _arm_deadline(budget_s: float):
    """Hard stop at the wall budget (a thread, so it fires while the main thread sits in a
    child wait or a collective) and on SIGTERM from the driver."""
    import signal
    import threading
    global _LINE_LOCK
    _LINE_LOCK = threading.Lock()
    left = budget_s - (time.monotonic() - _T_START)
    t = threading.Timer(max(1.0, left), _deadline, args=("wall budget reached",))
    t.daemon = True
    t.start()
    try:
        signal.signal(signal.SIGTERM, lambda *_: _deadline("SIGTERM"))
    except ValueError:   # (not the main thread)
        pass


class _Phases:
    """Per-phase wall budget: rank 0 decides each phase's child timeout (its own limit, cut
    to what is left of --budget-s minus a reserve for the phases' result exchange) and
    every rank follows that decision (host-only gloo group), so all ranks skip or run a
    phase together."""

    def __init__(self, budget_s: float, world: int, rank: int, ctrl, min_s=None):
        self.budget_s, self.world, self.rank, self.ctrl = budget_s, world, rank, ctrl
        self.min_s = min_s
        self.skipped = {}

    def left(self) -> float:
        return self.budget_s - (time.monotonic() - _T_START)

    def timeout(self, name: str, own: float, minimum: float, reserve: float = 15.0):
        """-> the child timeout for this phase, or None to skip it (agreed on all ranks)."""
        import torch.distributed as dist
        minimum = self.min_s if self.min_s is not None else minimum
        t = min(own, self.left() - reserve)
        t = t if t >= minimum else -1.0
        if self.world > 1:
            box = [t]
            dist.broadcast_object_list(box, src=0, group=self.ctrl)
            t = box[0]
        if t < 0:
            self.skipped[name] = f"skipped: budget ({max(0.0, self.left()):.0f} s left of {self.budget_s:.0f})"
            return None
        return t


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
    ap.add_argument("--num-layers", type=int, default=None,
                    help="override the model's depth (tests / memory rehearsals; the bench line says so)")
    ap.add_argument("--num-experts", type=int, default=0, help="MoE: experts per MoE layer (every 2nd layer)")
    ap.add_argument("--ep", type=int, default=1, help="MoE expert-parallel size")
    ap.add_argument("--topk", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true",
                    help="disable hipGraph step capture (default: the whole step, its ZeRO-1 "
                         "reduce-scatter / all-gather included, is one graph at every N)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--no-tuned-gemm", action="store_true",
                    help="do not load the checked-in TunableOp GEMM solution tables")
    ap.add_argument("--tune-gemm", action="store_true",
                    help="TunableOp: benchmark every GEMM solution during warmup and write the table "
                         "to $PYTORCH_TUNABLEOP_FILENAME (see scripts/tune_gemms.sh)")
    ap.add_argument("--no-fused-linear", action="store_true",
                    help="hipBLASLt for the Linear forward / dgrad GEMMs + separate bias-GeLU kernels "
                         "(default: csrc/gemm_nt.hip with fused epilogues)")
    ap.add_argument("--no-maskrcnn", action="store_true",
                    help="skip the Mask R-CNN images/s measurements")
    ap.add_argument("--maskrcnn-batches", default="1,4",
                    help="images per GPU of the Mask R-CNN runs (tensorpack 1, aws-samples 4)")
    ap.add_argument("--maskrcnn-steps", default="60:15,40:10",
                    help="timed:warmup steps per Mask R-CNN run (one pair per batch)")
    ap.add_argument("--maskrcnn-workers", type=int, default=6)
    ap.add_argument("--maskrcnn-args", default="",
                    help="extra arguments for scripts/bench_maskrcnn.py, one shell-quoted string "
                         "(tests: a small synthetic set and image size on the CPU)")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="skip the BASELINE config 4 / 5 phases (GPT-3 6.7B tokens/s, Ray-Train ResNet-50 "
                         "images/s) that follow the Mask R-CNN runs")
    ap.add_argument("--extra-steps", default="8:3",
                    help="timed:warmup steps of the GPT-3 6.7B phase")
    ap.add_argument("--resnet-steps", type=int, default=40, help="steps of the ResNet-50 phase (3 warm-up)")
    ap.add_argument("--gpt3-args", default="", help="extra bench.py arguments of the GPT-3 phase (tests)")
    ap.add_argument("--resnet-args", default="", help="extra train_resnet50.py arguments (tests)")
    ap.add_argument("--xgmi", choices=["0", "1", "auto"], default=None,
                    help="direct xGMI peer-to-peer collectives (csrc/comm/xgmi.hip) for the DP "
                         "reduce-scatter / all-gather, the TP all-reduce and the Mask R-CNN bucket "
                         "all-reduce: 0 = RCCL only, 1 = always, auto (default at N > 1) = a fail-fast "
                         "probe, then a bit-exact check against RCCL and a timing of both per message "
                         "size on the live group, agreed on every rank; any failure -> RCCL everywhere. "
                         "The per-size decision is recorded in the JSON line (config.collectives)")
    ap.add_argument("--budget-s", type=float, default=float(os.environ.get("MXTRAIN_BENCH_BUDGET_S", "540")),
                    help="whole-run wall budget (s, from process start).  Each child phase gets "
                         "min(its own timeout, what is left); phases that no longer fit are recorded as "
                         "'skipped: budget'; at the budget the line is printed with what was measured")
    ap.add_argument("--preflight-timeout", type=float, default=150.0,
                    help="wall limit of the xGMI preflight children (N > 1, --xgmi 1/auto)")
    ap.add_argument("--min-phase-s", type=float, default=None, help=argparse.SUPPRESS)   # tests
    ap.add_argument("--test-hang", choices=["start", "after-gpt"], default=None, help=argparse.SUPPRESS)
    ap.add_argument("--lib-set", action="append", default=[], metavar="SETTER=INT",
                    help="call a kernel-library A/B setter before the run (e.g. mx_flash_dropmask_variant=0)")
    args = ap.parse_args()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank_env = int(os.environ.get("RANK", "0"))
    _LINE["rank"] = rank_env
    _arm_deadline(args.budget_s)
    if args.test_hang == "start":   # (tests: a phase child that never finishes)
        time.sleep(3600)
    if args.xgmi is None:
        args.xgmi = "auto" if world_env > 1 else "0"
    os.environ.setdefault("MXTRAIN_XGMI", args.xgmi)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    # xGMI preflight: the direct peer-memory kernels are proven in throwaway children
    # BEFORE this process touches its GPU (mxtrain/parallel/preflight.py); any failure on
    # any rank -> MXTRAIN_XGMI=0 (RCCL) on every rank, with the reason in the line
    from mxtrain.parallel import preflight as _pre
    pre = None
    if _pre.should_run(world_env, os.environ["MXTRAIN_XGMI"]):
        pre = _pre.run_preflight(world_env, rank_env, timeout_s=args.preflight_timeout)
        if rank_env == 0:
            print(f"[bench] xGMI preflight: {pre}", file=sys.stderr, flush=True)

    import torch
    import torch.distributed as dist

    def _sync():
        if torch.cuda.is_available():   # (CPU / gloo rehearsal runs: tests/test_bench_cpu.py)
            torch.cuda.synchronize()

    from mxtrain.models.gpt import GPT_CONFIGS, GPTConfig
    from mxtrain.parallel import state as pstate
    from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch

    ps = pstate.initialize_model_parallel(tp=args.tp, pp=args.pp, sequence_parallel=args.sequence_parallel,
                                          cp=args.cp)
    world = ps.world_size
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    ctrl = dist.new_group(backend="gloo") if world > 1 else None   # host-only phase decisions / waits
    phases = _Phases(args.budget_s, world, ps.rank, ctrl, args.min_phase_s)
    if ps.rank == 0:   # what the deadline prints if the headline phase itself never ends
        _LINE["out"] = {"metric": "tokens/sec Megatron-DeepSpeed GPT-2 345M pretrain (DP+ZeRO-1)", "value": None,
                        "unit": "tokens/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
                        "error": "GPT phase did not finish within the budget"}
    torch.backends.cuda.matmul.allow_tf32 = False
    try:
        torch.backends.cuda.preferred_blas_library("hipblaslt")
    except Exception:
        pass
    from mxtrain.runtime.gemm_tuning import use_tuned_gemms
    if args.lib_set:
        from mxtrain.ops import _lib
        for kv in args.lib_set:
            name, val = kv.split("=")
            _lib._fn(name)(int(val))
    n_tables = 0 if args.no_tuned_gemm else use_tuned_gemms(tune=args.tune_gemm,
                                                               tables=[] if args.tune_gemm else None)
    mcfg = dict(GPT_CONFIGS[args.model])
    if args.seq_length:
        mcfg.update(seq_length=args.seq_length,
                    max_position_embeddings=max(args.seq_length, mcfg.get("max_position_embeddings", 0)))
    if args.num_layers:
        mcfg.update(num_layers=args.num_layers)
    if args.num_experts > 1:
        mcfg.update(num_experts=args.num_experts, moe_topk=args.topk)
    cfg = GPTConfig(**mcfg)
    tcfg = TrainConfig(micro_batch_size=args.micro_batch_size, global_batch_size=args.global_batch_size,
                       overlap_grad_reduce=not args.no_overlap, lr_warmup_iters=0,
                       moe_expert_parallel_size=args.ep, fused_linear=not args.no_fused_linear)
    tr = GPTTrainer(cfg, tcfg, ps)
    gen = torch.Generator().manual_seed(1 + ps.dp_rank)
    tokens, labels = synthetic_batch(cfg, tr.num_micro, args.micro_batch_size, ps.device, gen)

    def barrier():
        if world > 1:
            dist.barrier()

    use_graph = not args.no_graph and torch.cuda.is_available()
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
                "optimizer": "adamw",
                "tuned_gemm_tables": n_tables,
                "collectives": _coll_summary(tr),
                "xgmi_mode": os.environ.get("MXTRAIN_XGMI", "0"),
                "fused_linear": not args.no_fused_linear,
            },
            "tflops_per_gpu": round(flops / world / 1e12, 1),
            "mfu_bf16_dense_2.5pf": round(flops / world / 2.5e15, 4),
            "loss": round(float(loss.item()), 4) if loss is not None else None,
        }
        if args.num_layers:
            out["config"]["num_layers"] = cfg.num_layers
        if pre is not None:
            out["config"]["xgmi_preflight"] = pre
        if graph_err:
            out["graph_error"] = graph_err
        if use_graph and getattr(tr, "graph_census", None):
            out["graph_nodes"] = tr.graph_census
    else:
        out = None
    _LINE["out"] = out   # from here on the deadline prints at least the headline fields
    if args.test_hang == "after-gpt":   # (tests: a stuck later phase; the deadline must print)
        time.sleep(3600)

    def _free_gpt():
        nonlocal tr, tokens, labels
        tr = tokens = labels = None
        import gc
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    if not args.no_maskrcnn:
        # BASELINE.json metric, part 2: Mask R-CNN images/s with the same N GPUs, outside
        # the GPT timed window.  The GPT model is freed first; every rank then runs one child.
        _free_gpt()
        batches = [int(b) for b in args.maskrcnn_batches.split(",") if b]
        sw = [tuple(int(v) for v in p.split(":")) for p in args.maskrcnn_steps.split(",")]
        ports = [_free_port() for _ in batches] if ps.rank == 0 else None
        if world > 1:
            box = [ports]
            dist.broadcast_object_list(box, src=0)
            ports = box[0]
        res = {}
        for i, b in enumerate(batches):
            st, wu = sw[min(i, len(sw) - 1)]
            tmo = phases.timeout(f"maskrcnn_{b}img", 300.0, 45.0)
            if tmo is None:
                res[b] = {"error": phases.skipped[f"maskrcnn_{b}img"]}
                continue
            res[b] = run_maskrcnn(b, st, wu, world=world, rank=ps.rank, port=ports[i],
                                  extra=shlex.split(args.maskrcnn_args), workers=args.maskrcnn_workers,
                                  timeout=tmo)
            if "error" in res[b]:
                print(f"maskrcnn {b} img/GPU: {res[b]['error']}", file=sys.stderr, flush=True)
            if world > 1:   # a failed child on any rank is reported by rank 0
                errs = [None] * world
                dist.all_gather_object(errs, res[b].get("error"), group=ctrl)
                if ps.rank == 0 and "error" not in res[b] and any(errs):
                    res[b] = {"error": next(e for e in errs if e)}
            if out is not None:
                out[f"maskrcnn_img_s_{b}img"] = res[b].get("img_s")
                out.setdefault("maskrcnn_config", {
                    "model": "Mask R-CNN R50-FPN (tensorpack layout)", "n_gpus": world, "dtype": "bf16",
                    "data": "synthetic COCO-shaped 800x<=1333, random-init weights", "unit": "images/s (whole job)",
                    "parallelism": f"dp{world} (one child rank per GPU, bucketed gradient all-reduce)",
                    "conv_search": "MIOpen find (in-repo find-db) + implicit-GEMM HIP convolutions",
                    "step": "whole-step hipGraph replay (gradient all-reduces captured at N > 1)"})
                out["maskrcnn_config"][f"{b}img"] = {k: v for k, v in res[b].items() if k != "img_s"}
    if not args.no_extra_configs:
        # BASELINE.json configs 4 and 5, each a fresh child job on the same N GPUs after the
        # headline phases (outside every timed window above)
        if tr is not None:
            _free_gpt()
        port = _free_port() if ps.rank == 0 else None
        if world > 1:
            box = [port]
            dist.broadcast_object_list(box, src=0, group=ctrl)
            port = box[0]
        st, wu = (int(v) for v in args.extra_steps.split(":"))
        tmo = phases.timeout("gpt3", 300.0, 60.0)
        if tmo is None:
            g3 = {"error": phases.skipped["gpt3"]}
        else:
            g3 = run_gpt3(world, ps.rank, port, st, wu, extra=shlex.split(args.gpt3_args), timeout=tmo)
            if "error" in g3:
                print(f"gpt3-6.7b: {g3['error']}", file=sys.stderr, flush=True)
            if world > 1:
                errs = [None] * world
                dist.all_gather_object(errs, g3.get("error"), group=ctrl)
                if ps.rank == 0 and "error" not in g3 and any(errs):
                    g3 = {"error": next(e for e in errs if e)}
        if out is not None:
            out["gpt3_6.7b_tok_s"] = g3.get("tok_s")
            out["gpt3_6.7b_config"] = {
                "model": "gpt3-6.7b (32 x 4096, 32 heads, seq 2048)", "n_gpus": world, "dtype": "bf16",
                "data": "synthetic tokens, random-init weights", "unit": "tokens/s (whole job)",
                "optimizer": "ZeRO-1 AdamW + clip 1.0", "dropout": "0.1 / 0.1",
                **{k: v for k, v in g3.items() if k != "tok_s"}}
        tmo = phases.timeout("resnet50", 300.0, 45.0)
        rn = None
        if tmo is None:
            rn = {"error": phases.skipped["resnet50"]}
        elif ps.rank == 0:
            rn = run_resnet(world, args.resnet_steps, extra=shlex.split(args.resnet_args), timeout=tmo)
            if "error" in rn:
                print(f"resnet50: {rn['error']}", file=sys.stderr, flush=True)
        if world > 1 and tmo is not None:
            dist.barrier(group=ctrl)   # the other ranks idle on the host while rank 0's workers run
        if out is not None:
            out["resnet50_img_s"] = (rn or {}).get("img_s")
            out["resnet50_config"] = {
                "model": "ResNet-50 (BatchNorm), Ray-Train + Lightning launcher", "n_gpus": world,
                "dtype": "bf16 autocast, channels_last", "data": "synthetic ImageNet 224x224, random-init weights",
                "unit": "images/s (whole job)", **{k: v for k, v in (rn or {}).items() if k != "img_s"}}
    if out is not None:
        out["bench_wall_s"] = round(time.monotonic() - _T_START, 1)
        out["budget_s"] = args.budget_s
    _emit()
    if world > 1:
        dist.barrier(group=ctrl)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
