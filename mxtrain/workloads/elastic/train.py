"""Elastic data-parallel training smoke workload (run under torchrun's elastic agent).

    torchrun --nnodes $PET_NNODES --nproc_per_node $PET_NPROC_PER_NODE \\
        --rdzv_id $PET_RDZV_ID --rdzv_backend c10d --rdzv_endpoint $PET_RDZV_ENDPOINT \\
        -m mxtrain.workloads.elastic.train --ckpt-dir /fsx/ckpt --steps 40

The shape of the reference's elastic jobs (examples/accelerate/bert-glue-mrpc/pretrain.yaml:35-42:
torchrun + c10d rendezvous from PET_* env), small enough for a CPU/gloo test: a linear
regression trained with a fixed *global* batch that is split over however many ranks the
current rendezvous round produced, so the trajectory does not depend on the world size.
Rank 0 checkpoints after every step (atomic rename, ``weights_only`` loads); every
(re)started worker resumes from the newest checkpoint, so a worker failure, a replica
restart or a membership change costs at most one step.  ``MXTRAIN_FAULT`` injects
failures (obs.fault).  Runs on the GPU with RCCL as well (one rank per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.distributed as dist

from ...obs.fault import FaultInjector
from ...parallel.state import init_distributed

DIM = 16


def batch(step: int, global_batch: int):
    g = torch.Generator().manual_seed(1000 + step)
    x = torch.randn(global_batch, DIM, generator=g, dtype=torch.float64)
    w = torch.arange(1, DIM + 1, dtype=torch.float64) / DIM
    y = x @ w + 0.01 * torch.randn(global_batch, generator=g, dtype=torch.float64)
    return x, y


def init_params():
    g = torch.Generator().manual_seed(0)
    return torch.zeros(DIM, dtype=torch.float64).normal_(generator=g)


def train_step(w: torch.Tensor, step: int, global_batch: int, lr: float, rank: int, world: int):
    """One SGD step on this rank's contiguous slice of the global batch; gradients are
    summed over ranks (sum of per-sample grads / global batch = full-batch mean)."""
    x, y = batch(step, global_batch)
    per = global_batch // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    err = xs @ w - ys
    grad = 2.0 * xs.t() @ err / global_batch
    loss = torch.stack([(err * err).sum() / global_batch])
    if world > 1:
        dist.all_reduce(grad)
        dist.all_reduce(loss)
    return w - lr * grad, float(loss[0])


def reference(steps: int, global_batch: int, lr: float) -> torch.Tensor:
    """Single-process trajectory of the same job (what every elastic run must reproduce)."""
    w = init_params()
    for s in range(steps):
        w, _ = train_step(w, s, global_batch, lr, 0, 1)
    return w


def _ckpt_path(d):
    return os.path.join(d, "latest.pt")


def load(d):
    p = _ckpt_path(d)
    if d and os.path.exists(p):
        st = torch.load(p, weights_only=True)
        return st["w"], int(st["step"])
    return init_params(), 0


def save(d, w, step):
    os.makedirs(d, exist_ok=True)
    tmp = _ckpt_path(d) + f".tmp{os.getpid()}"
    torch.save({"w": w, "step": step}, tmp)
    os.replace(tmp, _ckpt_path(d))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--global-batch", type=int, default=48)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--ckpt-dir", required=True)
    ap.add_argument("--step-sleep", type=float, default=0.0, help="seconds per step (test pacing)")
    ap.add_argument("--out", default=None, help="rank 0 writes the final weights/loss as JSON")
    a = ap.parse_args(argv)
    world, rank, _, _ = init_distributed(device_type="cpu")
    if a.global_batch % world:
        raise SystemExit(f"global batch {a.global_batch} not divisible by world size {world}")
    w, start = load(a.ckpt_dir)
    restart = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    print(f"[elastic] round restart={restart} world={world} rank={rank} resume_step={start}", flush=True)
    fault = FaultInjector(rank)
    loss = float("nan")
    for step in range(start, a.steps):
        fault.maybe_fire(step)
        w, loss = train_step(w, step, a.global_batch, a.lr, rank, world)
        if rank == 0:
            save(a.ckpt_dir, w, step + 1)
        if world > 1:
            dist.barrier()
        if a.step_sleep:
            time.sleep(a.step_sleep)
    if rank == 0:
        print(f"[elastic] done steps={a.steps} world={world} loss={loss:.6f}", flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump({"w": w.tolist(), "loss": loss, "world": world}, f)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
