"""Horovod-style API over torch.distributed/RCCL (replaces Horovod 0.28 + OpenMPI for
`TRAINER=horovod`).

Ranks are spawned by mxtrain.launch.mpirun (or any OpenMPI-compatible launcher), so the
OpenMPI env (OMPI_COMM_WORLD_*) or the torchrun env (RANK/WORLD_SIZE/LOCAL_RANK) identify
the process; the data plane is RCCL ("nccl" backend) over xGMI, one process per MI355X.

  init()                      process group + device pinning (GPU = local rank)
  rank() / size() / local_rank() / local_size()
  broadcast_parameters(params, root_rank=0)     initial-state broadcast (M13)
  allreduce(t, average=True)                    one tensor
  DistributedDataParallel(model)                bucketed, backward-overlapped gradient
                                                all-reduce -- Horovod's tensor fusion (K18)
                                                done as DDP buckets sized for xGMI
"""
from __future__ import annotations

import os
from typing import Iterable, Optional

import torch
import torch.distributed as dist

_STATE = {"init": False}


def _env(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return int(v)
    return default


def rank() -> int:
    return _env("OMPI_COMM_WORLD_RANK", "RANK", "PMIX_RANK", default=0)


def size() -> int:
    return _env("OMPI_COMM_WORLD_SIZE", "WORLD_SIZE", default=1)


def local_rank() -> int:
    return _env("OMPI_COMM_WORLD_LOCAL_RANK", "LOCAL_RANK", default=0)


def local_size() -> int:
    return _env("OMPI_COMM_WORLD_LOCAL_SIZE", "LOCAL_WORLD_SIZE", default=1)


def device() -> torch.device:
    if torch.cuda.is_available() and os.environ.get("MXTRAIN_CPU_ONLY") != "1":
        return torch.device("cuda", local_rank() % max(torch.cuda.device_count(), 1))
    return torch.device("cpu")


def init(backend: Optional[str] = None):
    if _STATE["init"]:
        return
    dev = device()
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if size() > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if dev.type == "cuda" else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29501")
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank(), world_size=size(), **kw)
    _STATE["init"] = True


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()
    _STATE["init"] = False


def allreduce(t: torch.Tensor, average: bool = True) -> torch.Tensor:
    if size() > 1:
        dist.all_reduce(t)
        if average:
            t /= size()
    return t


def broadcast_parameters(params: Iterable[torch.Tensor], root_rank: int = 0):
    if size() <= 1:
        return
    for p in params:
        dist.broadcast(p.data if hasattr(p, "data") else p, src=root_rank)


def DistributedDataParallel(model: torch.nn.Module, bucket_cap_mb: int = 64):
    """Bucketed gradient all-reduce overlapped with backward.  64 MB buckets: a single
    xGMI ring moves ~150 GB/s, so a bucket costs ~0.5 ms -- large enough to amortise the
    launch latency, small enough that the last bucket does not trail backward by much."""
    if size() <= 1:
        return model
    dev = device()
    return torch.nn.parallel.DistributedDataParallel(
        model, device_ids=[dev.index] if dev.type == "cuda" else None, bucket_cap_mb=bucket_cap_mb,
        gradient_as_bucket_view=True, broadcast_buffers=False, find_unused_parameters=False)
