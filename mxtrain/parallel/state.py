"""Process-group topology: one rank per MI355X, groups for DP / TP / PP (+ SP on TP).

Rank order follows Megatron's convention (tensor-parallel fastest, then data, then
pipeline): rank = pp_rank * (dp * tp) + dp_rank * tp + tp_rank, so a TP group is a set
of adjacent GPUs.  On one MI355X node every GPU pair has its own xGMI link, so the
choice only matters for which ring RCCL builds, not for distance.

Replaces Megatron `mpu.initialize_model_parallel` driven by
`--tensor-model-parallel-size/--pipeline-model-parallel-size`
(examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-tp-pp-zero1.yaml:39-40).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    tp: int = 1
    pp: int = 1
    dp: int = 1
    cp: int = 1                              # Ulysses context parallel (sequence split)
    tp_rank: int = 0
    pp_rank: int = 0
    dp_rank: int = 0
    cp_rank: int = 0
    sequence_parallel: bool = False
    cp_group: Optional[object] = None
    grad_group: Optional[object] = None      # dp x cp: replicas that reduce gradients
    tp_group: Optional[object] = None
    pp_group: Optional[object] = None
    dp_group: Optional[object] = None
    mp_group: Optional[object] = None        # tp x pp (for grad-norm reduction)
    embed_group: Optional[object] = None     # first + last pipeline stage (tied embedding)
    pp_ranks: List[int] = field(default_factory=list)
    device: torch.device = torch.device("cpu")

    @property
    def grad_world(self):
        return self.dp * self.cp

    @property
    def is_first_stage(self):
        return self.pp_rank == 0

    @property
    def is_last_stage(self):
        return self.pp_rank == self.pp - 1

    def prev_rank(self):
        return self.pp_ranks[self.pp_rank - 1] if self.pp_rank > 0 else None

    def next_rank(self):
        return self.pp_ranks[self.pp_rank + 1] if self.pp_rank < self.pp - 1 else None

    def tp_active(self):
        return self.tp > 1


_STATE: Optional[ParallelState] = None


def get() -> ParallelState:
    global _STATE
    if _STATE is None:
        _STATE = ParallelState()
    return _STATE


def _env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init_distributed(backend: Optional[str] = None, device_type: Optional[str] = None):
    """Initialise torch.distributed from torchrun-style env (RANK/WORLD_SIZE/MASTER_*).
    backend "nccl" is RCCL on ROCm; gloo is used on CPU."""
    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", 0)
    local_rank = _env_int("LOCAL_RANK", 0)
    # NUMA-local cpuset chosen by the job controller (runtime.affinity)
    from ..runtime.affinity import pin_self_from_env
    cpus = pin_self_from_env(local_rank)
    if cpus and "OMP_NUM_THREADS" not in os.environ:
        torch.set_num_threads(max(1, len(cpus)))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if device_type == "cuda" else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return world, rank, local_rank, device


def initialize_model_parallel(tp: int = 1, pp: int = 1, sequence_parallel: bool = False,
                              backend: Optional[str] = None, device_type: Optional[str] = None,
                              cp: int = 1) -> ParallelState:
    """Rank order (Megatron): tensor fastest, then context (Ulysses), then data, then
    pipeline: rank = ((p * dp + d) * cp + c) * tp + t.  The gradient-reduction group of
    a rank is its dp x cp replicas (context-parallel ranks hold the same weights and see
    different tokens of the same sequences)."""
    global _STATE
    world, rank, local_rank, device = init_distributed(backend, device_type)
    assert world % (tp * pp * cp) == 0, f"world {world} not divisible by tp*pp*cp={tp * pp * cp}"
    dp = world // (tp * pp * cp)
    st = ParallelState(world_size=world, rank=rank, local_rank=local_rank, tp=tp, pp=pp, dp=dp, cp=cp,
                       sequence_parallel=sequence_parallel and tp > 1, device=device)

    def rank_of(p, d, t, c=0):
        return ((p * dp + d) * cp + c) * tp + t

    st.tp_rank = rank % tp
    st.cp_rank = (rank // tp) % cp
    st.dp_rank = (rank // (tp * cp)) % dp
    st.pp_rank = rank // (dp * cp * tp)
    st.pp_ranks = [rank_of(p, st.dp_rank, st.tp_rank, st.cp_rank) for p in range(pp)]
    if world > 1:
        # every rank must call new_group for every group, in the same order
        for p in range(pp):
            for d in range(dp):
                for c in range(cp):
                    ranks = [rank_of(p, d, t, c) for t in range(tp)]
                    g = dist.new_group(ranks)
                    if rank in ranks:
                        st.tp_group = g
        for p in range(pp):
            for t in range(tp):
                for c in range(cp):
                    ranks = [rank_of(p, d, t, c) for d in range(dp)]
                    g = dist.new_group(ranks)
                    if rank in ranks:
                        st.dp_group = g
        if cp > 1:
            for p in range(pp):
                for d in range(dp):
                    for t in range(tp):
                        ranks = [rank_of(p, d, t, c) for c in range(cp)]
                        g = dist.new_group(ranks)
                        if rank in ranks:
                            st.cp_group = g
            for p in range(pp):
                for t in range(tp):
                    ranks = [rank_of(p, d, t, c) for d in range(dp) for c in range(cp)]
                    g = dist.new_group(ranks)
                    if rank in ranks:
                        st.grad_group = g
        for d in range(dp):
            for c in range(cp):
                for t in range(tp):
                    ranks = [rank_of(p, d, t, c) for p in range(pp)]
                    g = dist.new_group(ranks)
                    if rank in ranks:
                        st.pp_group = g
                    eranks = sorted({ranks[0], ranks[-1]})
                    eg = dist.new_group(eranks)
                    if rank in eranks:
                        st.embed_group = eg
        for d in range(dp):
            for c in range(cp):
                ranks = [rank_of(p, d, t, c) for p in range(pp) for t in range(tp)]
                g = dist.new_group(ranks)
                if rank in ranks:
                    st.mp_group = g
    if cp == 1:
        st.grad_group = st.dp_group
    _STATE = st
    return st


def make_expert_groups(st: ParallelState, ep: int):
    """Expert parallelism over the gradient (dp x cp) group: consecutive blocks of ``ep``
    replicas form an EP group (experts split E/ep per rank, tokens exchanged all-to-all);
    replicas holding the same experts form the expert-data-parallel group.  Every rank
    calls new_group for every group in the same order.  Returns (ep_group, edp_group,
    ep_rank); groups are None when their size is 1."""
    W = st.dp * st.cp
    assert W % ep == 0, f"expert-parallel size {ep} must divide dp*cp = {W}"
    tp, pp, dp, cp = st.tp, st.pp, st.dp, st.cp

    def rank_of(p, d, t, c):
        return ((p * dp + d) * cp + c) * tp + t

    ep_group = edp_group = None
    my_idx = None
    for p in range(pp):
        for t in range(tp):
            members = [rank_of(p, d, t, c) for d in range(dp) for c in range(cp)]
            if st.rank in members:
                my_idx = members.index(st.rank)
            if ep > 1:
                for b in range(W // ep):
                    ranks = members[b * ep:(b + 1) * ep]
                    g = dist.new_group(ranks)
                    if st.rank in ranks:
                        ep_group = g
            if W // ep > 1:
                for j in range(ep):
                    ranks = members[j::ep]
                    g = dist.new_group(ranks)
                    if st.rank in ranks:
                        edp_group = g
    return ep_group, edp_group, (my_idx or 0) % ep


def destroy():
    global _STATE
    if dist.is_initialized():
        dist.destroy_process_group()
    _STATE = None
