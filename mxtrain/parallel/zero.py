"""ZeRO-1 distributed optimizer over the flat bucketed buffers (P1/P2, M2-M5, M10, M11).

Per step:
  1. backward writes bf16 grads into FlatParams.grad; as soon as every unit of a bucket
     has finished backward, the bucket is reduce-scattered over the DP group on a
     dedicated HIP stream (overlapped with the rest of backward);
  2. grad norm: one fused sum-of-squares over the rank's shard (TP/PP duplicates
     masked out) + one scalar all-reduce -- no host synchronisation anywhere;
  3. one fused AdamW launch over the whole fp32 shard, clip coefficient and inf/nan
     skip computed on device, bf16 params written straight into the all-gather source;
  4. all-gather of the updated bf16 shards back into FlatParams.data.

DeepSpeed ZeRO-1 equivalent of the reference's ds_config `"zero_optimization":
{"stage": 1}` (examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-zero1.yaml:33-38).
With dp == 1 the shard IS the flat buffer (no copies, no collectives).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import collectives as _C
from . import xgmi as _xgmi

from ..ops import optim as optim_ops
from .buffers import ALIGN, FlatParams


class LRSchedule:
    """Megatron OptimizerParamScheduler subset: linear warmup then cosine/linear/constant
    decay to min_lr at lr_decay_iters (`--lr-decay-style cosine`, `--lr-warmup-fraction`)."""

    def __init__(self, lr, min_lr=0.0, warmup_iters=0, decay_iters=None, style="cosine"):
        self.lr, self.min_lr = lr, min_lr
        self.warmup = warmup_iters
        self.decay = decay_iters
        self.style = style

    def __call__(self, it: int) -> float:
        if self.warmup > 0 and it <= self.warmup:
            return self.lr * it / self.warmup
        if self.style == "constant" or self.decay is None:
            return self.lr
        if it > self.decay:
            return self.min_lr
        r = (it - self.warmup) / max(1, self.decay - self.warmup)
        if self.style == "linear":
            c = 1.0 - r
        else:
            c = 0.5 * (math.cos(math.pi * r) + 1.0)
        return self.min_lr + c * (self.lr - self.min_lr)


class DistributedOptimizer:
    def __init__(self, flat: FlatParams, dp_group=None, lr=1.5e-4, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.01, clip_grad=1.0, overlap: bool = True, tp_rank: int = 0,
                 tp_group=None, sp_group=None, mp_group=None, embed_group=None,
                 pp_rank: int = 0, schedule: Optional[LRSchedule] = None,
                 overlap_param_gather: Optional[bool] = None,
                 grad_scale_world: Optional[int] = None, norm_groups=(), force_collectives: bool = False):
        self.flat = flat
        self.dp_group = dp_group
        self.world = dist.get_world_size(dp_group) if dp_group is not None else 1
        self.rank = dist.get_rank(dp_group) if dp_group is not None else 0
        # sharded path (reduce-scatter / all-gather per bucket) at world > 1; forced on a
        # one-rank group it runs the same collectives (tests: RCCL inside the step graph)
        self.sharded = self.world > 1 or (bool(force_collectives) and dp_group is not None)
        self.betas, self.eps, self.wd, self.clip = betas, eps, weight_decay, clip_grad
        # gradients are sum-reduced over dp_group and divided by gs_world (= the number of
        # replicas whose losses are averaged; larger than dp_group for expert parameters)
        self.gs_world = grad_scale_world or self.world
        self.norm_groups = [g for g in norm_groups if g is not None]
        self.schedule = schedule or LRSchedule(lr)
        self.tp_group, self.sp_group, self.mp_group, self.embed_group = (
            tp_group, sp_group, mp_group, embed_group)
        dev = flat.device
        self.device = dev
        # ---- shard geometry: rank r owns slice r of every bucket
        self.slices = []  # (bucket, flat_start, shard_off, n)
        off = 0
        for b in flat.buckets:
            n = b.size // self.world
            assert n % ALIGN == 0
            self.slices.append((b, b.start + self.rank * n, off, n))
            off += n
        self.shard_numel = off
        if not self.sharded:
            self.grad_shard = flat.grad
            self.param_shard = flat.data
        else:
            self.grad_shard = torch.zeros(off, dtype=flat.dtype, device=dev)
            self.param_shard = torch.zeros(off, dtype=flat.dtype, device=dev)
        self.master = torch.empty(off, dtype=torch.float32, device=dev)
        self._refresh_master()
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        # weight-decay and grad-norm inclusion flags per 64-element chunk of the shard
        norm_flags = torch.zeros(flat.numel // ALIGN, dtype=torch.uint8)
        for s in flat.specs:
            o = flat.offsets[s.name] // ALIGN
            n64 = (s.numel + ALIGN - 1) // ALIGN
            count = True
            if s.tp_duplicated and tp_rank != 0:
                count = False
            if s.name == "wte_head":  # tied copy on the last stage; counted on stage 0
                count = False
            norm_flags[o:o + n64] = 1 if count else 0
        norm_flags = norm_flags.to(dev)
        self.wd_flags = self._shard_of(flat.wd_flags)
        self.norm_flags = self._shard_of(norm_flags)
        self.hyper = torch.zeros(optim_ops.H_N, dtype=torch.float32, device=dev)
        # ring of pinned staging buffers: the host runs steps ahead of the GPU, so a
        # buffer is only rewritten once the async copy that last read it has executed
        self._hyper_ring = [torch.zeros(optim_ops.H_N, dtype=torch.float32, pin_memory=dev.type == "cuda")
                            for _ in range(4 if dev.type == "cuda" else 1)]
        self._hyper_events = [None] * len(self._hyper_ring)
        self._hyper_i = 0
        self.hyper_host = self._hyper_ring[0]
        # ||g||^2 is element 0 of a zero-padded 128-byte buffer: the padded size is a
        # valid xGMI message, so with the direct transport the norm all-reduce runs on the
        # device like the bucket collectives and the whole step stays graph-capturable
        self._normsq_buf = torch.zeros(max(32, 4 * self.world), dtype=torch.float32, device=dev)
        self.normsq = self._normsq_buf[:1]
        self.step_count = 0
        # ---- overlap bookkeeping
        self.overlap = overlap and self.sharded and dev.type == "cuda"
        self.comm_stream = torch.cuda.Stream(device=dev) if self.overlap else None
        self.units_left: Dict[int, int] = {}
        self._bucket_units = {b.index: set(b.units) for b in flat.buckets}
        self._shared_buckets = {flat.unit_to_bucket[s.unit] for s in flat.specs if s.shared}
        self._sp_names = [s.name for s in flat.specs if s.sp_reduce]
        self.started = set()
        self.reset_pending()
        # called with a bucket index right before that bucket's gradients are communicated
        # (the trainer's deferred LN / bias column reductions of that bucket: ops/norm.py
        # ColReduceQueue.flush_group)
        self.pre_reduce = None
        # xGMI registered-buffer mode (see _direct); names are local keys only
        self._direct_state: Optional[bool] = None
        self.comm_timing = os.environ.get("MXTRAIN_COMM_TIMING", "0") == "1"
        self._comm_events: List = []
        self._rg_grad, self._rg_pshard = f"zero{id(self)}.grad", f"zero{id(self)}.pshard"
        # ZeRO-1 parameter all-gather deferred to the start of the next step and overlapped
        # with its forward (bucket by bucket, in forward order); the layers wait on their
        # bucket's event (StepRuntime.before_unit -> wait_unit)
        self.overlap_param_gather = (self.overlap if overlap_param_gather is None
                                     else bool(overlap_param_gather) and self.sharded)
        self.gather_pending = False
        self._gather_events: Dict[int, object] = {}
        self._last_event = None

    # ------------------------------------------------------------------ helpers
    def _shard_of(self, per_chunk: torch.Tensor) -> torch.Tensor:
        parts = [per_chunk[fs // ALIGN:(fs + n) // ALIGN] for (_, fs, _, n) in self.slices]
        return torch.cat(parts) if len(parts) > 1 else parts[0].clone()

    def _refresh_master(self):
        for (_, fs, so, n) in self.slices:
            self.master[so:so + n].copy_(self.flat.data[fs:fs + n].float())
        if self.sharded:
            for (_, fs, so, n) in self.slices:
                self.param_shard[so:so + n].copy_(self.flat.data[fs:fs + n])

    def reset_pending(self):
        self.units_left = {b: len(u) for b, u in self._bucket_units.items()}
        self.started = set()

    # ------------------------------------------------------------------ comm timing
    def _timed(self, fn):
        """Run one DP collective; with comm timing on (MXTRAIN_COMM_TIMING=1 or
        ``comm_timing = True``) bracket it with timing events on the stream it runs on.
        Never inside a hipGraph capture (timing events are not capturable)."""
        if not self.comm_timing or self.device.type != "cuda" or torch.cuda.is_current_stream_capturing():
            return fn()
        s = torch.cuda.current_stream(self.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        out = fn()
        e1.record(s)
        self._comm_events.append((e0, e1))
        return out

    def take_comm_ms(self) -> Optional[float]:
        """Total GPU time of the DP collectives issued since the last call (ms; their
        events must have completed -- call after a synchronize), or None when off."""
        if not self.comm_timing:
            return None
        ev, self._comm_events = self._comm_events, []
        return sum(a.elapsed_time(b) for a, b in ev)

    # ------------------------------------------------------------------ DP collectives
    def _direct(self, c) -> bool:
        """Register the flat gradient buffer and the parameter shard with the xGMI
        communicator (once, collectively) so bucket reduce-scatters / all-gathers read the
        peers' buffers in place instead of staging each bucket through a copy-in buffer.
        Never during a hipGraph capture; any failure -> the staged kernels."""
        if self._direct_state is not None:
            return self._direct_state
        if torch.cuda.is_current_stream_capturing() or not _xgmi.direct_enabled():
            return False
        try:
            if not c.selftest_direct():
                raise _xgmi.XGMIUnavailable("registered-buffer self-test failed")
            c.register(self._rg_grad, self.flat.grad)
            c.register(self._rg_pshard, self.param_shard)
            self._direct_state = True
        except _xgmi.XGMIUnavailable as e:
            if self.rank == 0:
                print(f"[mxtrain] {e}; xGMI collectives keep the staged path", flush=True)
            self._direct_state = False
        return self._direct_state

    def _rs(self, out, inp, bstart: Optional[int] = None):
        return self._timed(lambda: self._rs_body(out, inp, bstart))

    def _ag(self, out, inp, shard_off: Optional[int] = None):
        return self._timed(lambda: self._ag_body(out, inp, shard_off))

    def _rs_body(self, out, inp, bstart: Optional[int] = None):
        """Bucket gradient reduce-scatter: direct xGMI kernel when selected (reading the
        peers' registered gradient buckets in place), else RCCL."""
        nb = inp.numel() * inp.element_size()
        c = _xgmi.route(self.dp_group, inp, "reduce_scatter", nb)
        if c is not None:
            if bstart is not None and self._direct(c):
                c.reduce_scatter_direct(out, self._rg_grad, bstart * inp.element_size(), nb)
            else:
                c.reduce_scatter(out, inp)
        else:
            dist.reduce_scatter_tensor(out, inp, group=self.dp_group)

    def _ag_body(self, out, inp, shard_off: Optional[int] = None):
        """Parameter-shard all-gather: direct xGMI kernel when selected (every rank's new
        shard read in place from its registered param_shard), else RCCL."""
        c = _xgmi.route(self.dp_group, inp, "all_gather", out.numel() * out.element_size())
        if c is not None:
            if shard_off is not None and self._direct(c):
                c.all_gather_direct(out, self._rg_pshard, shard_off * inp.element_size())
            else:
                c.all_gather(out, inp)
        else:
            dist.all_gather_into_tensor(out, inp, group=self.dp_group)

    # ------------------------------------------------------------------ grad sync
    def _sp_allreduce(self, bucket):
        if self.sp_group is None:
            return
        for name in self._sp_names:
            if self.flat.unit_to_bucket[self.flat.spec_by_name[name].unit] == bucket.index:
                _C.all_reduce_(self.flat.grads[name], self.sp_group)

    def _start_bucket(self, bi: int):
        if bi in self.started:
            return
        self.started.add(bi)
        b = self.flat.buckets[bi]
        if self.pre_reduce is not None:
            self.pre_reduce(bi)
        if not self.sharded:
            self._sp_allreduce(b)
            return
        (_, _, so, n) = self.slices[bi]
        if self.overlap:
            ev = torch.cuda.current_stream(self.device).record_event()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ev)
                self._sp_allreduce(b)
                self._rs(self.grad_shard[so:so + n], self.flat.grad[b.start:b.end], b.start)
        else:
            self._sp_allreduce(b)
            self._rs(self.grad_shard[so:so + n], self.flat.grad[b.start:b.end], b.start)

    def unit_done(self, unit: int):
        bi = self.flat.unit_to_bucket.get(unit)
        if bi is None:
            return
        self.units_left[bi] -= 1
        if self.units_left[bi] == 0 and bi not in self._shared_buckets:
            self._start_bucket(bi)

    def finish_grads(self):
        """Complete every bucket's reduction (tied-embedding all-reduce first)."""
        if self.embed_group is not None and dist.get_world_size(self.embed_group) > 1:
            for s in self.flat.specs:
                if s.shared == "word_embeddings":
                    _C.all_reduce_(self.flat.grads[s.name], self.embed_group)
        for bi in range(len(self.flat.buckets)):
            self._start_bucket(bi)
        if self.overlap:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)

    # ------------------------------------------------------------------ step
    def set_hyper(self, lr: float):
        t = self.step_count
        b1, b2 = self.betas
        i = self._hyper_i = (self._hyper_i + 1) % len(self._hyper_ring)
        if self._hyper_events[i] is not None:
            self._hyper_events[i].synchronize()
        h = self.hyper_host = self._hyper_ring[i]
        h[optim_ops.H_LR] = lr
        h[optim_ops.H_B1] = b1
        h[optim_ops.H_B2] = b2
        h[optim_ops.H_EPS] = self.eps
        h[optim_ops.H_WD] = self.wd
        h[optim_ops.H_BC1] = 1.0 - b1 ** t
        h[optim_ops.H_BC2] = 1.0 - b2 ** t
        h[optim_ops.H_GS] = 1.0 / self.gs_world
        h[optim_ops.H_CLIP] = self.clip if self.clip else 0.0
        self.hyper.copy_(h, non_blocking=True)
        if self.device.type == "cuda" and not torch.cuda.is_current_stream_capturing():
            self._hyper_events[i] = torch.cuda.current_stream(self.device).record_event()

    def grad_norm_sq(self) -> torch.Tensor:
        optim_ops.sumsq_bf16(self.grad_shard, 1.0 / self.gs_world, out=self.normsq,
                             flags=self.norm_flags)
        from .collectives import all_reduce_
        for g in [self.dp_group if self.world > 1 else None, self.mp_group] + self.norm_groups:
            if g is not None and dist.get_world_size(g) > 1:
                if self._normsq_buf.numel() * 4 % (16 * dist.get_world_size(g)):
                    all_reduce_(self.normsq, g)          # (RCCL: no padding needed)
                else:
                    all_reduce_(self._normsq_buf, g)     # padding stays 0 on every rank
        return self.normsq

    def step(self, lr: Optional[float] = None):
        self.finish_grads()
        self.step_count += 1
        self.set_hyper(lr if lr is not None else self.schedule(self.step_count))
        normsq = self.grad_norm_sq()
        optim_ops.adamw_step(self.master, self.exp_avg, self.exp_avg_sq, self.grad_shard,
                             self.param_shard, self.hyper, normsq=normsq, wd_flags=self.wd_flags)
        self.gather_params()
        self.reset_pending()
        return normsq

    # ------------------------------------------------------------------ param all-gather
    def gather_params(self):
        """After the update: all-gather the new bf16 shards now, or (overlap mode) mark
        them pending for begin_param_gather() at the next step's start."""
        if not self.sharded:
            return
        if self.overlap_param_gather:
            self.gather_pending = True
            return
        for (b, fs, so, n) in self.slices:
            self._ag(self.flat.data[b.start:b.end], self.param_shard[so:so + n], so)

    def begin_param_gather(self):
        """Start the parameter all-gather deferred from the previous step
        (overlap_param_gather), per bucket in forward order.  On the GPU it runs on the comm
        stream and records one event per bucket for wait_unit(); on the CPU it runs inline."""
        gat = self.gather_pending and self.sharded
        self.gather_pending = False
        if not gat:
            return
        cuda = self.device.type == "cuda"
        side = self.comm_stream if cuda else None
        ev0 = torch.cuda.current_stream(self.device).record_event() if side is not None else None
        # buckets are laid out last-layer-first; the forward needs them in reverse order
        for bi in reversed(range(len(self.slices))):
            b, fs, so, n = self.slices[bi]
            if side is not None:
                with torch.cuda.stream(side):
                    side.wait_event(ev0)
                    self._ag(self.flat.data[b.start:b.end], self.param_shard[so:so + n], so)
                    self._gather_events[bi] = self._last_event = side.record_event()
            else:
                self._ag(self.flat.data[b.start:b.end], self.param_shard[so:so + n], so)

    def wait_unit(self, unit: int):
        bi = self.flat.unit_to_bucket.get(unit)
        ev = self._gather_events.pop(bi, None) if bi is not None else None
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)

    def wait_all(self):
        """Order the current stream after every bucket's deferred all-gather (the comm
        stream is in order, so its last event covers all of them)."""
        self._gather_events.clear()
        if self._last_event is not None:
            torch.cuda.current_stream(self.device).wait_event(self._last_event)
            self._last_event = None

    def finish_param_gather(self):
        """Make every parameter current (before eval / checkpointing / inspection)."""
        self.begin_param_gather()
        if self.device.type == "cuda":
            self.wait_all()

    # ------------------------------------------------------------------ checkpoint
    def shard_state(self) -> dict:
        return {"master": self.master, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "step": self.step_count}

    def load_shard_state(self, sd: dict):
        self.master.copy_(sd["master"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.step_count = int(sd["step"])
        # re-materialise bf16 params from the master shard
        for (b, fs, so, n) in self.slices:
            self.param_shard[so:so + n].copy_(self.master[so:so + n].to(self.flat.dtype))
        if self.sharded:
            for (b, fs, so, n) in self.slices:
                self._ag(self.flat.data[b.start:b.end], self.param_shard[so:so + n])


def joint_update(opts: List["DistributedOptimizer"]) -> torch.Tensor:
    """Optimizer body over several flat buffers (dense + MoE experts) that share ONE
    gradient-clipping norm: finish every reduction, sum the squared norms, one fused
    AdamW per buffer, then the parameter all-gathers.  Hyper-parameters must already be
    set (set_hyper); no host synchronisation (capturable)."""
    for o in opts:
        o.finish_grads()
    total = opts[0].grad_norm_sq()
    for o in opts[1:]:
        total.add_(o.grad_norm_sq())
    for o in opts:
        optim_ops.adamw_step(o.master, o.exp_avg, o.exp_avg_sq, o.grad_shard, o.param_shard,
                             o.hyper, normsq=total, wd_flags=o.wd_flags)
    for o in opts:
        o.gather_params()
    return total


def joint_step(opts: List["DistributedOptimizer"], lr: Optional[float] = None) -> torch.Tensor:
    for o in opts:
        o.step_count += 1
        o.set_hyper(lr if lr is not None else o.schedule(o.step_count))
    total = joint_update(opts)
    for o in opts:
        o.reset_pending()
    return total
