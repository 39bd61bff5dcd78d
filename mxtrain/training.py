"""GPT training engine: model stage + flat buffers + ZeRO-1 optimizer + schedules.

This is the in-process replacement of the Megatron-DeepSpeed training loop the
reference launches (`torchrun pretrain_gpt.py --deepspeed ...`,
examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-zero1.yaml:72-84):
one process per MI355X, RCCL process groups for DP/TP/PP, micro-batch accumulation,
1F1B pipeline schedule (parallel/pipeline.py), optional hipGraph capture of the whole
step (`capture_graph=True`).
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .models.gpt import GPTConfig, GPTStage, gpt_param_specs
from .ops.rng import DropoutSeed
from .parallel import state as pstate
from .parallel.buffers import FlatParams
from .parallel.zero import DistributedOptimizer, LRSchedule


@dataclass
class TrainConfig:
    micro_batch_size: int = 4
    global_batch_size: Optional[int] = None   # default: micro * dp
    lr: float = 1.5e-4
    min_lr: float = 1e-5
    lr_warmup_iters: int = 0
    lr_decay_iters: Optional[int] = None
    lr_decay_style: str = "cosine"
    weight_decay: float = 0.01
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_eps: float = 1e-8
    clip_grad: float = 1.0
    seed: int = 1234
    overlap_grad_reduce: bool = True
    bucket_numel: int = 40_000_000
    capture_graph: bool = False
    # the first micro-batch's weight-gradient GEMMs write their gradients (beta = 0), so the
    # per-step zero-fill covers only the other ~1 % of the flat gradient buffer (pp = 1)
    overwrite_wgrads: bool = True
    moe_expert_parallel_size: int = 1   # --moe-expert-parallel-size
    # Linear forward / dgrad GEMMs with fused bias / bias-GeLU / GeLU' epilogues
    # (csrc/gemm_nt.hip); False = hipBLASLt + separate bias-GeLU kernels
    fused_linear: bool = True
    # run the ZeRO-1 reduce-scatter / all-gather even on a one-rank data group (tests: the
    # RCCL collectives inside the captured step on one GPU)
    force_dp_collectives: bool = False


class GPTTrainer:
    def __init__(self, cfg: GPTConfig, tcfg: TrainConfig, ps: Optional[pstate.ParallelState] = None,
                 dtype: torch.dtype = torch.bfloat16):
        self.cfg, self.tcfg = cfg, tcfg
        self.ps = ps = ps or pstate.get()
        self.device = ps.device
        self.dtype = dtype
        # (context-parallel ranks share sequences: the batch is split over dp only)
        gb = tcfg.global_batch_size or tcfg.micro_batch_size * ps.dp
        assert gb % (tcfg.micro_batch_size * ps.dp) == 0, "global batch must divide mbs*dp"
        self.num_micro = gb // (tcfg.micro_batch_size * ps.dp)
        self.global_batch = gb
        specs = gpt_param_specs(cfg, ps.tp, ps.pp, ps.pp_rank, ps.sequence_parallel)
        self.flat = FlatParams(specs, self.device, dtype, dp_world=ps.grad_world,
                               bucket_numel=tcfg.bucket_numel)
        gen = torch.Generator().manual_seed(tcfg.seed + 1000 * ps.pp_rank + 100 * ps.tp_rank)
        self.flat.initialize(gen, cfg.num_layers)
        self._sync_initial_params()
        self.seed = DropoutSeed(self.device, *self.seed_bases(tcfg, ps))
        self.stage = GPTStage(cfg, self.flat.params, self.flat.grads, tp=ps.tp, tp_rank=ps.tp_rank,
                              tp_group=ps.tp_group, pp=ps.pp, pp_rank=ps.pp_rank,
                              sequence_parallel=ps.sequence_parallel, seed_t=self.seed.t,
                              cp=ps.cp, cp_rank=ps.cp_rank, cp_group=ps.cp_group,
                              attn_seed_t=self.seed.attn_t)
        self.stage.rt.micro_base = ps.dp_rank * self.num_micro   # global micro-batch index base
        self.stage.rt.batch_dmasks = os.environ.get("MXTRAIN_BATCH_DMASKS", "1") != "0"
        self.stage.rt.fused_linear = tcfg.fused_linear
        self._overwrite = bool(tcfg.overwrite_wgrads and ps.pp == 1)
        if self._overwrite:
            self.flat.set_overwritten(self.stage.gemm_grad_names())
        sched = LRSchedule(tcfg.lr, tcfg.min_lr, tcfg.lr_warmup_iters, tcfg.lr_decay_iters,
                           tcfg.lr_decay_style)
        self.eflat = self.eopt = None
        if cfg.num_experts > 1:
            self._setup_moe(cfg, tcfg, ps, dtype, sched)
        dp_group = ps.grad_group if ps.grad_world > 1 else None
        if dp_group is None and tcfg.force_dp_collectives and dist.is_initialized():
            # (WORLD is the data group only when there is nothing but data parallelism:
            # with TP / PP ranks it would reduce gradients across different shards)
            if dist.get_world_size() != 1:
                raise ValueError("force_dp_collectives with grad_world == 1 needs a 1-rank job "
                                 f"(world {dist.get_world_size()}: tp {ps.tp}, pp {ps.pp}, cp {ps.cp})")
            dp_group = dist.group.WORLD
        self.opt = DistributedOptimizer(
            self.flat, dp_group=dp_group, lr=tcfg.lr, force_collectives=tcfg.force_dp_collectives,
            betas=(tcfg.adam_beta1, tcfg.adam_beta2), eps=tcfg.adam_eps,
            weight_decay=tcfg.weight_decay, clip_grad=tcfg.clip_grad,
            overlap=tcfg.overlap_grad_reduce, tp_rank=ps.tp_rank, tp_group=ps.tp_group,
            sp_group=ps.tp_group if ps.sequence_parallel else None,
            mp_group=ps.mp_group if ps.tp * ps.pp > 1 else None,
            embed_group=ps.embed_group if ps.pp > 1 and cfg.tie_embeddings else None,
            pp_rank=ps.pp_rank, schedule=sched)
        self._setup_xgmi()
        # LN / bias gradient column reductions deferred and batched: ~100 colreduce launches
        # of a GPT-2 step become one at the end of backward (one rank), or one per gradient
        # bucket right before its reduce-scatter is issued (data parallel)
        if (self.device.type == "cuda" and ps.tp == 1 and ps.pp == 1 and self.eopt is None
                and os.environ.get("MXTRAIN_DEFER_COLREDUCE", "1") != "0"):
            from .ops.norm import ColReduceQueue
            group_of = None
            if self.opt.sharded:
                group_of = self.flat.bucket_of_grad_ptr
            self.stage.rt.colq = ColReduceQueue(self.device, group_of=group_of)
            if group_of is not None:
                self.opt.pre_reduce = self.stage.rt.colq.flush_group
        self.pipeline = None
        if ps.pp > 1:
            from .parallel.pipeline import PipelineSchedule
            self.pipeline = PipelineSchedule(self)
        self.iteration = 0
        self._graph = None
        self._static = None
        # checkpoint.AsyncCheckpointer.fence: makes the stream wait for an in-flight
        # checkpoint snapshot before the optimizer rewrites what it is copying
        self.ckpt_fence = None

    # ------------------------------------------------------------------ init
    @staticmethod
    def seed_bases(tcfg, ps):
        """(hidden-dropout seed, attention-dropout seed) of this rank before any step.  The
        same on every data-parallel rank: the masks are keyed on the GLOBAL micro-batch index
        (StepRuntime.micro_base) and element / head / position, so DP ranks draw disjoint
        bits of the one-rank run's masks.  Hidden dropout differs per context-parallel rank
        (different tokens of each sequence); the attention mask is keyed on global heads /
        positions, so it is shared by CP ranks."""
        return (tcfg.seed + 7 * ps.cp_rank, tcfg.seed + 3)

    def _setup_moe(self, cfg, tcfg, ps, dtype, sched):
        """Expert parameters: E/ep experts per rank in a second flat buffer with its own
        ZeRO-1 optimizer over the expert-data-parallel group (models/moe.py)."""
        from .models.gpt import stage_layer_range
        from .models.moe import moe_param_specs
        ep = tcfg.moe_expert_parallel_size
        assert cfg.num_experts % ep == 0, "num_experts must be divisible by the EP size"
        assert ps.pp == 1, "MoE runs with pipeline-parallel size 1 (use expert parallelism)"
        self.ep_group, self.edp_group, self.ep_rank = pstate.make_expert_groups(ps, ep) \
            if ps.world_size > 1 else (None, None, 0)
        edp = ps.grad_world // ep
        l0, l1 = stage_layer_range(cfg, ps.pp, ps.pp_rank)
        especs = moe_param_specs(cfg, l0, l1, ep)
        self.eflat = FlatParams(especs, self.device, dtype, dp_world=edp, bucket_numel=tcfg.bucket_numel)
        # every EP rank initialises different experts; replicas of the same experts agree
        gen = torch.Generator().manual_seed(tcfg.seed + 7777 + 31 * self.ep_rank + 1000 * ps.pp_rank)
        self.eflat.initialize(gen, cfg.num_layers)
        self.eopt = DistributedOptimizer(
            self.eflat, dp_group=self.edp_group, lr=tcfg.lr, betas=(tcfg.adam_beta1, tcfg.adam_beta2),
            eps=tcfg.adam_eps, weight_decay=tcfg.weight_decay, clip_grad=tcfg.clip_grad,
            overlap=tcfg.overlap_grad_reduce, schedule=sched, grad_scale_world=ps.grad_world,
            mp_group=ps.mp_group if ps.tp * ps.pp > 1 else None, norm_groups=(self.ep_group,))
        rt = self.stage.rt
        rt.eparams, rt.egrads, rt.ep_group = self.eflat.params, self.eflat.grads, self.ep_group
        rt.aux_log = []

    def _setup_xgmi(self):
        """Build the direct-xGMI communicators (MXTRAIN_XGMI=1|auto) eagerly, in the same
        group order on every rank, so no handle exchange / autotune happens mid-step."""
        from .parallel import xgmi
        ps = self.ps
        self.xgmi_comms = {}
        if not xgmi.enabled() or self.device.type != "cuda":
            return
        for name, g, n in (("dp", ps.grad_group, ps.grad_world), ("tp", ps.tp_group, ps.tp)):
            if g is not None and n > 1:
                self.xgmi_comms[name] = xgmi.get_comm(g, self.device)

    @property
    def _check_every(self) -> int:
        """Steps between xGMI error-word checks (0 = never): only when xGMI kernels carry
        this rank's traffic; each check synchronises the device once."""
        from .parallel import xgmi
        if not (xgmi._COMMS or xgmi._P2PS):
            return 0
        return int(os.environ.get("MXTRAIN_XGMI_CHECK_EVERY", "100"))

    def check_comms(self) -> None:
        """Raise if any xGMI collective barrier or p2p wait of this rank timed out since the
        start (a timed-out kernel leaves its output unwritten: training must not go on)."""
        from .parallel import xgmi
        for c in list(xgmi._COMMS.values()) + list(xgmi._P2PS.values()):
            if c is not None:
                c.check()

    def _sync_initial_params(self):
        ps = self.ps
        # DP replicas start identical (same generator seed per (pp, tp) already); tied
        # embedding copy on the last stage starts from the first stage's table.
        if ps.pp > 1 and self.cfg.tie_embeddings and ps.embed_group is not None:
            name = "wte" if ps.is_first_stage else ("wte_head" if ps.is_last_stage else None)
            if name is not None:
                src = ps.pp_ranks[0]
                dist.broadcast(self.flat.params[name], src=src, group=ps.embed_group)

    # ------------------------------------------------------------------ step
    def _unit_done(self, unit):
        self.opt.unit_done(unit)
        self.eopt.unit_done(unit)

    def _micro_forward_backward(self, ids, labels, B, S, last_micro, first_micro=False, micro=0):
        rt = self.stage.rt
        rt.wgrad_overwrite = self._overwrite and first_micro
        if self.eopt is not None:
            rt.unit_done = self._unit_done if last_micro else None
        else:
            rt.unit_done = self.opt.unit_done if last_micro else None
        loss = self.stage.forward(ids=ids, labels=labels, B=B, S=S, micro=micro)
        loss.backward()
        return loss.detach()

    def _local(self, t: torch.Tensor) -> torch.Tensor:
        """Whole sequences in, this context-parallel rank's S/cp slice out."""
        if self.ps.cp == 1:
            return t
        from .parallel.ulysses import local_chunk
        return local_chunk(t, self.ps.cp, self.ps.cp_rank)

    def _cp_mean(self, loss: torch.Tensor) -> torch.Tensor:
        if self.ps.cp > 1:
            dist.all_reduce(loss, group=self.ps.cp_group)
            loss = loss / self.ps.cp
        return loss

    def train_step(self, tokens: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """tokens/labels: [num_micro, micro_batch, seq] int64 on device (whole sequences,
        also under context parallelism).  Returns the mean loss over the step as a device
        scalar (last stage; 0 elsewhere)."""
        tokens, labels = self._local(tokens), self._local(labels)
        if self._check_every and self.iteration and self.iteration % self._check_every == 0:
            self.check_comms()
        if self._graph is not None:
            self._static[0].copy_(tokens)
            self._static[1].copy_(labels)
            for o in self._opts:
                o.step_count += 1   # bias corrections use the new step, as in eager step()
                o.set_hyper(o.schedule(o.step_count))
            if self.ckpt_fence is not None:
                self.ckpt_fence()
            self._graph.replay()
            # the replay left this step's update un-gathered (the next replay's body, or a
            # sync_params(), gathers it; re-gathering an unchanged shard is idempotent)
            for o in self._opts:
                o.gather_pending = o.overlap_param_gather
            self.iteration += 1
            return self._static_loss
        return self._train_step_eager(tokens, labels)

    @property
    def _opts(self):
        return [self.opt] + ([self.eopt] if self.eopt is not None else [])

    def _prepare_step(self, nm, B, S):
        self._begin_step()
        self.flat.zero_grad()
        if self.eflat is not None:
            self.eflat.zero_grad()
            self.stage.rt.aux_scale = self.cfg.moe_loss_coeff / nm
            self.stage.rt.aux_log.clear()
        self.seed.advance()
        self.stage.rt.grad_scale = 1.0 / (nm * B * S)
        if self.stage.rt.colq is not None:
            self.stage.rt.colq.begin()
        self.stage.rt.dmasks = None   # regenerated (all layers, one launch) by the first forward

    def _train_step_eager(self, tokens, labels):
        nm, B, S = tokens.shape
        if self.ckpt_fence is not None and any(o.overlap_param_gather for o in self._opts):
            self.ckpt_fence()   # the deferred parameter gather runs at the step's start
        self._prepare_step(nm, B, S)
        if self.pipeline is not None:
            loss = self.pipeline.run(tokens, labels)
        else:
            loss = torch.zeros((), dtype=torch.float32, device=self.device)
            for m in range(nm):
                loss = loss + self._micro_forward_backward(tokens[m].reshape(-1),
                                                           labels[m].reshape(-1), B, S,
                                                           m == nm - 1, m == 0, micro=m)
        if self.stage.rt.colq is not None:
            self.stage.rt.colq.flush()
        if self.ckpt_fence is not None:
            self.ckpt_fence()
        if self.eopt is not None:
            from .parallel.zero import joint_step
            joint_step(self._opts)
        else:
            self.opt.step()
        self.iteration += 1
        return self._cp_mean(loss)

    def capture(self, tokens, labels, warmup: int = 2):
        """Capture one whole training step (fwd, bwd, grad reduce, optimizer) into a
        hipGraph; later steps replay it (no per-kernel launch cost).  The ``warmup``
        side-stream steps are real training steps on (tokens, labels); the loss of the
        last one is returned so callers can account for it."""
        assert self.device.type == "cuda"
        tokens, labels = self._local(tokens), self._local(labels)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        last = None
        with torch.cuda.stream(s):
            for _ in range(warmup):
                last = self._train_step_eager(tokens, labels)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self._static = (tokens.clone(), labels.clone())
        g = torch.cuda.CUDAGraph(keep_graph=True)
        # the optimizer step counter / hyper-parameters are host-driven: set_hyper copies
        # from a pinned buffer that the captured memcpy re-reads on every replay
        step0 = [o.step_count for o in self._opts]
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            loss = self._graph_body()
        for o, c in zip(self._opts, step0):
            o.step_count = c
        # memset nodes replay wrong under the runtime's graph packet capture: fill kernels
        # instead (csrc/graph.hip); the census is kept for diagnostics
        from mxtrain.runtime import graphfix
        self.graph_census = graphfix.census(g)
        self.graph_census["memsets_as_kernels"] = graphfix.memsets_to_kernels(g)
        g.instantiate()
        self._graph = g
        self._static_loss = loss
        return last

    def _graph_body(self):
        tokens, labels = self._static
        nm, B, S = tokens.shape
        # the captured step starts by gathering the shards the previous replay updated
        for o in self._opts:
            o.gather_pending = o.overlap_param_gather
        self._prepare_step(nm, B, S)
        if self.pipeline is not None:
            loss = self.pipeline.run(tokens, labels)
        else:
            loss = torch.zeros((), dtype=torch.float32, device=self.device)
            for m in range(nm):
                loss = loss + self._micro_forward_backward(tokens[m].reshape(-1),
                                                           labels[m].reshape(-1), B, S,
                                                           m == nm - 1, m == 0, micro=m)
        if self.stage.rt.colq is not None:
            self.stage.rt.colq.flush()
        # optimizer body without host-side hyper update (done before each replay)
        from .parallel.zero import joint_update
        joint_update(self._opts)
        for o in self._opts:
            o.gather_pending = False   # (overlap mode) the next replay's body gathers
            o._gather_events.clear()
            o._last_event = None
            o.reset_pending()
        return self._cp_mean(loss)

    def _wait_unit_all(self, unit):
        for o in self._opts:
            o.wait_unit(unit)

    def _begin_step(self):
        for o in self._opts:
            o.begin_param_gather()
        if any(o.overlap_param_gather for o in self._opts):
            self.stage.rt.before_unit = self._wait_unit_all if self.eopt is not None else self.opt.wait_unit
        else:
            self.stage.rt.before_unit = None

    def sync_params(self):
        """Complete a deferred parameter all-gather (call before reading parameters)."""
        for o in self._opts:
            o.finish_param_gather()
        self.stage.rt.before_unit = None

    @torch.no_grad()
    def eval_step(self, tokens: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """Forward-only loss (dropout off, no gradients, optimizer untouched); mean over
        the step's tokens on the last stage."""
        tokens, labels = self._local(tokens), self._local(labels)
        nm, B, S = tokens.shape
        self.sync_params()
        rt = self.stage.rt
        rt.training = False
        rt.unit_done = None
        rt.grad_scale = 1.0 / (nm * B * S)
        try:
            if self.pipeline is not None:
                return self._cp_mean(self.pipeline.run_forward_only(tokens, labels))
            loss = torch.zeros((), dtype=torch.float32, device=self.device)
            for m in range(nm):
                loss = loss + self.stage.forward(ids=tokens[m].reshape(-1), labels=labels[m].reshape(-1),
                                                 B=B, S=S, micro=m).detach()
            return self._cp_mean(loss)
        finally:
            rt.training = True

    # ------------------------------------------------------------------ utils
    def tokens_per_step(self):
        return self.global_batch * self.cfg.seq_length


def synthetic_batch(cfg: GPTConfig, num_micro: int, micro_batch: int, device, generator=None):
    """Synthetic token stream of the configured shape (no dataset on the box)."""
    x = torch.randint(0, cfg.vocab_size, (num_micro, micro_batch, cfg.seq_length + 1),
                      generator=generator, dtype=torch.int64)
    x = x.to(device)
    return x[..., :-1].contiguous(), x[..., 1:].contiguous()
