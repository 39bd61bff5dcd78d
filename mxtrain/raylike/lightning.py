"""Minimal Lightning-style training loop with the `ray.train.lightning` integration points
(RayDDPStrategy, RayLightningEnvironment, RayTrainReportCallback, prepare_trainer), so
the reference's Ray Lightning workloads keep their structure ("Lightning
Trainer.fit loop ... ray.train.report metrics/checkpoints").

Only what those workloads use: ``LightningModule`` (training_step / validation_step /
configure_optimizers / self.log), ``Trainer(max_epochs, max_steps, precision,
limit_*_batches, callbacks, strategy)``.fit(model, train_dataloaders, val_dataloaders).
``precision="bf16-mixed"`` (or "16-mixed") autocasts to bf16 on the MI355X.
"""
from __future__ import annotations

import os
import tempfile
import time
from typing import Any, Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .train import Checkpoint, get_context, report
from .train.torch import get_device


class LightningModule(nn.Module):
    def __init__(self):
        super().__init__()
        self._logged: Dict[str, float] = {}
        self.trainer: Optional["Trainer"] = None

    @property
    def device(self):
        try:
            return next(self.parameters()).device
        except StopIteration:
            return torch.device("cpu")

    def log(self, name: str, value, prog_bar: bool = False, sync_dist: bool = False, on_step=None, on_epoch=None,
            **kw):
        v = value.detach().float() if torch.is_tensor(value) else torch.tensor(float(value))
        if sync_dist and dist.is_initialized():
            v = v.to(self.device)
            dist.all_reduce(v)
            v = v / dist.get_world_size()
        # kept as a (device) tensor and read only when the metrics are (epoch end, progress
        # lines): a float() here synchronised the host with the GPU on every step, so the
        # next step's launches could never run ahead of the GPU
        self._logged[name] = v

    def logged_metrics(self) -> Dict[str, float]:
        return {k: float(v) for k, v in self._logged.items()}

    def log_dict(self, d: Dict[str, Any], **kw):
        for k, v in d.items():
            self.log(k, v, **kw)

    # hooks to override
    def training_step(self, batch, batch_idx):
        raise NotImplementedError

    def validation_step(self, batch, batch_idx):
        return None

    def configure_optimizers(self):
        raise NotImplementedError

    def on_train_epoch_end(self):
        pass

    def on_validation_epoch_end(self):
        pass


class RayDDPStrategy:
    def __init__(self, find_unused_parameters: bool = False, bucket_cap_mb: int = 64, **kw):
        self.kw = dict(find_unused_parameters=find_unused_parameters, bucket_cap_mb=bucket_cap_mb,
                       gradient_as_bucket_view=True)


class RayLightningEnvironment:
    """Cluster environment plugin: ranks come from the worker group env."""


class Callback:
    def on_train_epoch_end(self, trainer: "Trainer", module: LightningModule):
        pass


class RayTrainReportCallback(Callback):
    """Report trainer.callback_metrics (+ a checkpoint of the module) once per epoch."""

    def on_train_epoch_end(self, trainer, module):
        metrics = dict(trainer.callback_metrics)
        metrics["epoch"] = trainer.current_epoch
        metrics["step"] = trainer.global_step
        with tempfile.TemporaryDirectory() as d:
            ckpt = None
            if get_context().get_world_rank() == 0:
                torch.save({"state_dict": trainer.unwrapped.state_dict(), "epoch": trainer.current_epoch,
                            "global_step": trainer.global_step}, os.path.join(d, "checkpoint.ckpt"))
                ckpt = Checkpoint.from_directory(d)
            report(metrics, checkpoint=ckpt)


def prepare_trainer(trainer: "Trainer") -> "Trainer":
    if trainer.strategy is None:
        trainer.strategy = RayDDPStrategy()
    return trainer


class Trainer:
    def __init__(self, max_epochs: int = 1, max_steps: int = -1, devices="auto", accelerator="auto", strategy=None,
                 plugins=None, callbacks: Optional[List[Callback]] = None, enable_progress_bar: bool = True,
                 limit_train_batches=None, limit_val_batches=None, precision="32", log_every_n_steps: int = 50,
                 enable_checkpointing: bool = False, num_sanity_val_steps: int = 0, default_root_dir=None,
                 hipgraph: Optional[bool] = None, **kw):
        self.max_epochs, self.max_steps = max_epochs, max_steps
        # hipGraph replay of the training step (forward, backward, SGD) after GRAPH_WARMUP
        # eager steps: None = on when it applies (one GPU worker, torch.optim.SGD without
        # dampening; MXTRAIN_LIGHTNING_GRAPH=0 turns it off)
        self.hipgraph = hipgraph
        self.graph_info: Dict[str, Any] = {}
        self.strategy = strategy
        self.callbacks = callbacks or []
        self.limit_train, self.limit_val = limit_train_batches, limit_val_batches
        self.precision = str(precision)
        self.log_every = log_every_n_steps
        self.progress = enable_progress_bar
        self.callback_metrics: Dict[str, float] = {}
        self.current_epoch = 0
        self.global_step = 0
        self.unwrapped: Optional[LightningModule] = None
        self.throughput: Dict[str, float] = {}

    def _autocast(self, dev):
        if dev.type == "cuda" and ("16" in self.precision):
            return torch.autocast("cuda", dtype=torch.bfloat16)
        import contextlib
        return contextlib.nullcontext()

    @staticmethod
    def _to(b, dev):
        from .train.torch import _to
        return _to(b, dev)

    def fit(self, model: LightningModule, train_dataloaders=None, val_dataloaders=None, datamodule=None):
        dev = get_device()
        model.to(dev)
        model.trainer = self
        self.unwrapped = model
        ddp = _StepWrapper(model)
        if dist.is_initialized() and dist.get_world_size() > 1:
            kw = self.strategy.kw if isinstance(self.strategy, RayDDPStrategy) else {}
            ddp = torch.nn.parallel.DistributedDataParallel(
                ddp, device_ids=[dev.index] if dev.type == "cuda" else None, **kw)
        opt_cfg = model.configure_optimizers()
        sched = None
        if isinstance(opt_cfg, dict):
            opt = opt_cfg["optimizer"]
            sched = opt_cfg.get("lr_scheduler")
            if isinstance(sched, dict):
                sched = sched.get("scheduler")
        elif isinstance(opt_cfg, (list, tuple)):
            opts, scheds = opt_cfg if len(opt_cfg) == 2 and isinstance(opt_cfg[0], (list, tuple)) else (opt_cfg, [])
            opt = opts[0]
            sched = scheds[0] if scheds else None
        else:
            opt = opt_cfg
        rank = get_context().get_world_rank()
        world = get_context().get_world_size()
        graph = None
        done = False
        for epoch in range(self.max_epochs):
            self.current_epoch = epoch
            sampler = getattr(train_dataloaders, "sampler", None)
            if hasattr(sampler, "set_epoch"):
                sampler.set_epoch(epoch)
            model.train()
            t0, nsamp = None, 0
            loss = out = None
            for i, batch in enumerate(train_dataloaders):
                if self.limit_train is not None and i >= self.limit_train:
                    break
                batch = self._to(batch, dev)
                captured = False
                if graph is None and self.global_step >= GRAPH_WARMUP and self._graph_ok(dev, opt, world):
                    # the last eager step's loss keeps its autograd graph (and AccumulateGrad
                    # nodes bound to the default stream) alive: a capture that reaches them
                    # waits across streams and the runtime crashes at capture end
                    loss = out = None
                    graph = self._capture(ddp, opt, batch, i, dev)
                    captured = True
                if graph is not None and graph.matches(batch):
                    loss = graph.replay(batch)
                else:
                    with self._autocast(dev):
                        out = ddp("training_step", batch, i)
                    loss = out["loss"] if isinstance(out, dict) else out
                    opt.zero_grad(set_to_none=True)
                    loss.backward()
                    opt.step()
                if sched is not None:
                    sched.step()
                self.global_step += 1
                if i == 2 or captured:   # exclude warm-up batches (and the capture) from the throughput
                    if dev.type == "cuda":
                        torch.cuda.synchronize()
                    t0, nsamp = time.time(), 0
                elif t0 is not None:
                    nsamp += _batch_len(batch) * world
                if self.progress and rank == 0 and self.global_step % self.log_every == 0:
                    print(f"Epoch {epoch} step {self.global_step}: loss {float(loss.detach()):.4f}", flush=True)
                if 0 < self.max_steps <= self.global_step:
                    done = True
                    break
            if dev.type == "cuda":
                torch.cuda.synchronize()
            if t0 is not None and nsamp:
                ips = nsamp / (time.time() - t0)
                model._logged["samples_per_sec"] = ips
                self.throughput[f"epoch{epoch}"] = ips
            model._logged["train_loss"] = float(loss.detach())
            if val_dataloaders is not None:
                model.eval()
                with torch.no_grad():
                    for i, batch in enumerate(val_dataloaders):
                        if self.limit_val is not None and i >= self.limit_val:
                            break
                        with self._autocast(dev):
                            model.validation_step(self._to(batch, dev), i)
                model.on_validation_epoch_end()
            model.on_train_epoch_end()
            self.callback_metrics = model.logged_metrics()
            if rank == 0:
                print(f"Epoch {epoch}: " + " ".join(f"{k}={v:.4f}" for k, v in self.callback_metrics.items()),
                      flush=True)
            for cb in self.callbacks:
                cb.on_train_epoch_end(self, model)
            if done:
                break
        return self


    # ------------------------------------------------------------------ hipGraph step
    def _graph_ok(self, dev, opt, world) -> bool:
        on = self.hipgraph if self.hipgraph is not None else os.environ.get("MXTRAIN_LIGHTNING_GRAPH", "1") != "0"
        if not on or dev.type != "cuda" or world != 1 or type(opt) is not torch.optim.SGD:
            return False
        return all(not g.get("dampening") and not g.get("maximize") for g in opt.param_groups)

    def _capture(self, ddp, opt, batch, idx, dev):
        """Capture one training step (forward under autocast, backward, SGD with device
        learning rates) into a hipGraph; None (eager from here on) if anything fails."""
        try:
            step = _GraphedStep(self, ddp, opt, batch, idx, dev)
            self.graph_info = {"captured_at_step": self.global_step, "nodes": step.census}
            return step
        except Exception as e:   # noqa: BLE001 -- keep training eagerly
            self.hipgraph = False
            self.graph_info = {"error": repr(e)[:300]}
            print(f"[mxtrain.lightning] hipGraph capture failed, eager steps: {e!r}"[:400], flush=True)
            return None


@torch.no_grad()
def sgd_step_device_lr(opt: torch.optim.SGD, lrs: List[torch.Tensor]) -> None:
    """torch.optim.SGD.step (momentum, Nesterov, weight decay; dampening 0) with each
    group's learning rate read from a device scalar, so the update can live inside a
    captured graph while an LR scheduler changes the rate every step.  Momentum buffers
    start at zero, which gives torch's first-step buf = d."""
    for g, lr in zip(opt.param_groups, lrs):
        ps = [p for p in g["params"] if p.grad is not None]
        if not ps:
            continue
        ps = _sgd_multi(opt, g, ps, lr)   # one HIP launch for the dense fp32 ones; the rest below
        if not ps:
            continue
        grads = [p.grad for p in ps]
        if g["weight_decay"]:
            grads = torch._foreach_add(grads, ps, alpha=g["weight_decay"])
        mom = g["momentum"]
        if mom:
            bufs = []
            for p in ps:
                st = opt.state[p]
                if st.get("momentum_buffer") is None:
                    st["momentum_buffer"] = torch.zeros_like(p)
                bufs.append(st["momentum_buffer"])
            torch._foreach_mul_(bufs, mom)
            torch._foreach_add_(bufs, grads)
            upd = torch._foreach_add(grads, bufs, alpha=mom) if g["nesterov"] else bufs
        else:
            upd = grads
        torch._foreach_add_(ps, torch._foreach_mul(upd, lr), alpha=-1.0)


def _sgd_dense(p, gr, buf) -> bool:
    return (p.is_cuda and p.dtype == torch.float32 and gr.dtype == torch.float32 and p.numel() % 4 == 0
            and p.stride() == gr.stride() and (buf is None or buf.stride() == p.stride())
            and (p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last)))
            and all(t is None or t.data_ptr() % 16 == 0 for t in (p, gr, buf)))


def _sgd_multi(opt, g, ps, lr):
    """The group's update for its dense fp32 parameters in one csrc/optim.hip mx_sgd_multi
    launch per 96 (torch's multi-tensor kernels: ~19 launches per ResNet-50 step); returns the
    parameters left for the torch path."""
    from ..ops import _lib
    if not ps[0].is_cuda or not _lib.use_hip(ps[0]) or g.get("dampening", 0):
        return ps
    mom = g["momentum"]
    jobs, rest = [], []
    for p in ps:
        buf = opt.state[p].get("momentum_buffer") if mom else None
        if mom and buf is None:
            buf = opt.state[p]["momentum_buffer"] = torch.zeros_like(p)
        (jobs if _sgd_dense(p, p.grad, buf) else rest).append((p, buf))
    from ..models.compute_weights import ctypes_int64_array
    for i in range(0, len(jobs), 96):
        chunk = jobs[i:i + 96]
        d = ctypes_int64_array([v for p, b in chunk
                                for v in (p.data_ptr(), p.grad.data_ptr(), b.data_ptr() if b is not None else 0,
                                          p.numel())])
        _lib.call("mx_sgd_multi", d, len(chunk), lr.data_ptr(), float(g["weight_decay"]), float(mom),
                  int(bool(g["nesterov"])), _lib.stream())
    return [p for p, _ in rest]


GRAPH_WARMUP = 3   # eager steps before the capture (lazy state, momentum buffers, MIOpen / GEMM choices)


class _GraphedStep:
    def __init__(self, trainer, ddp, opt, batch, idx, dev):
        from ..runtime.graphfix import census, memsets_to_kernels
        self.opt = opt
        self.lrs = [torch.tensor(float(g["lr"]), dtype=torch.float32, device=dev) for g in opt.param_groups]
        for g in opt.param_groups:   # buffers exist before capture (allocated outside the pool)
            for p in g["params"]:
                if g["momentum"] and opt.state[p].get("momentum_buffer") is None:
                    opt.state[p]["momentum_buffer"] = torch.zeros_like(p)
        self.static = _clone(batch)
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            with trainer._autocast(dev):
                out = ddp("training_step", self.static, idx)
            loss = out["loss"] if isinstance(out, dict) else out
            loss.backward()
            sgd_step_device_lr(opt, self.lrs)
        self.loss = loss
        # memset nodes (MIOpen zeroes workspaces with hipMemsetAsync) replay wrong under this
        # runtime's graph packet capture: fill-kernel nodes instead (runtime/graphfix.py)
        self.census = census(self.graph)
        self.census["memsets_as_kernels"] = memsets_to_kernels(self.graph)
        self.graph.instantiate()

    def matches(self, batch) -> bool:
        return _shapes(self.static) == _shapes(batch)

    def replay(self, batch):
        _copy_into(self.static, batch)
        for t, g in zip(self.lrs, self.opt.param_groups):
            t.fill_(float(g["lr"]))
        self.graph.replay()
        return self.loss


def _shapes(b):
    if torch.is_tensor(b):
        return (tuple(b.shape), b.dtype, b.device)
    if isinstance(b, dict):
        return tuple((k, _shapes(v)) for k, v in sorted(b.items()))
    if isinstance(b, (list, tuple)):
        return tuple(_shapes(v) for v in b)
    return None


def _clone(b):
    if torch.is_tensor(b):
        return b.clone()
    if isinstance(b, dict):
        return {k: _clone(v) for k, v in b.items()}
    if isinstance(b, (list, tuple)):
        return type(b)(_clone(v) for v in b)
    return b


def _copy_into(dst, src):
    if torch.is_tensor(dst):
        dst.copy_(src, non_blocking=True)
    elif isinstance(dst, dict):
        for k in dst:
            _copy_into(dst[k], src[k])
    elif isinstance(dst, (list, tuple)):
        for a, b in zip(dst, src):
            _copy_into(a, b)


class _StepWrapper(nn.Module):
    """DDP wraps this, so the step function runs inside DDP.forward (gradient buckets
    get registered) while the LightningModule keeps its own forward()."""

    def __init__(self, module: LightningModule):
        super().__init__()
        self.module = module

    def forward(self, name, batch, idx):
        return getattr(self.module, name)(batch, idx)


def _batch_len(b) -> int:
    if torch.is_tensor(b):
        return b.shape[0]
    if isinstance(b, dict):
        return _batch_len(next(iter(b.values())))
    if isinstance(b, (list, tuple)):
        return _batch_len(b[0])
    return 1
