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
        self._logged[name] = float(v)

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
                 enable_checkpointing: bool = False, num_sanity_val_steps: int = 0, default_root_dir=None, **kw):
        self.max_epochs, self.max_steps = max_epochs, max_steps
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
        done = False
        for epoch in range(self.max_epochs):
            self.current_epoch = epoch
            sampler = getattr(train_dataloaders, "sampler", None)
            if hasattr(sampler, "set_epoch"):
                sampler.set_epoch(epoch)
            model.train()
            t0, nsamp = None, 0
            for i, batch in enumerate(train_dataloaders):
                if self.limit_train is not None and i >= self.limit_train:
                    break
                batch = self._to(batch, dev)
                with self._autocast(dev):
                    out = ddp("training_step", batch, i)
                loss = out["loss"] if isinstance(out, dict) else out
                opt.zero_grad(set_to_none=True)
                loss.backward()
                opt.step()
                if sched is not None:
                    sched.step()
                self.global_step += 1
                if i == 2:          # exclude warm-up batches from the throughput figure
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
            self.callback_metrics = dict(model._logged)
            if rank == 0:
                print(f"Epoch {epoch}: " + " ".join(f"{k}={v:.4f}" for k, v in self.callback_metrics.items()),
                      flush=True)
            for cb in self.callbacks:
                cb.on_train_epoch_end(self, model)
            if done:
                break
        return self


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
