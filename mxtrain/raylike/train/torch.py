"""`ray.train.torch` equivalents: TorchTrainer, prepare_model, prepare_data_loader,
get_device -- one rank per MI355X, RCCL DDP."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import DataParallelTrainer, get_context


class TorchTrainer(DataParallelTrainer):
    pass


def get_device() -> torch.device:
    if torch.cuda.is_available() and os.environ.get("MXTRAIN_CPU_ONLY") != "1":
        return torch.device("cuda", get_context().get_local_rank() % torch.cuda.device_count())
    return torch.device("cpu")


def setup_process_group():
    dev = get_device()
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if get_context().get_world_size() > 1 and not dist.is_initialized():
        backend = "nccl" if dev.type == "cuda" else "gloo"
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=get_context().get_world_rank(),
                                world_size=get_context().get_world_size(), **kw)


def teardown_process_group():
    if dist.is_initialized():
        dist.destroy_process_group()


def prepare_model(model: torch.nn.Module, move_to_device: bool = True, parallel_strategy: str = "ddp",
                  parallel_strategy_kwargs=None):
    dev = get_device()
    if move_to_device:
        model = model.to(dev)
    if get_context().get_world_size() > 1 and parallel_strategy == "ddp":
        kw = dict(bucket_cap_mb=64, gradient_as_bucket_view=True)
        kw.update(parallel_strategy_kwargs or {})
        model = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[dev.index] if dev.type == "cuda" else None, **kw)
    return model


class _DeviceLoader:
    """Moves each batch to the device one batch AHEAD, on a copy stream from pinned host
    memory: batch i + 1's host-to-device copy overlaps step i's kernels instead of
    blocking the host in front of them (a pageable ``.to(non_blocking=True)`` is a
    synchronous staged copy).  The consumer's stream waits for the copy's event."""

    def __init__(self, dl, device):
        self.dl, self.device = dl, device

    def __len__(self):
        return len(self.dl)

    def __iter__(self):
        if self.device.type != "cuda":
            for b in self.dl:
                yield _to(b, self.device)
            return
        stream = torch.cuda.Stream(device=self.device)
        it = iter(self.dl)

        def fetch():
            try:
                b = next(it)
            except StopIteration:
                return None
            b = _pin(b)
            with torch.cuda.stream(stream):
                d = _to(b, self.device)
            return d, stream.record_event(), b

        nxt = fetch()
        while nxt is not None:
            d, ev, host = nxt
            torch.cuda.current_stream(self.device).wait_event(ev)
            _record(d, torch.cuda.current_stream(self.device))   # allocator: used on the compute stream
            nxt = fetch()
            yield d
            del host

    @property
    def sampler(self):
        return self.dl.sampler


def _pin(b):
    if torch.is_tensor(b):
        return b if b.is_pinned() else b.pin_memory()
    if isinstance(b, dict):
        return {k: _pin(v) for k, v in b.items()}
    if isinstance(b, (list, tuple)):
        return type(b)(_pin(v) for v in b)
    return b


def _record(b, stream):
    if torch.is_tensor(b):
        if b.is_cuda:
            b.record_stream(stream)
    elif isinstance(b, dict):
        for v in b.values():
            _record(v, stream)
    elif isinstance(b, (list, tuple)):
        for v in b:
            _record(v, stream)


def _to(b, dev):
    if torch.is_tensor(b):
        return b.to(dev, non_blocking=True)
    if isinstance(b, dict):
        return {k: _to(v, dev) for k, v in b.items()}
    if isinstance(b, (list, tuple)):
        return type(b)(_to(v, dev) for v in b)
    return b


def prepare_data_loader(dl: torch.utils.data.DataLoader, add_dist_sampler: bool = True, move_to_device: bool = True):
    ctx = get_context()
    if add_dist_sampler and ctx.get_world_size() > 1 and not isinstance(dl.sampler,
                                                                       torch.utils.data.DistributedSampler):
        shuffle = isinstance(dl.sampler, torch.utils.data.RandomSampler)
        sampler = torch.utils.data.DistributedSampler(dl.dataset, num_replicas=ctx.get_world_size(),
                                                      rank=ctx.get_world_rank(), shuffle=shuffle)
        dl = torch.utils.data.DataLoader(dl.dataset, batch_size=dl.batch_size, sampler=sampler,
                                         num_workers=dl.num_workers, collate_fn=dl.collate_fn,
                                         pin_memory=get_device().type == "cuda", drop_last=dl.drop_last)
    elif move_to_device and get_device().type == "cuda" and not dl.pin_memory:
        # pinned batches (pinned by the loader's own pin thread, off the training loop) so the
        # device copies below are truly asynchronous
        kw = dict(batch_size=dl.batch_size, sampler=dl.sampler, num_workers=dl.num_workers,
                  collate_fn=dl.collate_fn, pin_memory=True, drop_last=dl.drop_last)
        if dl.num_workers > 0:
            kw.update(persistent_workers=dl.persistent_workers, prefetch_factor=dl.prefetch_factor)
        dl = torch.utils.data.DataLoader(dl.dataset, **kw)
    return _DeviceLoader(dl, get_device()) if move_to_device else dl
