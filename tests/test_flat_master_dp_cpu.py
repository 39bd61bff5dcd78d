"""Data-parallel FlatMaster (models/compute_weights.py): 2 gloo ranks, each on its own
half batch, with bucketed all-reduces started from the per-bucket backward nodes, must
give exactly Horovod's semantics -- the average of the ranks' gradients, clipped by its
global norm, then torch.optim.SGD -- i.e. one process doing the same on both halves."""
import copy
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from test_flat_master_cpu import Tiny, _opt

pytestmark = pytest.mark.dist


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    g = torch.Generator().manual_seed(3)
    return [[torch.randn(2, 3, 6, 6, generator=g) for _ in range(2)] for _ in range(3)]


def _worker(rank, port, clip, q):
    import torch.distributed as dist
    from mxtrain.models.compute_weights import FlatMaster
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    torch.manual_seed(0)
    mod = Tiny()
    opt = _opt(mod)
    # tiny buckets: several all-reduces per step, started as backward reaches them
    fm = FlatMaster(mod, opt, clip, dt=torch.float32, bucket_bytes=256)
    assert len(fm.buckets) >= 3
    order = []
    orig = fm._reduce_bucket
    fm._reduce_bucket = lambda k: (order.append(k), orig(k))
    for step, xs in enumerate(_data()):
        lr = 0.05 * (step + 1)
        opt.zero_grad(set_to_none=True)
        with fm.compute_weights():
            loss = mod(xs[rank])
        loss.backward()
        fm.step(lr)
    q.put((rank, {n: p.detach().clone().numpy() for n, p in mod.named_parameters()}, order,
           float(fm.normsq[0]), fm.dp_route))
    dist.destroy_process_group()


@pytest.mark.parametrize("clip", [0.0, 0.02])
def test_flat_master_dp_matches_averaged_single_process(clip):
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, clip, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: per-half gradients averaged (Horovod allreduce average), clip, SGD
    torch.manual_seed(0)
    ref = Tiny()
    opt = _opt(ref)
    params = [p for p in ref.parameters() if p.requires_grad]
    for step, xs in enumerate(_data()):
        for g in opt.param_groups:
            g["lr"] = 0.05 * (step + 1)
        acc = [torch.zeros_like(p) for p in params]
        for x in xs:
            opt.zero_grad(set_to_none=True)
            ref(x, folded_ref=True).backward()
            for a, p in zip(acc, params):
                a += p.grad / len(xs)
        for a, p in zip(acc, params):
            p.grad = a
        gn = torch.nn.utils.clip_grad_norm_(params, clip) if clip > 0 else None
        opt.step()
    for rank, sd, order, normsq, route in res:
        assert route == "gloo"
        # buckets reduced last-to-first, the same sequence on both ranks
        nb = max(order) + 1
        assert order == list(range(nb - 1, -1, -1)) * 3 and order == res[0][2]
        for n, p in ref.named_parameters():
            torch.testing.assert_close(torch.from_numpy(sd[n]), p.detach(), rtol=1e-5, atol=1e-6, msg=n)
        if gn is not None:
            assert abs(normsq ** 0.5 - float(gn)) < 1e-4 * float(gn)
