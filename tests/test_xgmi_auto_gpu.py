"""``MXTRAIN_XGMI=auto`` -- the N > 1 bench default -- on the box's one MI355X: several
processes share the GPU, build the group's xGMI communicator through ``get_comm`` (IPC
handle exchange, fail-fast probe, bit-exact check against the reference collective, timing
of both) and every rank must come out with the SAME per-size route table, without hanging.

RCCL cannot put two ranks on one GPU, so the reference side of the autotune is emulated
with gloo on host copies (as tests/test_xgmi_gpu.py).  The second case makes the probe fail
on ONE rank only (one-sided flag visibility on a real node): the verdict must be agreed, so
both ranks fall back to RCCL instead of one rank entering the timed loop alone."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _emu(world, rank):
    import torch.distributed as dist

    def emu(self, op, o, i):
        if op == "all_reduce":
            c = o.cpu()
            dist.all_reduce(c)
        elif op == "reduce_scatter":
            parts = [x.clone() for x in i.cpu().chunk(world)]
            for x in parts:
                dist.all_reduce(x)
            c = parts[rank]
        else:
            lst = [torch.empty_like(i.cpu()) for _ in range(world)]
            dist.all_gather(lst, i.cpu())
            c = torch.cat(lst)
        o.copy_(c)
    return emu


def _worker(rank, world, port, fail_rank, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXTRAIN_XGMI="auto",
                          MXTRAIN_XGMI_TIMEOUT_S="20", MXTRAIN_XGMI_MAX_MB="4")
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from mxtrain.parallel import xgmi
        xgmi.XGMICommunicator._rccl = _emu(world, rank)
        if rank == fail_rank:
            real = xgmi.XGMICommunicator.all_reduce_

            def broken(self, t):   # the probe's all-reduce never completes on this rank
                raise RuntimeError("injected probe failure")
            xgmi.XGMICommunicator.all_reduce_ = broken
        c = xgmi.get_comm(dist.group.WORLD, torch.device("cuda", 0))
        if rank == fail_rank:
            xgmi.XGMICommunicator.all_reduce_ = real
        assert c is not None
        t = torch.full((4096,), 1.0, device="cuda")
        routed = xgmi.route(dist.group.WORLD, t, "all_reduce", t.numel() * 4)
        if routed is not None:
            routed.all_reduce_(t)
        else:
            dist.all_reduce(t)
        torch.cuda.synchronize()
        ok = bool((t == world).all())
        q.put((rank, dict(prefer=c.prefer, autotune_ok=c.autotune_ok, routed=routed is not None, ok=ok), None))
        dist.barrier()
        xgmi.destroy_all()
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()[-2000:]))


def _spawn(world, fail_rank=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = sorted([q.get(timeout=200) for _ in ps], key=lambda t: t[0])
        for p in ps:
            p.join(timeout=30)
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
    for rank, out, err in res:
        assert err is None, (rank, err)
    return [out for _, out, _ in res]


@pytest.mark.timeout(260)
def test_xgmi_auto_selects_same_routes_on_8_ranks():
    outs = _spawn(8)
    for o in outs:
        assert o["autotune_ok"] is True, o
        assert set(o["prefer"]) == {"all_reduce", "reduce_scatter", "all_gather"}, o
        assert all(len(v) >= 1 for v in o["prefer"].values()), o
        assert o["prefer"] == outs[0]["prefer"], (o, outs[0])
        assert o["ok"], o


@pytest.mark.timeout(200)
def test_xgmi_auto_one_sided_probe_failure_falls_back_everywhere():
    outs = _spawn(2, fail_rank=1)
    for o in outs:
        assert o["autotune_ok"] is False and o["prefer"] == {}, o
        assert not o["routed"] and o["ok"], o
