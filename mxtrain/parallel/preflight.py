"""xGMI preflight: prove the direct peer-to-peer collectives on the live node in THROWAWAY
child processes before any long-lived rank touches peer memory.

The direct 7-link kernels (csrc/comm/xgmi.hip) map every peer's HBM through IPC handles
and spin on system-scope flags.  A fault there (a bad mapping, a fence that is not visible
across devices) cannot be caught by the process that runs it, so the first contact must
not happen in the process holding a measurement or a training run.  ``run_preflight`` is
called by every rank of a job (bench.py, the launcher) BEFORE it initialises its GPU:

1. the ranks agree on a fresh rendezvous port through a TCP store (torchrun's agent store
   when present, else one hosted by rank 0 next to ``MASTER_PORT``);
2. every rank starts ONE child (``python -m mxtrain.parallel.preflight``, a new process,
   never an exec) on its GPU; the children form an N-rank RCCL job that runs the handle
   exchange, ``selftest_direct`` (registered-buffer reduce-scatter / all-gather vs the
   staged kernels), the autotune (every op x message size checked bit-exact against RCCL
   and timed) and a p2p round trip with both ring neighbours (the 1F1B channel);
3. each rank posts its child's exit code / verdict; rank 0 writes ONE verdict that every
   rank reads.  Any non-zero exit, fault, timeout or failed check on any rank ->
   ``MXTRAIN_XGMI=0`` on every rank (RCCL everywhere), with the reason.

The reference has no such step: its collectives are NCCL over NVSwitch/EFA inside the
training containers (examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-zero1.yaml:7-8,35;
charts/machine-learning/training/mpijob-horovod-tensorflow-gpu/values.yaml:64-65).

Test hooks (CPU): ``MXTRAIN_PREFLIGHT_CPU=1`` runs the children on gloo (the agreement
plumbing without a GPU); ``MXTRAIN_PREFLIGHT_FAIL_RANK=r`` makes child rank r exit 3;
``MXTRAIN_PREFLIGHT_HANG_RANK=r`` makes it sleep past its timeout.  GPU tests on a one-GPU
box: ``MXTRAIN_PREFLIGHT_EMU=1`` puts every child on device 0 with the RCCL side of the
checks emulated on gloo (RCCL refuses two ranks on one GPU).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time
from datetime import timedelta
from typing import Dict, Optional

_DONE = "MXTRAIN_XGMI_PREFLIGHT_DONE"


def _child_env(world: int, rank: int, port: int) -> dict:
    """A child rank's environment: same rank / local rank, a NEW rendezvous on ``port``
    hosted by child rank 0 (torchrun's agent-store variables dropped)."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    for k in ("GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE", "ROLE_NAME"):
        env.pop(k, None)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_RANK=os.environ.get("LOCAL_RANK", str(rank)),
               LOCAL_WORLD_SIZE=os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    return env


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _store(world: int, rank: int, timeout_s: float):
    """A TCP store every rank of the job can reach without a process group: torchrun's
    agent store if the job runs under torchrun, else one hosted by rank 0."""
    import torch.distributed as dist
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    tmo = timedelta(seconds=timeout_s)
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true":
        base = dist.TCPStore(host, port, world, False, timeout=tmo, wait_for_workers=False)
    else:   # (the job's own rendezvous comes later on MASTER_PORT: stay off it)
        base = dist.TCPStore(host, port + 97, world, rank == 0, timeout=tmo, wait_for_workers=False)
    run = os.environ.get("TORCHELASTIC_RUN_ID", "") + os.environ.get("TORCHELASTIC_RESTART_COUNT", "")
    return dist.PrefixStore(f"mx_xgmi_preflight/{run}/", base), base


def should_run(world: int, xgmi_mode: str) -> bool:
    if world <= 1 or xgmi_mode == "0" or os.environ.get(_DONE) == "1":
        return False
    if os.environ.get("MXTRAIN_XGMI_PREFLIGHT", "1") == "0":
        return False
    if os.environ.get("MXTRAIN_PREFLIGHT_CPU") == "1":
        return True
    import torch
    return torch.cuda.device_count() > 0   # (counting devices does not initialise the GPU)


def run_preflight(world: int, rank: int, timeout_s: float = 150.0) -> Dict:
    """Collective over the job's ranks (call on every rank, before any GPU work).  Returns
    ``{"ok", "reason", "s", ...}`` -- the same verdict on every rank -- and sets
    ``MXTRAIN_XGMI=0`` in this process's environment when the verdict is negative."""
    t0 = time.time()
    verdict: Dict = {"ok": False, "reason": "", "s": 0.0}
    store = base = None
    try:
        store, base = _store(world, rank, timeout_s + 60)
        if rank == 0:
            store.set("port", str(_free_port()))
        port = int(store.get("port").decode())
        out = tempfile.mktemp(prefix=f"mx_xgmi_pre_r{rank}_", suffix=".json")
        cmd = [sys.executable, "-m", "mxtrain.parallel.preflight", "--out", out]
        env = _child_env(world, rank, port)
        env["PYTHONPATH"] = os.pathsep.join(
            [os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))]
            + ([env["PYTHONPATH"]] if env.get("PYTHONPATH") else []))
        mine: Dict = {"rank": rank}
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env,
                             start_new_session=True)
        # wait for the child; a peer rank that already reported a failure ends the wait
        # (this rank's child would otherwise sit in a rendezvous / collective until timeout)
        deadline = time.time() + timeout_s
        peers = [r for r in range(world) if r != rank]
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.25)
            for r in list(peers):
                if store.check([f"res/{r}"]):
                    peers.remove(r)
                    pr = json.loads(store.get(f"res/{r}").decode())
                    if pr.get("rc") != 0 or not pr.get("ok"):
                        mine["rc"] = "aborted"
                        mine["why"] = f"peer rank {r} failed"
                        deadline = 0.0
                        break
        if p.poll() is None:
            import signal
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass
            mine.setdefault("rc", 124)
        else:
            mine["rc"] = p.returncode
        text = p.communicate()[0]
        try:
            with open(out) as f:
                mine.update(json.load(f))
            os.remove(out)
        except (OSError, ValueError):
            pass
        if mine["rc"] != 0:
            mine["tail"] = (text or "")[-300:]
        store.set(f"res/{rank}", json.dumps(mine))
        if rank == 0:
            res = []
            try:
                store.wait([f"res/{r}" for r in range(world)], timedelta(seconds=60))
                res = [json.loads(store.get(f"res/{r}").decode()) for r in range(world)]
            except Exception as e:   # noqa: BLE001 -- a rank that never posted: RCCL
                verdict["reason"] = f"preflight results missing: {e!r}"[:300]
            if res:
                bad = [r for r in res if r.get("rc") != 0 or not r.get("ok")]
                # the root cause first: a rank that failed by itself, not one that timed out
                # waiting for it or was stopped because of it
                bad.sort(key=lambda r: {"aborted": 2, 124: 1}.get(r.get("rc"), 0))
                if bad:
                    b = bad[0]
                    why = {124: "timeout", "aborted": "aborted"}.get(b.get("rc"), f"rc={b.get('rc')}") \
                        if b.get("rc") != 0 else b.get("why", "check failed")
                    verdict["reason"] = f"rank {b['rank']}: {why}" + (f" ({b['tail'][-160:]})" if b.get("tail") else "")
                else:
                    verdict["ok"] = True
                    verdict["reason"] = "xgmi selftest + autotune + p2p ok"
                    for k in ("prefer", "p2p_ok", "direct_ok"):
                        if k in res[0]:
                            verdict[k] = res[0][k]
            store.set("verdict", json.dumps(verdict))
        else:
            verdict = json.loads(store.get("verdict").decode())
    except Exception as e:   # noqa: BLE001 -- the store itself failed: RCCL, reason recorded
        verdict = {"ok": False, "reason": f"preflight error: {e!r}"[:300]}
    verdict["s"] = round(time.time() - t0, 1)
    if not verdict["ok"]:
        os.environ["MXTRAIN_XGMI"] = "0"
    os.environ[_DONE] = "1"   # children of this rank (bench phases) inherit the verdict
    del store, base
    return verdict


# ----------------------------------------------------------------------------- child side
def _emulated_rccl(world: int, rank: int):
    import torch
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


def _child(out: str) -> int:
    import torch
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    res: Dict = {"ok": False}
    if os.environ.get("MXTRAIN_PREFLIGHT_FAIL_RANK") == str(rank):
        return 3
    if os.environ.get("MXTRAIN_PREFLIGHT_HANG_RANK") == str(rank):
        time.sleep(3600)
    cpu = os.environ.get("MXTRAIN_PREFLIGHT_CPU") == "1"
    if cpu:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        t = torch.full((16,), float(rank + 1))
        dist.all_reduce(t)
        res["ok"] = bool((t == world * (world + 1) / 2).all())
        res["why"] = "" if res["ok"] else "gloo all-reduce mismatch"
    else:
        from . import xgmi as X
        emu = os.environ.get("MXTRAIN_PREFLIGHT_EMU") == "1"
        local = 0 if emu else int(os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if emu:
            # (tests on a one-GPU box: the ranks share the GPU, which RCCL refuses -- the
            # reference side of the checks runs on gloo over host copies)
            dist.init_process_group("gloo", rank=rank, world_size=world)
            X.XGMICommunicator._rccl = _emulated_rccl(world, rank)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        g = dist.group.WORLD
        # RCCL itself first: a failure here is not the xGMI kernels' and is reported as such
        t = torch.full((1024,), float(rank + 1), device=dev)
        dist.all_reduce(t)
        if not bool((t == world * (world + 1) / 2).all().item()):
            res["why"] = "rccl all-reduce mismatch"
        else:
            c = X.XGMICommunicator(g, dev, max_bytes=64 << 20, timeout_s=10.0)
            res["direct_ok"] = bool(c.selftest_direct())
            c.autotune(sizes=(1 << 16, 1 << 20, 8 << 20, 64 << 20), iters=4)
            res["prefer"] = {op: [[nb, bool(w)] for nb, w in v] for op, v in (c.prefer or {}).items()}
            peers = sorted({(rank - 1) % world, (rank + 1) % world} - {rank})
            p2p = X.XGMIP2P(g, dev, peers, 1 << 20, timeout_s=10.0)
            res["p2p_ok"] = bool(p2p.selftest())
            p2p.close()
            c.close()
            res["ok"] = bool(res["direct_ok"] and c.autotune_ok and res["p2p_ok"])
            if not res["ok"]:
                res["why"] = (f"direct_ok={res['direct_ok']} autotune_ok={c.autotune_ok} "
                              f"p2p_ok={res['p2p_ok']}")
        torch.cuda.synchronize(dev)
    dist.barrier()
    dist.destroy_process_group()
    with open(out, "w") as f:
        json.dump(res, f)
    return 0


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    sys.exit(_child(ap.parse_args().out))
